import importlib
import os
import subprocess
import sys

import pytest

# torch before any engine library: the process then has one HIP runtime
# (liblkfwd.so binds to the libamdhip64 torch loaded, as in bench.py, which
# imports torch first).  A test process that loaded liblkfwd first left torch
# on a second runtime that reported no GPU to the tests that use torch.
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def _make(dirpath):
    subprocess.run(["make", "-s", "-j8", "-C", dirpath], check=True)


@pytest.fixture(scope="session")
def pkg():
    """The product package (livekit-server_amd), with its C libraries built."""
    if not os.path.exists(os.path.join(ROOT, "livekit-server_amd", "lib", "liblkfsynth.so")):
        _make(os.path.join(ROOT, "livekit-server_amd", "csrc"))
    return importlib.import_module("livekit-server_amd")


@pytest.fixture(scope="session")
def workload(pkg):
    return importlib.import_module("livekit-server_amd.workload")


@pytest.fixture(scope="session")
def abi(pkg):
    return importlib.import_module("livekit-server_amd.abi")


@pytest.fixture(scope="session")
def oracle():
    from tests import oracle_lib
    return oracle_lib.load()


@pytest.fixture(autouse=True)
def _bounds_checked(request):
    """With LKF_LIB=liblkfwd_checked.so every GPU test ends with the checked
    kernels' violation record read and required empty (site, index and
    capacity of the first out-of-bounds index otherwise)."""
    checked = "checked" in os.environ.get("LKF_LIB", "") and request.node.get_closest_marker("gpu")
    if checked:
        p = importlib.import_module("livekit-server_amd")
        p.debug_check(reset=True)
    yield
    if checked:
        rec = p.debug_check(reset=True)
        assert rec is not None, "LKF_LIB is not a checked build"
        assert rec[0] == 0, "out-of-bounds index: %d violations, first at site %d index %d capacity %d" % rec
