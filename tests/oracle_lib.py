"""Test-side loader of the CPU oracle (oracle/, test infrastructure only).

Builds oracle/_build with its Makefile if needed and binds the orc_* entry
points, which mirror the engine's lkf_* C-ABI so parity tests drive both
identically.
"""
import ctypes as C
import importlib
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "liblkf_oracle.so")
KAT = os.path.join(ORACLE_DIR, "_build", "kat")

_cache = {}


def build():
    subprocess.run(["make", "-s", "-j8", "-C", ORACLE_DIR], check=True)


class Oracle:
    def __init__(self, lib, abi):
        self.lib = lib
        self.abi = abi
        self.api = abi.bind_engine_api(lib, "orc_")
        lib.orc_create.restype = C.c_void_p
        lib.orc_create.argtypes = [C.c_uint32]
        lib.orc_destroy.restype = None
        lib.orc_destroy.argtypes = [C.c_void_p]
        lib.orc_run.restype = C.c_int
        lib.orc_run.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]
        lib.orc_run_timed.restype = C.c_double
        lib.orc_run_timed.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_int]

    def create(self, seq_size=500):
        return self.lib.orc_create(seq_size)

    def destroy(self, h):
        self.lib.orc_destroy(h)

    def run(self, h, pkts, n, arena, alen, dd=None):
        """orc_submit_dd (when the batch has a lkf_pkt_dd side array) + orc_run."""
        if dd is not None:
            assert self.api["submit_dd"](h, C.cast(dd, C.c_void_p), n) == 0
        rc = self.lib.orc_run(h, C.cast(pkts, C.c_void_p), n, C.cast(arena, C.c_void_p), alen)
        assert rc == 0, rc


def load():
    if "o" in _cache:
        return _cache["o"]
    if not os.path.exists(LIB) or not os.path.exists(KAT):
        build()
    abi = importlib.import_module("livekit-server_amd.abi")
    o = Oracle(C.CDLL(LIB), abi)
    _cache["o"] = o
    return o
