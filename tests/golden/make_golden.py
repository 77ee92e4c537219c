"""Regenerates tests/golden/*.json from the CPU oracle (test infrastructure).

    python tests/golden/make_golden.py

The oracle is pinned to the reference's own unit tests by oracle/kat.cpp; the
fixtures written here capture its end-to-end outputs on small synthetic traces
so the engine can be checked against committed data.  Regenerate only when the
synthetic generator or the oracle changes on purpose, and commit the diff.
"""
import ctypes as C
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tests import golden_lib  # noqa: E402
from tests.oracle_lib import load as load_oracle  # noqa: E402


def main_control(o, abi, wl, pkg):
    for name, kw in golden_lib.CONTROL_CASES:
        tr = wl.Trace(**kw)
        h = o.create(500)
        fx = golden_lib.run_control_case(o.api, h, tr, wl, lambda: pkg.drain_arrays(o.api, h),
                                         lambda pk, n, ar, alen: o.run(h, pk, n, ar, alen), abi, name)
        fx["case"] = name
        fx["trace"] = kw
        with open(golden_lib.path(name), "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
        o.destroy(h)
        tr.close()
        print("wrote", golden_lib.path(name), "steps", len(fx["steps"]))


def main():
    abi = importlib.import_module("livekit-server_amd.abi")
    wl = importlib.import_module("livekit-server_amd.workload")
    pkg = importlib.import_module("livekit-server_amd")
    o = load_oracle()
    os.makedirs(golden_lib.GOLDEN_DIR, exist_ok=True)
    main_control(o, abi, wl, pkg)
    if "--control-only" in sys.argv:
        return
    for name, kw in golden_lib.CASES:
        tr = wl.Trace(**kw)
        h = o.create(500)

        def stats():
            st = abi.lkf_stats()
            o.api["get_stats"](h, C.byref(st))
            return st.as_dict()

        fx = golden_lib.run_case(o.api, h, tr, wl, stats, lambda: pkg.drain_arrays(o.api, h),
                                 lambda pk, n, ar, alen, dd: o.run(h, pk, n, ar, alen, dd), abi)
        fx["case"] = name
        fx["trace"] = kw
        with open(golden_lib.path(name), "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
        o.destroy(h)
        tr.close()
        print("wrote", golden_lib.path(name), "batches", len(fx["batches"]),
              "forwarded", sum(b["stats"]["forwarded"] for b in fx["batches"]))


if __name__ == "__main__":
    main()
