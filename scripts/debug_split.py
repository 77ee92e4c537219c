"""Debug: replay the cfg1 alloc scenario, splitting batch B at packet S
(engine and oracle alike), and compare the watched DownTrack's DD selector
state after the prefix.  SPLITS=a,b,c tries several split points (fresh
engines each)."""
import ctypes as C
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.oracle_lib import load as load_oracle  # noqa: E402
from tests.test_alloc_gpu import stream_allocator_steps, run_step, video_mask  # noqa: E402


def dd_state(fn, h, dt):
    v = (C.c_uint64 * 16)()
    fn(h, dt, v)
    v = list(v)
    v[13] = int(v[13] != 0)
    return v


def run(split, B, watch):
    pkg = importlib.import_module("livekit-server_amd")
    wl = importlib.import_module("livekit-server_amd.workload")
    abi = pkg.abi
    o = load_oracle()
    tr = wl.Trace(5, duration_s=6.0, batch_s=1.0, rooms=6, svc_dd=1)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    ge = eng.lib.lkf_debug_dd_state
    ge.restype = C.c_int
    ge.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64)]
    oe = o.lib.orc_debug_dd_state
    oe.restype = C.c_int
    oe.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64)]
    wl.load_topology(eng.api, eng.h, tr)
    wl.load_topology(o.api, oh, tr)
    for b in range(B + 1):
        for step in stream_allocator_steps(abi, tr.ndts, b, video_mask(abi, tr)):
            run_step(eng.api, eng.h, abi, step)
            run_step(o.api, oh, abi, step)
        pk, n, ar, alen = tr.batch(b)
        dd = tr.batch_dd(b)[0]
        if b < B:
            wl.queue_events(eng.api, eng.h, tr, b)
            wl.queue_events(o.api, oh, tr, b)
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen, dd)
            eng.drain()
            pkg.drain_arrays(o.api, oh)
            continue
        evp, ne = wl.events_ptr(tr, b)
        evs = [evp[k] for k in range(ne)]
        parts = [(0, split), (split, n)]
        for (s0, s1) in parts:
            sel = [e for e in evs if s0 <= e.at_pkt < s1 or (s1 == n and e.at_pkt >= n)]
            if sel:
                arr = (abi.lkfs_event * len(sel))()
                for i, e in enumerate(sel):
                    C.memmove(C.byref(arr[i]), C.byref(e), C.sizeof(e))
                    arr[i].at_pkt = e.at_pkt - s0
                for api, h in ((eng.api, eng.h), (o.api, oh)):
                    assert api["ctl_batch"](h, C.cast(arr, C.c_void_p), len(sel)) == 0
            cnt = s1 - s0
            p2 = C.c_void_p(C.cast(pk, C.c_void_p).value + 64 * s0)
            d2 = C.c_void_p(C.cast(dd, C.c_void_p).value + 32 * s0)
            eng.submit(p2, cnt, ar, alen, d2)
            eng.run()
            eng.sync()
            o.run(oh, p2, cnt, ar, alen, d2)
            grec, _ = eng.drain()
            orec, _ = pkg.drain_arrays(o.api, oh)
            same = len(grec) == len(orec) and all(np.array_equal(grec[f], orec[f]) for f in abi.OUT_DTYPE.names)
            g, r = dd_state(ge, eng.h, watch), dd_state(oe, oh, watch)
            print("split %d part [%d,%d): records %s, dd state of dt %d %s" % (
                split, s0, s1, "equal" if same else "DIFFER", watch, "equal" if g == r else "DIFFER"))
            if g != r:
                names = ["init", "base", "last"] + ["m%d" % i for i in range(8)] + ["broken", "active", "exp", "fnLast", "cur"]
                print("    " + "; ".join("%s g=%#x o=%#x" % (names[i], g[i], r[i]) for i in range(16) if g[i] != r[i]))
    eng.close()
    o.destroy(oh)


if __name__ == "__main__":
    watch = int(os.environ.get("WATCH_DT", "160"))
    B = int(os.environ.get("BATCH", "3"))
    for s in [int(v) for v in os.environ.get("SPLITS", "4034").split(",")]:
        run(s, B, watch)
