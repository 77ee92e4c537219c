"""Debug: test_pause_and_next_higher_match_oracle[cfg1] with mismatch details
(engine vs oracle output records of the first mismatching batch)."""
import ctypes as C
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.oracle_lib import load as load_oracle  # noqa: E402
from tests.test_alloc_gpu import stream_allocator_steps, run_step, video_mask  # noqa: E402


def main():
    pkg = importlib.import_module("livekit-server_amd")
    wl = importlib.import_module("livekit-server_amd.workload")
    abi = pkg.abi
    o = load_oracle()
    cfg = dict(config=5, rooms=int(os.environ.get("ROOMS", "6")), svc_dd=int(os.environ.get("SVC_DD", "1")))
    tr = wl.Trace(cfg.pop("config"), duration_s=6.0, batch_s=1.0, **cfg)
    lib = os.environ.get("LKF_LIB")
    eng = pkg.Engine.for_trace(tr, lib_path=os.path.join(ROOT, "livekit-server_amd", "lib", lib) if lib else None)
    oh = o.create(500)
    wl.load_topology(eng.api, eng.h, tr)
    wl.load_topology(o.api, oh, tr)
    for b in range(tr.nbatches):
        for step in stream_allocator_steps(abi, tr.ndts, b, video_mask(abi, tr)):
            run_step(eng.api, eng.h, abi, step)
            run_step(o.api, oh, abi, step)
        # states before the batch
        pre = {}
        for dt in range(tr.ndts):
            gs = abi.lkf_fwd_state()
            eng.api["get_state"](eng.h, dt, C.byref(gs))
            pre[dt] = gs
        wt = eng.lib.lkf_debug_wtime
        wt.restype = C.c_int
        wt.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32]
        logbuf = (C.c_uint32 * (4 * 4096))()
        have_log = os.environ.get("LKF_LIB", "").startswith("liblkfwd_svcwatch") and wt(eng.h, logbuf, 4096) == 0
        log0 = logbuf[0] if have_log else 0
        wl.queue_events(eng.api, eng.h, tr, b)
        wl.queue_events(o.api, oh, tr, b)
        pk, n, ar, alen = tr.batch(b)
        dd = tr.batch_dd(b)[0] if tr.has_dd() else None
        eng.submit(pk, n, ar, alen, dd)
        eng.run()
        eng.sync()
        o.run(oh, pk, n, ar, alen, dd)
        # DD selector states after the batch
        ge = eng.lib.lkf_debug_dd_state
        ge.restype = C.c_int
        ge.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64)]
        oe = o.lib.orc_debug_dd_state
        oe.restype = C.c_int
        oe.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64)]
        nd = 0
        for dt in range(tr.ndts):
            g16 = (C.c_uint64 * 16)()
            o16 = (C.c_uint64 * 16)()
            if ge(eng.h, dt, g16) != 0:
                break
            oe(oh, dt, o16)
            if o16[0] == 0 and g16[0] == 0:
                continue
            gl, ol = list(g16), list(o16)
            gl[13], ol[13] = int(gl[13] != 0), int(ol[13] != 0)  # (expectation sets vs lists: presence only)
            if dt == int(os.environ.get("WATCH_DT", "160")):
                print("  batch %d watch dt %d gpu: %s" % (b, dt, " ".join("%x" % v for v in gl)))
                print("  batch %d watch dt %d orc: %s" % (b, dt, " ".join("%x" % v for v in ol)))
            if gl != ol:
                nd += 1
                if nd <= 3:
                    names = ["init", "base", "last"] + ["m%d" % i for i in range(8)] + ["broken", "active", "exp", "fnLast", "cur"]
                    diffs = ["%s g=%#x o=%#x" % (names[i], gl[i], ol[i]) for i in range(16) if gl[i] != ol[i]]
                    print("  batch %d dt %d DD state differs: %s" % (b, dt, "; ".join(diffs)))
        if nd:
            print("  batch %d: %d DTs with different DD state" % (b, nd))
        if have_log and b == int(os.environ.get("BATCH", "3")):
            wt(eng.h, logbuf, 4096)
            lo, hi = int(os.environ.get("LOG_LO", "3980")), int(os.environ.get("LOG_HI", "4045"))
            for i in range(log0, min(logbuf[0], 4095)):
                k, a1, a2, a3 = logbuf[4 + 4 * i: 8 + 4 * i]
                if lo <= a1 <= hi:
                    print("   log %s pkt %d %s" % ({1: "run ", 2: "unif", 3: "full"}.get(k, k), a1,
                          ("x %d why %d" % (a2, a3)) if k == 1 else ("cLast %d broken/active %#x" % (a2, a3)) if k == 3 else ""))
        grec, gar = eng.drain()
        orec, oar = pkg.drain_arrays(o.api, oh)
        bad = np.zeros(len(grec), bool) if len(grec) == len(orec) else None
        if bad is None:
            print("batch %d: record counts differ %d vs %d" % (b, len(grec), len(orec)))
            return
        for f in abi.OUT_DTYPE.names:
            bad |= grec[f] != orec[f]
        print("batch %d: %d records, %d differ" % (b, len(grec), bad.sum()))
        if bad.any():
            pkts = np.ctypeslib.as_array(C.cast(pk, C.POINTER(C.c_uint8)), shape=(n * 64,)).reshape(n, 64)
            idx = np.nonzero(bad)[0][:12]
            for i in idx:
                g, r = grec[i], orec[i]
                dt = int(g["dt"])
                print(" rec %d dt %d pkt %d  gpu flags %d sn %d | oracle flags %d sn %d | pkt flags %#x layer %d" % (
                    i, dt, g["pkt"], g["flags"], g["ext_sn"], r["flags"], r["ext_sn"], pkts[g["pkt"], 44],
                    np.int8(pkts[g["pkt"], 53])))
            # the DT's track packets before the first mismatch
            i0 = idx[0]
            dt0 = int(grec[i0]["dt"])
            trk = tr.downtracks[dt0].track
            ddp = tr.batch_dd(b)[0]
            dda = np.ctypeslib.as_array(C.cast(ddp, C.POINTER(C.c_uint8)), shape=(n * 32,)).reshape(n, 32)
            tracks = pkts[:, 28:32].copy().view("<u4").ravel()
            gset = set(int(v) for v in grec["pkt"][grec["dt"] == dt0])
            oset = set(int(v) for v in orec["pkt"][orec["dt"] == dt0])
            gfl = {int(r["pkt"]): int(r["flags"]) for r in grec[grec["dt"] == dt0]}
            ofl = {int(r["pkt"]): int(r["flags"]) for r in orec[orec["dt"] == dt0]}
            p0 = int(grec[i0]["pkt"])
            sel = [k for k in range(n) if tracks[k] == trk and p0 - 400 <= k <= p0 + 10]
            for k in sel[-60:]:
                esn = int(pkts[k, 0:8].copy().view("<u8")[0])
                efn = int(dda[k, 0:8].copy().view("<u8")[0])
                kfn = int(dda[k, 8:16].copy().view("<u8")[0])
                print("   pkt %5d esn %d sp %d tp %d hdr1 %#x pflags %#x | efn %d kfn %d ddfl %#x | gpu %s%s orc %s%s" % (
                    k, esn, np.int8(pkts[k, 42]), np.int8(pkts[k, 43]), pkts[k, 41], pkts[k, 44], efn, kfn, dda[k, 19],
                    "F" if k in gset else "-", gfl.get(k, ""), "F" if k in oset else "-", ofl.get(k, "")))
            evp, ne = wl.events_ptr(tr, b)
            for k in range(ne):
                ev = evp[k]
                if ev.dt == dt0:
                    print("   event dt %d op %d a %s at %d" % (ev.dt, ev.op, list(ev.a), ev.at_pkt))
            # the DT's records around the first mismatch
            i0 = idx[0]
            dt = int(grec[i0]["dt"])
            sel = np.nonzero(grec["dt"] == dt)[0]
            j = np.searchsorted(sel, i0)
            for k in sel[max(0, j - 4): j + 4]:
                print("   dt rec %d pkt %d gpu f=%d o f=%d sn %d" % (k, grec[k]["pkt"], grec[k]["flags"], orec[k]["flags"],
                                                                     grec[k]["ext_sn"]))
            return
    print("no mismatch")


if __name__ == "__main__":
    main()
