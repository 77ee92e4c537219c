"""Diagnostic: where the SVC runs of k_decide_dt<true> stop on configs[4]
(needs the LKF_SVC_STATS build: make -C livekit-server_amd/csrc ab
ABNAME=svcst ABFLAGS=-DLKF_SVC_STATS=1, run with LKF_LIB=liblkfwd_svcst.so).
Prints the counters per batch (forwarding path, ExtPackets)."""
import ctypes as C
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
pkg = importlib.import_module("livekit-server_amd")
workload = importlib.import_module("livekit-server_amd.workload")

WHY = {1: "start/seq", 2: "vp9 switch", 3: "frame order", 4: "ndti", 5: "frame head", 6: "struct/active/kfn/nchain",
       7: "switch/fn init", 8: "chain", 9: "fdiff dropped/long", 10: "marshal", 11: "reorder/pad", 12: "excl",
       13: "osn/ots", 14: "expect", 15: "window end"}


def main():
    rooms = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    svc_dd = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 5  # (2 with batch 0.01: the 10-ms tick)
    batch_s = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
    dur = float(sys.argv[5]) if len(sys.argv) > 5 else 3.0
    kw = dict(svc_dd=svc_dd) if cfg == 5 else {}
    tr = workload.Trace(cfg, duration_s=dur, batch_s=batch_s, rooms=rooms, **kw)
    eng = pkg.Engine.for_trace(tr)
    workload.load_topology(eng.api, eng.h, tr)
    fn = eng.lib.lkf_debug_svc_stats
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    fn.restype = C.c_int
    out = (C.c_uint64 * 48)()
    fn(eng.h, out, 1)
    for b in range(tr.nbatches):
        workload.queue_events(eng.api, eng.h, tr, b)
        pk, n, ar, alen = tr.batch(b)
        dd = tr.batch_dd(b)[0] if tr.has_dd() else None
        t0 = time.time()
        eng.submit(pk, n, ar, alen, dd)
        eng.run()
        eng.sync()
        dt = time.time() - t0
        assert fn(eng.h, out, 1) == 0
        v = list(out)
        print(f"batch {b}: n={n} {dt*1e3:.1f} ms  runs={v[0]} run_pkts={v[1]} full_steps={v[2]} refused={v[3]}",
              flush=True)
        print("   stops: " + ", ".join(f"{WHY.get(i, i)}={v[16 + i]}" for i in range(16) if v[16 + i]), flush=True)
        if v[9]:  # per SVC DownTrack, s_memtime (shader clock) cycles, thousands
            print("   per DT (kcycles): prologue %.1f runs %.1f full steps %.1f rest of loop %.1f epilogue %.1f (n=%d)" %
                  tuple([v[k] / v[9] / 1000.0 for k in (4, 5, 6, 7, 8)] + [v[9]]), flush=True)
            print("   in DD runs (kcycles per DT): decision %.1f marshal %.1f munger/seq decision %.1f" %
                  tuple(v[k] / v[9] / 1000.0 for k in (10, 11, 12)), flush=True)
            if v[14]:
                print("   dd_select: %d calls, %.1f kcycles per call" % (v[14], v[13] / v[14] / 1000.0), flush=True)
                if v[43]:
                    print("      reaching the marshal (%d): chains %.1f, selection %.1f, marshal %.1f kcycles each" %
                          (v[43], v[40] / v[43] / 1e3, v[41] / v[43] / 1e3, v[42] / v[43] / 1e3), flush=True)
                if v[45]:
                    print("      of which with a structure attached: %d, marshal %.1f kcycles each" %
                          (v[45], v[44] / v[45] / 1e3), flush=True)
        if v[36]:  # the plain DownTracks (k_decide_dt<false>)
            print("   plain DTs (kcycles per DT): hot load %.2f rest of prologue %.2f body %.2f epilogue %.2f "
                  "(n=%d, %.2f pkts/DT)" % tuple([v[k] / v[36] / 1000.0 for k in (32, 33, 34, 35)] +
                                                 [v[36], v[37] / v[36]]), flush=True)
            print("      body: to the first chunk's packets %.2f, RTPStatsSender folds %.2f" %
                  (v[38] / v[36] / 1000.0, v[39] / v[36] / 1000.0), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
