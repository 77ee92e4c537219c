"""Diagnostic: svc_run counters (k_decide_dt<true>, -DLKF_SVC_DIAG=1 build).

    make -C livekit-server_amd/csrc svcdiag && python3 scripts/svc_diag.py [rooms] [batches]

Runs configs[4] batches (SVC with dependency descriptors) through
liblkfwd_svcdiag.so and prints: svc_run calls, runs, lanes decided in runs,
uniform-precondition failures, and the condition that stopped each run at an
in-window lane (the packet then takes the full step).
"""
import ctypes as C
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WHY = {1: "forward before start / sequencer init", 2: "VP9 switch point", 3: "frame order", 4: "ndti",
       5: "DTI differs within frame", 6: "attached/structure/active update/keyframe num/chains",
       7: "DD switch / first frame number", 8: "chain", 9: "frame reference dropped", 10: "marshal",
       11: "munger (reorder/dup/padding/ssrc)", 12: "drop with open range moved", 13: "sequencer",
       14: "awaited frame (chain expectation)"}


def main():
    rooms = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    svc_dd = int(os.environ.get("SVC_DD", "1"))
    pkg = importlib.import_module("livekit-server_amd")
    wl = importlib.import_module("livekit-server_amd.workload")
    tr = wl.Trace(5, duration_s=float(nb), batch_s=1.0, rooms=rooms, svc_dd=svc_dd)
    lib = os.path.join(ROOT, "livekit-server_amd", "lib", os.environ.get("DIAG_LIB", "liblkfwd_svcdiag.so"))
    eng = pkg.Engine.for_trace(tr, lib_path=lib)
    fn = eng.lib.lkf_debug_counters
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    wl.load_topology(eng.api, eng.h, tr)
    buf = (C.c_uint64 * 32)()
    for b in range(nb):
        wl.queue_events(eng.api, eng.h, tr, b)
        pk, n, ar, alen = tr.batch(b)
        eng.submit(pk, n, ar, alen, tr.batch_dd(b)[0] if tr.has_dd() else None)
        eng.run()
        eng.sync()
        assert fn(eng.h, buf, 1) == 0
        v = list(buf)
        print("batch %d: svc_run %d, uniform fail %d, runs %d, lanes in runs %d, window ends %d" % (
            b, v[0], v[4], v[1], v[2], v[13]))
        stops = {k: v[16 + k] for k in range(16) if v[16 + k]}
        tot = sum(stops.values())
        for k, c in sorted(stops.items(), key=lambda t: -t[1]):
            print("   stop %-55s %8d (%.1f%%)" % (WHY.get(k, "none (%d)" % k), c, 100.0 * c / max(1, tot)))
    eng.close()


if __name__ == "__main__":
    main()
