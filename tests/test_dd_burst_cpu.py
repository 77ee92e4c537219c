"""The DD burst workload (synth svc_dd = 3) reaches the
regime the engine's old 16-frame cap refused: chain 0 follows every frame,
every other frame number is lost for 2 s of every 3, so each arriving frame
makes its chain wait on the lost one before it (FrameChain.expectFrames,
framechain.go:30,67-110).  The CPU oracle (an unbounded list, as the
reference) is driven over the trace and must hold more than 16 distinct
expected frames on some DownTrack, while staying inside the decision cache's
256-frame window (selectordecisioncache.go:60-110).
"""
import ctypes as C

from tests.oracle_lib import load as load_oracle


def test_burst_trace_exceeds_old_expectation_cap(workload):
    o = load_oracle()
    tr = workload.Trace(5, duration_s=4.0, batch_s=0.5, rooms=4, svc_dd=3, seed=91)
    h = o.create(500)
    f = o.lib.orc_debug_dd_state
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64)]
    out = (C.c_uint64 * 16)()
    try:
        workload.load_topology(o.api, h, tr)
        peak = 0
        for b in range(tr.nbatches):
            workload.queue_events(o.api, h, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(h, pk, n, ar, alen, tr.batch_dd(b)[0])
            for d in range(tr.ndts):
                assert f(h, d, out) == 0
                peak = max(peak, int(out[13]))
        assert peak > 16, peak
        assert peak < 256, peak
    finally:
        o.destroy(h)
        tr.close()
