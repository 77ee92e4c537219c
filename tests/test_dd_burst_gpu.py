"""DD chains waiting on more than 16 frames: the engine
keeps FrameChain.expectFrames as a 512-bit ring over the decision cache's
window (dd_device.h) instead of a 16-entry list that raised LKF_EINVAL.  On
the burst workload (synth svc_dd = 3: chains waiting on up to ~47 frames, see
tests/test_dd_burst_cpu.py) the engine must forward exactly as the CPU oracle
(every record and wire byte per batch, every Forwarder state, no error), and
after every batch each DownTrack's set of expected frames must have the
oracle's size.
"""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch_s,rooms,seed", [(0.5, 4, 91), (1.0, 12, 92), (0.1, 3, 93)])
def test_dd_burst_expectations_match_oracle(pkg, workload, abi, batch_s, rooms, seed):
    tr = workload.Trace(5, duration_s=4.0, batch_s=batch_s, rooms=rooms, svc_dd=3, seed=seed)
    o = load_oracle()
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    fe = eng.lib.lkf_debug_dd_state
    fe.restype, fe.argtypes = C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64)]
    fo = o.lib.orc_debug_dd_state
    fo.restype, fo.argtypes = C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64)]
    ge, go = (C.c_uint64 * 16)(), (C.c_uint64 * 16)()
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        dd_dts = [d for d in range(tr.ndts) if tr.tracks[tr.downtracks[d].track].has_dd]
        assert dd_dts
        peak = 0
        for b in range(tr.nbatches):
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            dd = tr.batch_dd(b)[0]
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            eng.sync()  # (LKF_EINVAL here was the old cap)
            o.run(oh, pk, n, ar, alen, dd)
            ost = abi.lkf_stats()
            o.api["get_stats"](oh, C.byref(ost))
            assert eng.stats() == ost.as_dict(), b
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            assert len(grec) == len(orec), b
            for fld in abi.OUT_DTYPE.names:
                assert np.array_equal(grec[fld], orec[fld]), (b, fld)
            assert np.array_equal(gar, oar), b
            for d in dd_dts:
                assert fe(eng.h, d, ge) == 0 and fo(oh, d, go) == 0
                assert ge[13] == go[13], ("expected frames", b, d, ge[13], go[13])
                assert ge[11] == go[11] and ge[12] == go[12], ("chain broken/active bits", b, d)
                peak = max(peak, int(go[13]))
        assert peak > 16, peak
        for d in range(tr.ndts):
            gs, os_ = abi.lkf_fwd_state(), abi.lkf_fwd_state()
            assert eng.api["get_state"](eng.h, d, C.byref(gs)) == 0
            assert o.api["get_state"](oh, d, C.byref(os_)) == 0
            assert gs.as_tuple() == os_.as_tuple(), d
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()
