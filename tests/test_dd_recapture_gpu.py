"""The round-5 DD-cursor report: graph re-captures forced
while earlier dependency-descriptor runs are still queued.

A run whose control ops outgrow the batch context's staging (and op buffers)
drains the engine and re-captures that context's stage graphs; before commit
c303318 a re-capture destroyed the previous graph executable while its last
launch could still be queued, and the batch's DD bump cursor was then found
holding a pointer-sized value.  Here configs[4] (AV1/VP9 with
dependency descriptors) runs pipelined with no sync between runs, and two of
the runs carry thousands of extra control ops (SetMaxTemporalLayer at the
current maximum, at spread packet indices), so their contexts re-capture
under queued runs.  Afterwards every context's cursors must be within the DD
arena, no capacity error may be reported, and the cumulative counters, every
Forwarder state and the per-DownTrack summaries must equal the CPU oracle's.
"""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle

pytestmark = pytest.mark.gpu


def _extra_ops(abi, trace, n_pkts, count, seed):
    rng = np.random.default_rng(seed)
    video = [d for d in range(trace.ndts) if trace.tracks[trace.downtracks[d].track].kind == abi.LKF_KIND_VIDEO]
    ev = (abi.lkfs_event * count)()
    for i in range(count):
        ev[i].dt = int(video[int(rng.integers(len(video)))])
        ev[i].op = abi.LKF_CTL_SET_MAX_TEMPORAL
        ev[i].a[0] = 3  # DefaultMaxLayerTemporal: the value the DownTracks already have
        ev[i].at_pkt = int(rng.integers(max(1, n_pkts)))
    return ev


def test_dd_cursors_after_recapture_under_queued_runs(pkg, workload, abi):
    tr = workload.Trace(5, duration_s=3.0, batch_s=0.5, rooms=60)
    o = load_oracle()
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    f = eng.lib.lkf_debug_dd_cursors
    f.restype, f.argtypes = C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        cum = {"tuples": 0, "forwarded": 0, "out_bytes": 0, "arena_bytes": 0}
        keep = []
        for b in range(tr.nbatches):
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            if b in (2, 4):  # staging growth: a drain and a re-capture of this context's graphs
                ev = _extra_ops(abi, tr, n, 6000 * b, seed=b)
                keep.append(ev)
                assert eng.api["ctl_batch"](eng.h, C.cast(ev, C.c_void_p), len(ev)) == 0
                assert o.api["ctl_batch"](oh, C.cast(ev, C.c_void_p), len(ev)) == 0
            dd = tr.batch_dd(b)[0]
            eng.submit(pk, n, ar, alen, dd)
            eng.run()  # no sync: earlier runs stay queued
            o.run(oh, pk, n, ar, alen, dd)
            st = abi.lkf_stats()
            o.api["get_stats"](oh, C.byref(st))
            for k, v in st.as_dict().items():
                if k in cum:
                    cum[k] += v
        eng.sync()  # a capacity error (a corrupt cursor) would be reported here
        cur = (C.c_uint64 * 7)()
        assert f(eng.h, cur) == 0
        for c in range(3):
            assert cur[2 * c] <= cur[6], ("context %d DD cursor %d beyond the arena %d" % (c, cur[2 * c], cur[6]))
            assert cur[2 * c + 1] < (1 << 31)
        assert max(cur[0], cur[2], cur[4]) > 0  # the DD arena was used
        g = eng.cumulative()
        assert {k: g[k] for k in cum} == cum
        for d in range(tr.ndts):
            gs, os_ = abi.lkf_fwd_state(), abi.lkf_fwd_state()
            assert eng.api["get_state"](eng.h, d, C.byref(gs)) == 0
            assert o.api["get_state"](oh, d, C.byref(os_)) == 0
            assert gs.as_tuple() == os_.as_tuple(), d
        gsum = pkg.downtrack_summaries(eng.api, eng.h)
        osum = pkg.downtrack_summaries(o.api, oh)
        for fld in abi.DT_SUMMARY_DTYPE.names:
            assert np.array_equal(gsum[fld], osum[fld]), fld
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()
