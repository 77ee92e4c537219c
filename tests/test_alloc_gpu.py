"""Forwarder.AllocateOptimal (forwarder.go:591-725), AllocateNextHigher
(:1107-1217), GetNextHigherTransition (:1219-1306) and Pause (:1308-1351),
engine vs oracle.

The oracle's restatement is pinned by TestForwarderAllocateOptimal
(oracle/kat_sfu.inc).  Here every DownTrack of a trace gets an allocation with
random available layers, bitrate tables (zeros included: feed dry, measurement
pending) and overshoot permission, between forwarded batches and twice in a row
(BandwidthDelta against the previous allocation): the allocations, the batches
forwarded after them (new targets, resyncs when paused) and the Forwarder state
must be identical."""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle

pytestmark = pytest.mark.gpu


def make_alloc_reqs(abi, ndts, seed):
    rng = np.random.default_rng(seed)
    r = np.zeros(ndts, dtype=abi.ALLOC_REQ_DTYPE)
    r["dt"] = rng.permutation(ndts)
    r["available_layers"] = rng.integers(0, 8, ndts)
    brs = rng.integers(100_000, 3_000_000, (ndts, 3, 4))
    brs[rng.random((ndts, 3, 4)) < 0.3] = 0
    brs[rng.random(ndts) < 0.1] = 0  # feed dry
    r["bitrates"] = brs
    r["allow_overshoot"] = rng.integers(0, 2, ndts)
    return r


def allocate(api, h, reqs, abi):
    out = np.zeros(len(reqs), dtype=abi.ALLOCATION_DTYPE)
    assert api["allocate_optimal"](h, reqs.ctypes.data, len(reqs), out.ctypes.data) == 0
    return out


def pause(api, h, reqs, abi):
    out = np.zeros(len(reqs), dtype=abi.ALLOCATION_DTYPE)
    assert api["pause"](h, reqs.ctypes.data, len(reqs), out.ctypes.data) == 0
    return out


def next_higher(api, h, reqs, caps, abi):
    out = np.zeros(len(reqs), dtype=abi.ALLOCATION_DTYPE)
    caps = np.ascontiguousarray(caps, dtype=np.int64)
    assert api["allocate_next_higher"](h, reqs.ctypes.data, caps.ctypes.data, len(reqs), out.ctypes.data) == 0
    return out


def transition(api, h, reqs, abi):
    out = np.zeros(len(reqs), dtype=abi.VIDEO_TRANSITION_DTYPE)
    assert api["next_higher_transition"](h, reqs.ctypes.data, len(reqs), out.ctypes.data) == 0
    return out


def video_mask(abi, trace):
    """Per DownTrack: its track is video (the stream allocator manages only those)."""
    return np.array([trace.tracks[trace.downtracks[d].track].kind == abi.LKF_KIND_VIDEO for d in range(trace.ndts)])


def stream_allocator_steps(abi, ndts, b, video):
    """The allocation calls the stream allocator makes between batch b-1 and b
    (streamallocator.go: allocateAllTracks -> AllocateOptimal / Pause, then
    probing -> GetNextHigherTransition / AllocateNextHigher): a list of
    (call, reqs, capacities).  Pause goes to video DownTracks only: the
    allocator tracks only video (Forwarder.Pause dereferences the video layer
    selector); `video` is the per-DownTrack mask."""
    rng = np.random.default_rng(1000 + b)
    steps = []
    if b == 1:
        steps.append(("optimal", make_alloc_reqs(abi, ndts, seed=70), None))
        r = make_alloc_reqs(abi, ndts, seed=71)
        pick = rng.random(ndts) < 0.6
        steps.append(("pause", r[pick & video[r["dt"]]], None))
    elif b >= 2:
        r = make_alloc_reqs(abi, ndts, seed=80 + b)
        r["bitrates"] = np.sort(r["bitrates"].reshape(ndts, -1), axis=1).reshape(ndts, 3, 4)  # layered: rising
        steps.append(("transition", r, None))
        caps = rng.choice(np.array([0, 50_000, 500_000, 5_000_000, 1 << 40]), ndts)
        steps.append(("next_higher", r, caps))
        steps.append(("transition", r, None))
    return steps


def run_step(api, h, abi, step):
    kind, reqs, caps = step
    if kind == "optimal":
        return allocate(api, h, reqs, abi)
    if kind == "pause":
        return pause(api, h, reqs, abi)
    if kind == "transition":
        return transition(api, h, reqs, abi)
    return next_higher(api, h, reqs, caps, abi)


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=5), dict(config=5, rooms=6, svc_dd=1),
                                 dict(config=5, rooms=6, svc_dd=0), dict(config=2, rooms=2, h264=1, seed=3)])
def test_allocate_optimal_matches_oracle(pkg, workload, cfg):
    o = load_oracle()
    abi = pkg.abi
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=4.0, batch_s=1.0, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        moved = 0
        for b in range(tr.nbatches):
            if b in (1, 3):
                for k in range(2):
                    reqs = make_alloc_reqs(abi, tr.ndts, seed=10 * b + k)
                    g = allocate(eng.api, eng.h, reqs, abi)
                    r = allocate(o.api, oh, reqs, abi)
                    for f in abi.ALLOCATION_DTYPE.names:
                        if f != "reserved":
                            assert np.array_equal(g[f], r[f]), (b, k, f)
                    moved += int((r["bandwidth_delta"] != 0).sum())
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            dd = tr.batch_dd(b)[0] if tr.has_dd() else None
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen, dd)
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            assert len(grec) == len(orec), b
            for f in abi.OUT_DTYPE.names:
                assert np.array_equal(grec[f], orec[f]), (b, f)
            assert np.array_equal(gar, oar), b
        assert moved > 0
        for dt in range(tr.ndts):
            gs, os_ = abi.lkf_fwd_state(), abi.lkf_fwd_state()
            eng.api["get_state"](eng.h, dt, C.byref(gs))
            o.api["get_state"](oh, dt, C.byref(os_))
            assert gs.as_tuple() == os_.as_tuple(), dt
        gsum, osum = pkg.downtrack_summaries(eng.api, eng.h), pkg.downtrack_summaries(o.api, oh)
        for f in abi.DT_SUMMARY_DTYPE.names:
            assert np.array_equal(gsum[f], osum[f]), f
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=6), dict(config=5, rooms=6, svc_dd=1),
                                 dict(config=2, rooms=2, h264=1, seed=4)])
def test_pause_and_next_higher_match_oracle(pkg, workload, cfg):
    """Pause, then per batch GetNextHigherTransition / AllocateNextHigher with
    random channel capacities (zero to unlimited): the results (boosted flag
    included), the batches forwarded after them and the Forwarder state."""
    o = load_oracle()
    abi = pkg.abi
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=6.0, batch_s=1.0, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        boosted = avail = 0
        for b in range(tr.nbatches):
            for step in stream_allocator_steps(abi, tr.ndts, b, video_mask(abi, tr)):
                g = run_step(eng.api, eng.h, abi, step)
                r = run_step(o.api, oh, abi, step)
                for f in g.dtype.names:
                    if f != "reserved":
                        assert np.array_equal(g[f], r[f]), (b, step[0], f)
                if step[0] == "next_higher":
                    boosted += int(r["boosted"].sum())
                if step[0] == "transition":
                    avail += int(r["available"].sum())
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            dd = tr.batch_dd(b)[0] if tr.has_dd() else None
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen, dd)
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            assert len(grec) == len(orec), b
            for f in abi.OUT_DTYPE.names:
                assert np.array_equal(grec[f], orec[f]), (b, f)
            assert np.array_equal(gar, oar), b
        assert boosted > 0 and avail > 0
        for dt in range(tr.ndts):
            gs, os_ = abi.lkf_fwd_state(), abi.lkf_fwd_state()
            eng.api["get_state"](eng.h, dt, C.byref(gs))
            o.api["get_state"](oh, dt, C.byref(os_))
            assert gs.as_tuple() == os_.as_tuple(), dt
        gsum, osum = pkg.downtrack_summaries(eng.api, eng.h), pkg.downtrack_summaries(o.api, oh)
        for f in abi.DT_SUMMARY_DTYPE.names:
            assert np.array_equal(gsum[f], osum[f]), f
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=41), dict(config=5, rooms=6, svc_dd=1, seed=42),
                                 dict(config=5, rooms=6, svc_dd=0, seed=43), dict(config=2, rooms=2, h264=1, seed=44)])
def test_provisional_pass_matches_oracle(pkg, workload, cfg):
    """The stream allocator's cooperative pass (Forwarder.Provisional*,
    forwarder.go:727-1105, and allocateAllTracks' greedy per subscriber) between
    batches: every result, the batches forwarded on the committed targets and
    the Forwarder state must be identical."""
    from tests import prov_lib
    o = load_oracle()
    abi = pkg.abi
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=4.0, batch_s=1.0, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        committed = 0
        for b in range(tr.nbatches):
            if b in (1, 2, 3):
                for i, step in enumerate(prov_lib.steps(tr, seed=100 * b + cfg.get("seed", 0))):
                    g = prov_lib.run(eng.api, eng.h, step)
                    r = prov_lib.run(o.api, oh, step)
                    if r is None:
                        continue
                    for f in r.dtype.names:
                        if f != "reserved":
                            assert np.array_equal(g[f], r[f]), (b, i, step[0], f)
                    if step[0] in ("commit", "allocate_all"):
                        committed += len(r)
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            dd = tr.batch_dd(b)[0] if tr.has_dd() else None
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen, dd)
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            assert len(grec) == len(orec), b
            for f in abi.OUT_DTYPE.names:
                assert np.array_equal(grec[f], orec[f]), (b, f)
            assert np.array_equal(gar, oar), b
        assert committed > 0
        for dt in range(tr.ndts):
            gs, os_ = abi.lkf_fwd_state(), abi.lkf_fwd_state()
            eng.api["get_state"](eng.h, dt, C.byref(gs))
            o.api["get_state"](oh, dt, C.byref(os_))
            assert gs.as_tuple() == os_.as_tuple(), dt
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()
