"""AllocateOptimal through the oracle's C entry point (the checker of the GPU
kernel): the transcribed TestForwarderAllocateOptimal sequence runs in
oracle/kat (test_oracle_kat); here the orc_allocate_optimal mirror of
lkf_allocate_optimal is driven on a forwarded trace and checked for the
reference's invariants: audio answers VideoAllocationDefault, a paused
allocation has no target and no request, BandwidthRequested is the optimal
bandwidth exactly when a target is set, and BandwidthDelta is taken against
the previous allocation (getBandwidthNeeded forwarder.go:1880-1886)."""
import numpy as np

from tests.oracle_lib import load as load_oracle
from tests.test_alloc_gpu import allocate, make_alloc_reqs, run_step, stream_allocator_steps, video_mask


def test_orc_allocate_optimal_invariants(pkg, workload):
    o = load_oracle()
    abi = pkg.abi
    tr = workload.Trace(2, duration_s=2.0, batch_s=1.0, rooms=2, seed=1)
    oh = o.create(500)
    try:
        workload.load_topology(o.api, oh, tr)
        workload.queue_events(o.api, oh, tr, 0)
        pk, n, ar, alen = tr.batch(0)
        o.run(oh, pk, n, ar, alen)
        reqs = make_alloc_reqs(abi, tr.ndts, seed=2)
        a = allocate(o.api, oh, reqs, abi)
        video = np.array([tr.tracks[tr.downtracks[int(d)].track].kind == 1 for d in a["dt"]])
        aud = a[~video]
        assert len(aud) and (aud["pause_reason"] == 3).all() and (aud["target_spatial"] == -1).all()
        vid = a[video]
        paused = vid["target_spatial"] == -1
        assert (vid["request_spatial"][paused] == -1).all()
        assert (vid["bandwidth_requested"][paused] == 0).all()
        assert (vid["bandwidth_requested"][~paused] == vid["bandwidth_needed"][~paused]).all()
        b = allocate(o.api, oh, reqs, abi)  # again: delta against getBandwidthNeeded(brs, target, last requested)
        for x, y, q in zip(a[video], b[video], reqs[video]):
            prev = x["bandwidth_requested"]
            if x["target_spatial"] >= 0 and q["bitrates"][x["target_spatial"], x["target_temporal"]] > 0:
                prev = q["bitrates"][x["target_spatial"], x["target_temporal"]]
            assert y["bandwidth_delta"] == y["bandwidth_requested"] - prev
    finally:
        o.destroy(oh)
        tr.close()


def test_orc_pause_next_higher_invariants(pkg, workload):
    """Pause / GetNextHigherTransition / AllocateNextHigher through the oracle's
    C entry points on a forwarded trace (the sequence the GPU parity test
    replays): Pause leaves no target and marks only the bandwidth reason
    deficient; a boost is a deficient DownTrack's move to a layer with a
    bitrate, its BandwidthDelta against the previous target's bitrate; a
    transition, when available, never goes down in bitrate."""
    o = load_oracle()
    abi = pkg.abi
    tr = workload.Trace(2, duration_s=5.0, batch_s=1.0, rooms=2, seed=6)
    oh = o.create(500)
    try:
        workload.load_topology(o.api, oh, tr)
        boosted = avail = 0
        for b in range(tr.nbatches):
            for step in stream_allocator_steps(abi, tr.ndts, b, video_mask(abi, tr)):
                r = run_step(o.api, oh, abi, step)
                kind, reqs, caps = step
                if kind == "pause":
                    assert (r["target_spatial"] == -1).all() and (r["request_spatial"] == -1).all()
                    assert (r["bandwidth_requested"] == 0).all()
                    assert ((r["pause_reason"] == 4) == (r["is_deficient"] == 1)).all()
                elif kind == "transition":
                    a = r[r["available"] == 1]
                    assert (a["bandwidth_delta"] >= 0).all()
                    avail += len(a)
                elif kind == "next_higher":
                    x = r[r["boosted"] == 1]
                    boosted += len(x)
                    q = reqs[r["boosted"] == 1]
                    got = q["bitrates"][np.arange(len(x)), x["target_spatial"], x["target_temporal"]]
                    assert (got == x["bandwidth_requested"]).all() and (got > 0).all()
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(oh, pk, n, ar, alen)
        assert boosted > 0 and avail > 0
    finally:
        o.destroy(oh)
        tr.close()
