"""The dependency-descriptor stream tracker (streamtracker_dd.go) on the CPU
oracle, fed by forwarded SVC batches: every DD track's tracker sees its
descriptors' active decode targets and reports per-layer bitrates at host
ticks; pause drains them, stop freezes them.  The restatement is pinned by
streamtracker_dd_test.go TestStreamTrackerDD (oracle/kat_tracker.inc)."""
import numpy as np

from tests.oracle_lib import load as load_oracle


def dd_tracks(trace):
    return [t for t in range(trace.ntracks) if trace.tracks[t].has_dd]


def tick(api, h, ids, elapsed, abi):
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    out = np.zeros(max(1, len(ids)), dtype=abi.DD_TRACKER_STATUS_DTYPE)
    assert api["dd_trackers_tick"](h, ids.ctypes.data, len(ids), elapsed, out.ctypes.data) == 0
    return out[:len(ids)]


def run_dd_trackers(pkg, workload, api, h, tr, runner, abi):
    """Adds a tracker per DD track, forwards every batch (runner(b)), ticks
    after each; pauses / stops some on the way.  Returns the tick outputs."""
    tracks = dd_tracks(tr)
    ids = [api["add_stream_tracker_dd"](h, t) for t in tracks]
    assert all(i >= 0 for i in ids)
    assert api["add_stream_tracker_dd"](h, tracks[0]) < 0  # one per track
    outs = []
    for b in range(tr.nbatches):
        if b == 2:
            assert api["dd_tracker_ctl"](h, ids[0], abi.TRACKER_PAUSE, 1) == 0
            assert api["dd_tracker_ctl"](h, ids[-1], abi.TRACKER_STOP, 0) == 0
        if b == 3:
            assert api["dd_tracker_ctl"](h, ids[0], abi.TRACKER_PAUSE, 0) == 0
        runner(b)
        outs.append(tick(api, h, ids, 1_000_000_000 + 12345 * b, abi))
    return outs


def test_dd_tracker_oracle(pkg, workload):
    abi = pkg.abi
    o = load_oracle()
    tr = workload.Trace(5, duration_s=5.0, batch_s=1.0, rooms=4, svc_dd=1, seed=51)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        assert o.api["add_stream_tracker_dd"](h, [t for t in range(tr.ntracks) if not tr.tracks[t].has_dd][0]) < 0

        def runner(b):
            workload.queue_events(o.api, h, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(h, pk, n, ar, alen, tr.batch_dd(b)[0])

        outs = run_dd_trackers(pkg, workload, o.api, h, tr, runner, abi)
        first = outs[0]
        assert (first["max_spatial"] >= 0).all() and (first["worker"] == 1).all()
        assert (first["bitrate"][:, 0, 0] > 0).all()  # the base layer carries bytes
        assert (first["notifications"][:, 0] >= 1).all()
        assert (outs[2]["bitrate"][0] == 0).all() and outs[2]["worker"][0] == 1  # paused: the drained report
        assert (outs[3]["bitrate"][0] == 0).all()  # unpaused: reset
        assert outs[4]["worker"][-1] == 0  # stopped: no worker, the last report stays
        assert (outs[4]["bitrate"][-1] == outs[1]["bitrate"][-1]).all()
    finally:
        o.destroy(h)
        tr.close()
