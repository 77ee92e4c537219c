"""Packet stream trackers (StreamTracker + StreamTrackerPacket,
streamtracker.go / streamtracker_packet.go; Observe from forwardRTP
receiver.go:686-695), engine vs oracle.

Every (video track, spatial layer) of a trace gets a tracker with random
SamplesRequired / CyclesRequired; 100-ms batches are forwarded, CheckStatus
ticks come every 500 ms and bitrate reports every second, and trackers are
reset, paused, resumed and stopped along the way: statuses, notification
counts, bitrates and cumulative bitrates must match at every tick."""
import numpy as np
import pytest

from tests import tracker_lib
from tests.oracle_lib import load as load_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=7), dict(config=1, seed=3)])
def test_stream_trackers_match_oracle(pkg, workload, cfg):
    o = load_oracle()
    abi = pkg.abi
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=6.0, batch_s=0.1, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    rng = np.random.default_rng(2)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        ids = tracker_lib.add_trackers(eng.api, eng.h, tr, seed=5)
        assert np.array_equal(ids, tracker_lib.add_trackers(o.api, oh, tr, seed=5))
        changes = 0
        for b in range(tr.nbatches):
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            eng.submit(pk, n, ar, alen)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen)
            eng.drain()
            if b % 5 == 4 or b % 10 == 9:
                check, el = b % 5 == 4, (10**9 if b % 10 == 9 else 0)
                g = tracker_lib.tick(eng.api, eng.h, ids, check, el)
                r = tracker_lib.tick(o.api, oh, ids, check, el)
                for f in ("tracker", "status", "bitrate_changed", "notifications", "bitrate", "cumulative"):
                    assert np.array_equal(g[f], r[f]), (b, f)
                changes += int(r["bitrate_changed"].sum())
            if b % 10 == 3:  # reset / pause / resume / stop a few trackers
                for k in rng.choice(ids, size=min(4, len(ids)), replace=False):
                    op = int(rng.integers(1, 4))
                    arg = int(rng.integers(0, 2))
                    assert eng.api["stream_tracker_ctl"](eng.h, int(k), op, arg) == 0
                    assert o.api["stream_tracker_ctl"](oh, int(k), op, arg) == 0
        final = tracker_lib.tick(o.api, oh, ids, True, 0)
        assert (final["status"] == 1).any() and changes > 0
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=8), dict(config=1, seed=4)])
def test_frame_trackers_match_oracle(pkg, workload, cfg):
    """StreamTrackerFrame (streamtracker_frame.go:39-211; no reference test:
    parity unpinned beyond this engine-vs-oracle check): marker packets per
    batch, CheckStatus ticks every 100-300 ms of virtual time (the frame
    tracker's own eval interval decides which ones count), bitrate reports
    every second, resets / pauses / stops along the way."""
    o = load_oracle()
    abi = pkg.abi
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=8.0, batch_s=0.1, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    rng = np.random.default_rng(3)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        ids = tracker_lib.add_frame_trackers(eng.api, eng.h, tr, seed=6)
        assert np.array_equal(ids, tracker_lib.add_frame_trackers(o.api, oh, tr, seed=6))
        stops = actives = 0
        for b in range(tr.nbatches):
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            eng.submit(pk, n, ar, alen)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen)
            eng.drain()
            now = tracker_lib.EPOCH + int((b + 1) * 0.1e9)
            check = b % int(rng.integers(1, 4)) == 0
            el = 10**9 if b % 10 == 9 else 0
            g = tracker_lib.tick_at(eng.api, eng.h, ids, check, el, now)
            r = tracker_lib.tick_at(o.api, oh, ids, check, el, now)
            for f in ("tracker", "status", "bitrate_changed", "notifications", "bitrate", "cumulative"):
                assert np.array_equal(g[f], r[f]), (b, f)
            actives += int((r["status"] == 1).sum())
            stops += int((r["status"] == 0).sum())
            if b % 15 == 7:
                for k in rng.choice(ids, size=min(4, len(ids)), replace=False):
                    op = int(rng.integers(1, 4))
                    arg = int(rng.integers(0, 2))
                    assert eng.api["stream_tracker_ctl"](eng.h, int(k), op, arg) == 0
                    assert o.api["stream_tracker_ctl"](oh, int(k), op, arg) == 0
        assert actives > 0 and stops > 0
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


@pytest.mark.parametrize("cfg", [dict(config=5, rooms=4, svc_dd=1, seed=51), dict(config=5, rooms=6, svc_dd=-1, seed=52)])
def test_dd_tracker_matches_oracle(pkg, workload, cfg):
    """StreamTrackerDependencyDescriptor (streamtracker_dd.go) observed in
    k_dd_decode per batch: every tick's max layers, notifications, statuses
    and bitrates (with a pause, an unpause and a stop on the way) equal the
    oracle's."""
    from tests.test_dd_tracker_cpu import run_dd_trackers
    o = load_oracle()
    abi = pkg.abi
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=5.0, batch_s=1.0, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)

        def run_eng(b):
            workload.queue_events(eng.api, eng.h, tr, b)
            pk, n, ar, alen = tr.batch(b)
            eng.submit(pk, n, ar, alen, tr.batch_dd(b)[0])
            eng.run()
            eng.sync()

        def run_orc(b):
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(oh, pk, n, ar, alen, tr.batch_dd(b)[0])

        g = run_dd_trackers(pkg, workload, eng.api, eng.h, tr, run_eng, abi)
        r = run_dd_trackers(pkg, workload, o.api, oh, tr, run_orc, abi)
        for b, (x, y) in enumerate(zip(g, r)):
            for f in abi.DD_TRACKER_STATUS_DTYPE.names:
                if f != "reserved":
                    assert np.array_equal(x[f], y[f]), (b, f, x[f], y[f])
        assert (r[0]["bitrate"][:, 0, 0] > 0).all()
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()
