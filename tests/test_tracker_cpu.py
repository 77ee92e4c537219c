"""Packet stream trackers on the CPU oracle (the checker of the GPU kernels;
the restatement is pinned by streamtracker_packet_test.go in
oracle/kat_tracker.inc): on a forwarded trace every streaming layer's tracker
turns active on its first packet, and its bitrate report gives each temporal
layer's bytes x 8 over the interval (streamtracker.go:286-310)."""
import ctypes as C

import numpy as np

from tests import tracker_lib
from tests.oracle_lib import load as load_oracle


def test_trackers_activate_and_report(workload):
    o = load_oracle()
    tr = workload.Trace(1, duration_s=1.0, batch_s=1.0, seed=1)
    oh = o.create(500)
    try:
        workload.load_topology(o.api, oh, tr)
        ids = tracker_lib.add_trackers(o.api, oh, tr, seed=1)
        pk, n, ar, alen = tr.batch(0)
        o.run(oh, pk, n, ar, alen)
        r = tracker_lib.tick(o.api, oh, ids, False, 10**9)
        assert (r["status"] == 1).all() and (r["notifications"] == 1).all()
        # bytes per (track, layer, temporal) of the batch, x 8 over one second
        pkts = [pk[i] for i in range(n)]
        k = 0
        for t in range(tr.ntracks):
            if tr.tracks[t].kind != 1:
                continue
            for layer in range(3):
                exp = np.zeros(4, dtype=np.int64)
                for p in pkts:
                    if p.track == t and p.layer == layer and p.payload_len > 0 and 0 <= p.temporal < 4:
                        exp[p.temporal] += (p.payload_off + p.payload_len) * 8
                assert np.array_equal(r["bitrate"][k], exp), (t, layer)
                k += 1
    finally:
        o.destroy(oh)
        tr.close()


def test_frame_trackers_active_then_stopped(workload):
    """StreamTrackerFrame on the oracle: every streaming layer's tracker turns
    active on its first packet and stays active while frames arrive (checks
    every 500 ms of virtual time); once the feed ends, the next checks find no
    two frames in the interval and report stopped (streamtracker_frame.go:124-142)."""
    o = load_oracle()
    tr = workload.Trace(1, duration_s=3.0, batch_s=0.1, seed=2)
    oh = o.create(500)
    try:
        workload.load_topology(o.api, oh, tr)
        ids = tracker_lib.add_frame_trackers(o.api, oh, tr, seed=1)
        for b in range(tr.nbatches):
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(oh, pk, n, ar, alen)
            now = tracker_lib.EPOCH + int((b + 1) * 0.1e9)
            r = tracker_lib.tick_at(o.api, oh, ids, b % 5 == 4, 0, now)
            if b >= 10:
                assert (r["status"] == 1).all(), b
        end = tracker_lib.EPOCH + int(tr.nbatches * 0.1e9)
        for k in range(1, 8):  # no packets any more: 2 s covers the 0.5 fps eval interval
            r = tracker_lib.tick_at(o.api, oh, ids, True, 0, end + k * 500_000_000)
        assert (r["status"] == 0).all()
        assert (r["notifications"] == 2).all()
    finally:
        o.destroy(oh)
        tr.close()
