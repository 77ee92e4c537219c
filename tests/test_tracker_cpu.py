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
