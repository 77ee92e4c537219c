"""NACK -> RTX on the CPU oracle (DownTrack.retransmitPackets, downtrack.go:1596-1712).

Self-consistency with the forwarding path: a retransmission's payload bytes
(munged VP8 descriptor + payload) equal the wire bytes the DownTrack forwarded
for that sequence number, its header carries the sequencer's marker/SN/TS and
the DownTrack's SSRC/PT; a repeated NACK inside the RTT is suppressed, later
ones count up to three (sequencer.go:263-332); deficient DownTracks drop the
disallowed layers (forwarder.go:1424-1432)."""
import ctypes as C

import numpy as np

from tests import rtx_lib
from tests.oracle_lib import load as load_oracle

EPOCH = 1700000000 * 10**9


def _forward(o, workload, trace, nb):
    h = o.create(500)
    workload.load_topology(o.api, h, trace)
    fwd = {}  # (dt, target_sn) -> (record, wire bytes) of the last forwarded copy
    pkg = __import__("importlib").import_module("livekit-server_amd")
    for b in range(nb):
        workload.queue_events(o.api, h, trace, b)
        pk, n, ar, alen = trace.batch(b)
        o.run(h, pk, n, ar, alen)
        rec, arena = pkg.drain_arrays(o.api, h)
        for r in rec:
            fwd[(int(r["dt"]), int(r["ext_sn"]) & 0xFFFF)] = (r, bytes(arena[r["out_off"]:r["out_off"] + r["out_len"]]))
    return h, fwd


def _payload(pkt):
    cc = pkt[0] & 0xF
    n = 12 + 4 * cc
    if pkt[0] & 0x10:
        n += 4 + 4 * ((pkt[n + 2] << 8) | pkt[n + 3])
    return pkt[n:]


def test_oracle_rtx_matches_forwarded_packets(workload):
    o = load_oracle()
    tr = workload.Trace(2, duration_s=3.0, batch_s=1.0, rooms=3, seed=9)
    nb = 3
    h, fwd = _forward(o, workload, tr, nb)
    try:
        idx = rtx_lib.packet_index(tr, nb)
        nacks = rtx_lib.make_nacks(o.api, h, tr, seed=3)
        assert len(nacks) > 100
        now = EPOCH + nb * 10**9 + 500 * 10**6
        rtx = rtx_lib.rtx_lookup(o.api, h, nacks, now)
        assert len(rtx) > 50
        assert np.all(rtx["nacked"] == 1)
        # the second NACK of the same SN in one list comes inside the RTT: suppressed
        pairs = set()
        for r in rtx:
            key = (int(r["dt"]), int(r["target_sn"]))
            assert key not in pairs
            pairs.add(key)
        out, wire = rtx_lib.rtx_emit(o.api, h, tr, rtx, idx)
        assert len(out) > 50
        checked = 0
        for r in out:
            pkt = bytes(wire[r["out_off"]:r["out_off"] + r["out_len"]])
            rx = rtx[r["pkt"]]
            dtp = tr.downtracks[int(r["dt"])]
            assert (pkt[2] << 8 | pkt[3]) == rx["target_sn"]
            assert int.from_bytes(pkt[8:12], "big") == dtp.ssrc and (pkt[1] & 0x7F) == dtp.payload_type
            assert bool(pkt[1] & 0x80) == bool(rx["marker"])
            f = fwd.get((int(r["dt"]), int(rx["target_sn"])))
            if f is not None:
                assert _payload(pkt) == _payload(f[1])  # same munged descriptor + payload as forwarded
                assert pkt[4:8] == f[1][4:8]            # same munged timestamp
                checked += 1
        assert checked > 50
        # a later NACK of the same records counts up (nacked 2), up to maxAck 3
        rtx2 = rtx_lib.rtx_lookup(o.api, h, nacks, now + 10**9)
        assert len(rtx2) == len(rtx) and np.all(rtx2["nacked"] == 2)
    finally:
        o.destroy(h)
        tr.close()


def _ext_element(pkt, eid):
    """The payload of extension element `eid` of an RTP packet (one- or two-byte profile), or None."""
    if not pkt[0] & 0x10:
        return None
    h = 12 + 4 * (pkt[0] & 0xF)
    prof = (pkt[h] << 8) | pkt[h + 1]
    q, end = h + 4, h + 4 + 4 * ((pkt[h + 2] << 8) | pkt[h + 3])
    while q < end:
        if pkt[q] == 0:
            q += 1
            continue
        if prof == 0xBEDE:
            i, ln, q = pkt[q] >> 4, (pkt[q] & 0xF) + 1, q + 1
        else:
            i, ln, q = pkt[q], pkt[q + 1], q + 2
        if i == eid:
            return bytes(pkt[q:q + ln])
        q += ln
    return None


def test_oracle_rtx_keeps_dependency_descriptor(workload):
    """RTX of a DD DownTrack: the pacer writes epm.ddBytes (sequencer.go:198-199,
    :326; downtrack.go:1684) — the same DD element the forwarded packet carried."""
    o = load_oracle()
    tr = workload.Trace(5, duration_s=3.0, batch_s=1.0, rooms=4, svc_dd=1, seed=14)
    nb = 3
    h = o.create(500)
    workload.load_topology(o.api, h, tr)
    pkg = __import__("importlib").import_module("livekit-server_amd")
    fwd = {}
    try:
        for b in range(nb):
            workload.queue_events(o.api, h, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(h, pk, n, ar, alen, tr.batch_dd(b)[0])
            rec, arena = pkg.drain_arrays(o.api, h)
            for r in rec:
                fwd[(int(r["dt"]), int(r["ext_sn"]) & 0xFFFF)] = bytes(arena[r["out_off"]:r["out_off"] + r["out_len"]])
        idx = rtx_lib.packet_index(tr, nb)
        nacks = rtx_lib.make_nacks(o.api, h, tr, seed=4)
        rtx = rtx_lib.rtx_lookup(o.api, h, nacks, EPOCH + nb * 10**9 + 500 * 10**6)
        out, wire = rtx_lib.rtx_emit(o.api, h, tr, rtx, idx)
        with_dd = 0
        for r in out:
            d = int(r["dt"])
            eid = int(tr.downtracks[d].ext_dd)
            pkt = bytes(wire[r["out_off"]:r["out_off"] + r["out_len"]])
            orig = fwd.get((d, int(r["ext_sn"]) & 0xFFFF))
            if not eid or orig is None:
                continue
            assert _ext_element(pkt, eid) == _ext_element(orig, eid), d
            assert _payload(pkt) == _payload(orig)
            with_dd += _ext_element(pkt, eid) is not None
        assert with_dd > 20
    finally:
        o.destroy(h)
        tr.close()


def test_oracle_rtx_from_bucket(workload):
    """The receivers' buckets (bucket_oracle.h) filled by ingest give the same
    retransmissions as the trace's own packets, wherever the bucket still
    holds the source (audio buckets keep 200 packets, video 500)."""
    o = load_oracle()
    tr = workload.Trace(2, duration_s=3.0, batch_s=1.0, rooms=2, seed=11, loss=0.02, reorder=0.01)
    nb = 3
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        workload.load_streams(o.api, h, tr)
        rtx_lib.ingest_forward(o.api, h, tr, workload, nb,
                               lambda b, pk, n, ar, alen: o.run(h, pk if n else None, n, ar, alen))
        nacks = rtx_lib.make_nacks(o.api, h, tr, seed=6)
        r = rtx_lib.rtx_lookup(o.api, h, nacks, EPOCH + nb * 10**9 + 5 * 10**8)
        assert len(r) > 50
        idx = rtx_lib.packet_index(tr, nb)
        io, iw = rtx_lib.rtx_emit(o.api, h, tr, r, idx)
        bo, bw = rtx_lib.rtx_emit_bucket(o.api, h, r)
        want, got = rtx_lib.wire_by_rtx(io, iw), rtx_lib.wire_by_rtx(bo, bw)
        assert set(got) <= set(want)
        for k, v in got.items():
            assert v == want[k], k
        video = [k for k in want if tr.tracks[tr.downtracks[int(r["dt"][k])].track].kind != 0]
        assert len(got) > 0.6 * len(want) and sum(k in got for k in video) > 0.9 * len(video), (len(got), len(want))
    finally:
        o.destroy(h)


def test_oracle_bucket_too_old_and_wrap(workload):
    """A 5-s batch wraps the audio buckets inside the batch and delivers one
    audio and one video datagram later than their bucket's window: both are
    rejected (ErrPacketTooOld: no ExtPacket, no LKF_FLOW_BUCKET) although
    RTPStatsReceiver counts them as out-of-order arrivals, and the RTX reads
    of the wrapped audio ring return the latest packets."""
    import importlib
    from tests import bucket_lib
    pkg = importlib.import_module("livekit-server_amd")
    abi = importlib.import_module("livekit-server_amd.abi")
    o = load_oracle()
    tr = workload.Trace(2, duration_s=5.0, batch_s=5.0, rooms=1, seed=3, loss=0.0, reorder=0.0)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        workload.load_streams(o.api, h, tr)
        arr, n, ar, alen, moved = bucket_lib.late_batch(tr)
        assert len(moved) == 2
        assert o.api["ingest"](h, arr, n, ar, alen) == 0
        f = pkg.flows_array(o.api, h)
        rej = [i for i in range(n) if (f["flags"][i] & abi.LKF_FLOW_OUT_OF_ORDER)
               and not (f["flags"][i] & (abi.LKF_FLOW_BUCKET | abi.LKF_FLOW_DUPLICATE | abi.LKF_FLOW_PADDING))]
        assert len(rej) == 2, rej
        assert all(not (f["flags"][i] & abi.LKF_FLOW_FORWARD) for i in rej)
        stored = int(np.count_nonzero(f["flags"] & abi.LKF_FLOW_BUCKET))
        assert stored == int(np.count_nonzero(f["flags"] & abi.LKF_FLOW_FORWARD)) > 1000
    finally:
        o.destroy(h)
