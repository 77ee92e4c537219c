"""Ingress (Buffer.calc) and active-speaker ranking on the CPU oracle.

The synthetic generator knows the ExtPacket each datagram should become; with
no loss or reordering the oracle's Buffer.calc restatement must reproduce the
generator's ExtPacket batch byte for byte (wrap-around unwrap, padding-free SN
adjustment, header/extension/VP8 parsing).  With loss and reordering, the flow
records must account for every datagram.
"""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle


def _ingested(o, abi, h):
    lib = o.lib
    lib.orc_ingested_ptr.argtypes = [C.c_void_p, C.POINTER(C.POINTER(abi.lkf_pkt)), C.POINTER(C.c_uint32)]
    lib.orc_ingested_ptr.restype = C.c_int
    pk = C.POINTER(abi.lkf_pkt)()
    n = C.c_uint32()
    lib.orc_ingested_ptr(h, C.byref(pk), C.byref(n))
    return pk, n.value


@pytest.mark.parametrize("kw", [
    dict(config=1, duration_s=2.0),
    dict(config=2, duration_s=2.0, rooms=2, loss=0.0, reorder=0.0),
    dict(config=3, duration_s=2.0, rooms=1),
    dict(config=5, duration_s=2.0, rooms=3, loss=0.0, reorder=0.0, svc_dd=0),  # VP9 descriptor, SVC dispatch
    dict(config=5, duration_s=2.0, rooms=3, loss=0.0, reorder=0.0),  # + AV1 / VP9 dependency descriptors
    dict(config=1, duration_s=2.0, h264=1),  # H.264 key frames (IsH264KeyFrame forms)
    dict(config=2, duration_s=2.0, rooms=2, loss=0.0, reorder=0.0, h264=1),
])
def test_oracle_ingest_reproduces_extpackets(kw, pkg, workload, abi):
    o = load_oracle()
    tr = workload.Trace(**kw)
    h = o.create(500)
    keys = 0
    try:
        workload.load_topology(o.api, h, tr)
        workload.load_streams(o.api, h, tr)
        for b in range(tr.nbatches):
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](h, rp, n, ar, alen) == 0
            pk, m = _ingested(o, abi, h)
            spk, sn, _, _ = tr.batch(b)
            assert m == sn == n
            got = C.string_at(pk, 64 * m) if m else b""
            want = C.string_at(spk, 64 * sn) if sn else b""
            assert got == want, "batch %d ExtPackets differ" % b
            if tr.has_dd():  # the DependencyDescriptorParser's view, per ExtPacket
                dsz = C.sizeof(abi.lkf_pkt_dd)
                buf = C.create_string_buffer(max(1, m) * dsz)
                k = C.c_uint32()
                assert o.api["ingested_dd"](h, buf, m, C.byref(k)) == 0 and k.value == m
                assert buf.raw[: m * dsz] == C.string_at(tr.batch_dd(b)[0], m * dsz), "batch %d DD differs" % b
            if kw.get("h264"):
                keys += int(np.sum(np.frombuffer(got, np.uint8).reshape(-1, 64)[:, abi.lkf_pkt.flags.offset] & 0x1 != 0)) if m else 0
            fl = pkg.flows_array(o.api, h)
            assert len(fl) == n
            assert np.all(fl["flags"] & 0x20)  # every datagram forwarded
            assert np.array_equal(fl["pkt"], np.arange(n, dtype=np.uint32))
        if kw.get("h264"):
            assert keys > 0
    finally:
        o.destroy(h)
        tr.close()


def test_oracle_ingest_loss_and_reorder_accounting(pkg, workload, abi):
    o = load_oracle()
    tr = workload.Trace(2, duration_s=3.0, rooms=2, loss=0.1, reorder=0.05, seed=5)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        workload.load_streams(o.api, h, tr)
        nloss = nooo = nfwd = 0
        for b in range(tr.nbatches):
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](h, rp, n, ar, alen) == 0
            fl = pkg.flows_array(o.api, h)
            fwd = (fl["flags"] & 0x20) != 0
            _, m = _ingested(o, abi, h)
            assert fwd.sum() == m
            assert np.array_equal(fl["pkt"][fwd], np.arange(m, dtype=np.uint32))
            assert np.all(fl["pkt"][~fwd] == 0xFFFFFFFF)
            loss = (fl["flags"] & 0x08) != 0
            assert np.all(fl["loss_end"][loss] > fl["loss_start"][loss])
            nloss += int((fl["loss_end"][loss] - fl["loss_start"][loss]).sum())
            nooo += int(((fl["flags"] & 0x04) != 0).sum())
            nfwd += m
        lost = sum(pkg.stream_stats(o.api, h, s)[4] for s in range(tr.nstreams))
        assert nloss > 0 and nooo > 0 and nfwd > 0
        assert lost <= nloss  # OOO arrivals refill reported holes
    finally:
        o.destroy(h)
        tr.close()


def test_oracle_speakers_ranked_and_quantised(pkg, workload, abi):
    o = load_oracle()
    tr = workload.Trace(3, duration_s=3.0, rooms=2)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        workload.load_streams(o.api, h, tr)
        seen = 0
        for b in range(tr.nbatches):
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](h, rp, n, ar, alen) == 0
            now = 1700000000 * 10**9 + (b + 1) * 10**9
            sp = pkg.speakers_array(o.api, h, now)
            for room in np.unique(sp["room"]):
                lv = sp["level"][sp["room"] == room]
                assert np.all(np.diff(lv) <= 0)  # descending
                assert np.all(np.abs(lv * 8 - np.round(lv * 8)) < 1e-6)  # multiples of 1/8
            seen += len(sp)
        assert seen > 0
    finally:
        o.destroy(h)
        tr.close()


def test_oracle_nack_rtcp_consistent(pkg, workload, oracle):
    """The oracle's RTCP NACKs (NackQueue.Pairs per datagram): one per datagram
    at most, in datagram order, pairs in range, and the streams' UpdateNack
    totals equal the NACKed sequence numbers of the packets sent."""
    o = oracle
    oh = o.create(500)
    tr = workload.Trace(2, duration_s=2.0, batch_s=0.1, rooms=4, loss=0.08, reorder=0.03, seed=9)
    try:
        workload.load_topology(o.api, oh, tr)
        workload.load_streams(o.api, oh, tr)
        nacked = 0
        pkts = 0
        for b in range(tr.nbatches):
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](oh, rp, n, ar, alen) == 0
            r, p = pkg.nacks_arrays(o.api, oh)
            if len(r):
                assert (np.diff(r["datagram"].astype(np.int64)) > 0).all()
                assert (r["n_pairs"] > 0).all() and (r["num_nacked"] > 0).all()
                assert r["pair_off"][-1] + r["n_pairs"][-1] == len(p)
            nacked += int(r["num_nacked"].sum())
            pkts += len(r)
        assert pkts > 50
        stats = sum(pkg.stream_stats(o.api, oh, s)[13] for s in range(tr.nstreams))
        assert stats == nacked
    finally:
        o.destroy(oh)


def test_oracle_receiver_timing_and_jitter(pkg, workload, abi):
    """RTPStatsReceiver's firstTime / highestTime, gap histogram and receive
    jitter (rtpstats_receiver.go:106-107, :201, :209-213, :237; updateJitter
    rtpstats_base.go:775-810) against an independent Python restatement that
    walks each stream's datagrams with the oracle's flow classification (no
    reference test covers these fields: parity unpinned beyond this
    cross-check and GPU = oracle).  Config 1 has no padding-only datagrams, so
    every handled datagram carries a payload and its flow SN is unadjusted."""
    import struct
    o = load_oracle()
    tr = workload.Trace(1, duration_s=4.0, batch_s=1.0, loss=0.08, reorder=0.05, seed=12)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        workload.load_streams(o.api, h, tr)
        st = {}
        for b in range(tr.nbatches):
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](h, rp, n, ar, alen) == 0
            fl = pkg.flows_array(o.api, h)
            for i in range(n):
                f = int(fl["flags"][i])
                if f & (abi.LKF_FLOW_NOT_HANDLED | abi.LKF_FLOW_BAD):
                    continue
                s = st.setdefault(int(rp[i].stream), dict(first=None, high=None, hsn=None, hts=None, lt=0,
                                                          ljt=0, j=0.0, mj=0.0, gap=[0] * 101))
                t, esn, ets = int(rp[i].arrival_ns), int(fl["ext_sn"][i]), int(fl["ext_ts"][i])
                clock = tr.tracks[tr.streams[int(rp[i].stream)].track].clock_rate
                if s["first"] is None:
                    s["first"] = s["high"] = t
                    pre_ts = (ets - 1) & 0xFFFFFFFF
                    s["hsn"] = esn - 1
                else:
                    pre_ts = s["hts"] & 0xFFFFFFFF
                if esn > s["hsn"]:  # in order
                    g = esn - s["hsn"]
                    if g >= 2:
                        s["gap"][100 if g - 1 > 101 else g - 2] += 1
                    if (ets & 0xFFFFFFFF) != pre_ts:
                        s["high"] = t
                    s["hsn"] = esn
                s["hts"] = ets if s["hts"] is None else max(s["hts"], ets)
                if not f & abi.LKF_FLOW_DUPLICATE and s["ljt"] != ets:  # updateJitter
                    since = (t - s["first"]) & (2**64 - 1)
                    prod = (since * clock) & (2**64 - 1)
                    prod = prod - 2**64 if prod >= 2**63 else prod
                    rtp = ((abs(prod) // 10**9) * (1 if prod >= 0 else -1)) & (2**64 - 1)  # Go's truncating /
                    transit = (rtp - ets) & (2**64 - 1)
                    if s["lt"] != 0:
                        d = (transit - s["lt"]) & (2**64 - 1)
                        d = d - 2**64 if d >= 2**63 else d
                        s["j"] += (float(abs(d)) - s["j"]) / 16
                        s["mj"] = max(s["mj"], s["j"])
                    s["lt"], s["ljt"] = transit, ets
        assert len(st) == tr.nstreams
        jit = 0
        for sid, s in st.items():
            g = abi.lkf_stream_stats()
            assert o.api["stream_stats_get"](h, sid, C.byref(g)) == 0
            assert g.first_time_ns == s["first"] and g.highest_time_ns == s["high"], sid
            assert list(g.gap_histogram) == s["gap"], sid
            assert g.last_transit == s["lt"] and g.last_jitter_ext_ts == s["ljt"], sid
            assert struct.pack("<d", g.jitter) == struct.pack("<d", s["j"]), (sid, g.jitter, s["j"])
            assert struct.pack("<d", g.max_jitter) == struct.pack("<d", s["mj"]), sid
            jit += g.jitter > 0
        assert jit == tr.nstreams
        assert sum(sum(s["gap"]) for s in st.values()) > 0
    finally:
        o.destroy(h)
        tr.close()
