"""DownTrack.rtpStats (buffer.RTPStatsSender) on the CPU oracle — the checker of
the GPU path (sender_kernels.hip).

A second, independent restatement of RTPStatsSender.Update
(rtpstats_sender.go:229-432, rtpStatsBase.updateJitter / updateGapHistogram
rtpstats_base.go:775-813, :871-882) in plain Python is replayed over the
oracle's own forwarded output (every DownTrack's packets in send order: the
munged SN/TS, marker, key-frame flag, the incoming header size and the
forwarded payload length from the wire bytes) and must equal what the oracle
accumulated while forwarding — every counter, the jitter bits and the snInfo
ring.  The reference has no RTPStatsSender test: beyond this cross-check the
restatement is parity unpinned.
"""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle

SN_INFO = 4096
GAP_BINS = 101
M64 = (1 << 64) - 1


def s64(v):
    v &= M64
    return v - (1 << 64) if v >> 63 else v


class PySender:
    """RTPStatsSender.Update, statement by statement (Go uint64/int64 wrap)."""

    def __init__(self, clock_rate):
        self.cr = clock_rate
        self.init = False
        self.first = self.highest_t = 0
        self.start_sn = self.high_sn = self.start_ts = self.high_ts = 0
        self.last_transit = self.last_jts = 0
        self.c = dict(bytes=0, header_bytes=0, bytes_duplicate=0, header_bytes_duplicate=0, bytes_padding=0,
                      header_bytes_padding=0, packets_duplicate=0, packets_padding=0, packets_out_of_order=0,
                      packets_lost=0, frames=0, key_frames=0)
        self.jitter = 0.0
        self.max_jitter = 0.0
        self.gap = [0] * GAP_BINS
        self.ring = [(0, 0, 0)] * SN_INFO

    def _lost(self, esn):
        off = s64(self.high_sn - esn)
        if off >= SN_INFO or off < 0:
            return False
        return self.ring[esn & (SN_INFO - 1)][0] == 0

    def update(self, t, esn, ets, marker, hdr, pay, pad):
        if not self.init:
            if pay == 0:
                return
            self.init = True
            self.first = self.highest_t = t
            self.start_sn, self.high_sn = esn, (esn - 1) & M64
            self.start_ts = self.high_ts = ets
        pkt = hdr + pay + pad
        flags = (1 if marker else 0) | (2 if pay == 0 else 0)
        dup = False
        g = s64(esn - self.high_sn)
        if g <= 0:
            if pay == 0 and esn < self.start_sn:
                return
            if esn < self.start_sn:
                self.c["packets_lost"] += self.start_sn - esn
                self.start_sn = esn
            if g != 0:
                self.c["packets_out_of_order"] += 1
            if not self._lost(esn):
                self.c["bytes_duplicate"] += pkt
                self.c["header_bytes_duplicate"] += hdr
                self.c["packets_duplicate"] += 1
                dup = True
            else:
                self.c["packets_lost"] = (self.c["packets_lost"] - 1) & M64
                self.ring[esn & (SN_INFO - 1)] = (pkt & 0xFFFF, hdr & 0xFF, flags | 4)
        else:
            if g >= 2:
                self.gap[min(g - 1, GAP_BINS) - 1] += 1
            for k in range(min(g - 1, SN_INFO)):
                self.ring[(self.high_sn + 1 + k) & (SN_INFO - 1)] = (0, 0, 0)
            self.c["packets_lost"] += g - 1
            self.ring[esn & (SN_INFO - 1)] = (pkt & 0xFFFF, hdr & 0xFF, flags)
            self.high_sn = esn
        if ets < self.start_ts:
            self.start_ts = ets
        if ets > self.high_ts:
            if pay > 0:
                self.highest_t = t
            self.high_ts = ets
        if not dup:
            if pay == 0:
                self.c["packets_padding"] += 1
                self.c["bytes_padding"] += pkt
                self.c["header_bytes_padding"] += hdr
            else:
                self.c["bytes"] += pkt
                self.c["header_bytes"] += hdr
                if marker:
                    self.c["frames"] += 1
                if self.last_jts != ets:
                    since = s64(t - self.first)
                    prod = s64(since * self.cr)
                    q = abs(prod) // 1000000000
                    rtp = (q if prod >= 0 else -q) & M64  # Go int64 division truncates toward zero
                    transit = (rtp - ets) & M64
                    if self.last_transit != 0:
                        d = abs(s64(transit - self.last_transit))
                        self.jitter += (float(d) - self.jitter) / 16
                        if self.jitter > self.max_jitter:
                            self.max_jitter = self.jitter
                    self.last_transit = transit
                    self.last_jts = ets


def _forward(pkg, workload, o, oh, tr, nb):
    """Forwards nb batches on the oracle; yields (batch pkts, records, wire)."""
    for b in range(nb):
        workload.queue_events(o.api, oh, tr, b)
        pk, n, ar, alen = tr.batch(b)
        o.run(oh, pk, n, ar, alen)
        rec, wire = pkg.drain_arrays(o.api, oh)
        pkts = np.ctypeslib.as_array(C.cast(pk, C.POINTER(C.c_uint8)), shape=(n * 64,)).view(
            np.dtype([("ext_sn", "<u8"), ("ext_ts", "<u8"), ("arrival_ns", "<i8"), ("x", "V12"),
                      ("payload_off", "<u2"), ("payload_len", "<u2"), ("y", "V24")])).copy()
        yield pkts, rec, wire


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=2, seed=21), dict(config=2, rooms=1, seed=22, loss=0.08),
                                 dict(config=5, rooms=3, seed=23)])
def test_sender_stats_restatements_agree(pkg, workload, cfg):
    abi = pkg.abi
    o = load_oracle()
    kw = dict(cfg)
    try:
        tr = workload.Trace(kw.pop("config"), duration_s=3.0, batch_s=1.0, **kw)
    except TypeError:
        pytest.skip("trace option unsupported")
    oh = o.create(500)
    try:
        workload.load_topology(o.api, oh, tr)
        ref = {}
        ooo = 0
        for pkts, rec, wire in _forward(pkg, workload, o, oh, tr, tr.nbatches):
            order = np.lexsort((np.arange(len(rec)), rec["dt"]))  # per DownTrack, send order
            for i in order:
                r = rec[i]
                d = int(r["dt"])
                s = ref.setdefault(d, PySender(int(tr.tracks[tr.downtracks[d].track].clock_rate)))
                w = wire[int(r["out_off"]):int(r["out_off"]) + int(r["out_len"])]
                h = 12 + 4 * (int(w[0]) & 0xF)
                if w[0] & 0x10:
                    h += 4 + 4 * ((int(w[h + 2]) << 8) | int(w[h + 3]))
                p = pkts[int(r["pkt"])]
                before = s.c["packets_out_of_order"]
                s.update(int(p["arrival_ns"]), int(r["ext_sn"]), int(r["ext_ts"]), bool(r["flags"] & abi.LKF_OUT_MARKER),
                         int(p["payload_off"]), int(r["out_len"]) - h, 0)
                if r["flags"] & abi.LKF_OUT_KEYFRAME:
                    s.c["key_frames"] += 1
                ooo += s.c["packets_out_of_order"] - before
        assert ref
        got = pkg.sender_stats(o.api, oh, range(tr.ndts))
        info = C.c_uint32()
        for d in range(tr.ndts):
            g = got[d]
            s = ref.get(d)
            if s is None:
                assert g["initialized"] == 0
                continue
            assert g["initialized"] == 1
            exp = dict(s.c, ext_start_sn=s.start_sn, ext_highest_sn=s.high_sn, ext_start_ts=s.start_ts,
                       ext_highest_ts=s.high_ts, first_time_ns=s.first, highest_time_ns=s.highest_t,
                       last_transit=s.last_transit, last_jitter_ext_ts=s.last_jts)
            for k, v in exp.items():
                assert int(g[k]) == v, (d, k, int(g[k]), v)
            assert np.float64(g["jitter"]).tobytes() == np.float64(s.jitter).tobytes(), (d, g["jitter"], s.jitter)
            assert np.float64(g["max_jitter"]).tobytes() == np.float64(s.max_jitter).tobytes()
            assert list(g["gap_histogram"]) == s.gap, d
            for esn in range(s.high_sn - 120, s.high_sn + 1):
                assert o.api["sender_sninfo"](oh, d, esn, C.byref(info)) == 0
                pk, hd, fl = s.ring[esn & (SN_INFO - 1)]
                assert info.value == pk | (hd << 16) | (fl << 24), (d, esn)
        if cfg["config"] == 2:
            assert ooo > 0  # reordered packets forwarded out of order reach the duplicate/OOO branch
            assert sum(sum(s.gap) for s in ref.values()) > 0
    finally:
        o.destroy(oh)
        tr.close()
