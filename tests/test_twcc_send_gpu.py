"""Send-side transport-wide sequence numbers, engine vs oracle.

With send-side BWE a video subscriber negotiates transport-cc instead of
abs-send-time (pkg/rtc/config.go:119-125) and pion's TWCC header-extension
interceptor (pkg/rtc/transport.go:352-355) stamps every RTP packet its
PeerConnection sends with the next transport-wide sequence number.  The
traces mix abs-send-time and transport-cc subscribers (Trace(twcc=1): every
second subscriber), DownTracks are bound to one transport per (room,
subscriber) with every seventh left unbound (its own counter); forwarded
batches, padding, blank frames and RTX interleave, and the protected output
(SRTP over headers that carry the element, packet by packet) is compared too.  Every record
and wire byte must equal the oracle's.  No reference test covers the
interceptor: parity unpinned beyond the oracle restatement."""
import numpy as np
import pytest

from tests import pad_lib, rtx_lib, srtp_lib
from tests.oracle_lib import load as load_oracle
from tests.test_parity_gpu import check_sender_stats

pytestmark = pytest.mark.gpu
EPOCH = 1700000000 * 10**9


def _tcc_values(tr, rec, ar):
    """(dt, transport-cc sequence number) of every record whose packet carries the element."""
    out = []
    for r in rec:
        d = int(r["dt"])
        tid = int(tr.downtracks[d].ext_transport_cc)
        if not tid:
            continue
        w = ar[int(r["out_off"]):int(r["out_off"]) + int(r["out_len"])]
        h = 12 + 4 * (int(w[0]) & 15)
        prof = (int(w[h]) << 8) | int(w[h + 1])
        q, end = h + 4, h + 4 + 4 * ((int(w[h + 2]) << 8) | int(w[h + 3]))
        while q < end:
            if w[q] == 0:
                q += 1
                continue
            if prof == 0xBEDE:
                eid, ln = int(w[q]) >> 4, (int(w[q]) & 15) + 1
                q += 1
            else:
                eid, ln = int(w[q]), int(w[q + 1])
                q += 2
            if eid == tid:
                out.append((d, (int(w[q]) << 8) | int(w[q + 1])))
                break
            q += ln
    return out


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=8, twcc=1),
                                 dict(config=5, rooms=3, seed=9, twcc=2)])
def test_transport_cc_matches_oracle(pkg, workload, abi, cfg):
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=3.0, batch_s=1.0, **kw)
    o = load_oracle()
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        tg = srtp_lib.bind_transports(pkg, eng.api, eng.h, tr, seed=6)
        to = srtp_lib.bind_transports(pkg, o.api, oh, tr, seed=6)
        assert sorted(tg) == sorted(to)
        stamped = 0
        for b in range(tr.nbatches):
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            dd = tr.batch_dd(b)[0] if tr.has_dd() else None
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            send = EPOCH + b * 10**9 + 123456789
            assert eng.api["protect"](eng.h, send) == 0
            eng.sync()
            o.run(oh, pk, n, ar, alen, dd)
            assert o.api["protect"](oh, send) == 0
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            assert len(grec) == len(orec)
            for f in abi.OUT_DTYPE.names:
                assert np.array_equal(grec[f], orec[f]), (b, f)
            assert np.array_equal(gar, oar), b
            gp, op = pkg.drain_protected(eng.api, eng.h), pkg.drain_protected(o.api, oh)
            assert len(gp) == len(op)
            for i in range(len(orec)):  # every protected packet (the gaps between them are unspecified)
                off = int(orec["out_off"][i]) + 16 * i
                ln = int(orec["out_len"][i]) + (10 if int(orec["dt"][i]) in tg else 0)
                assert np.array_equal(gp[off:off + ln], op[off:off + ln]), (b, i)
            tv = _tcc_values(tr, orec, oar)
            stamped += len(tv)
            now = EPOCH + (b + 1) * 10**9
            if b == 0:  # padding then blank frames between the batches
                reqs = pad_lib.make_reqs(tr.ndts, seed=31, frac=0.4)
                g, r = pad_lib.pad(eng.api, eng.h, reqs, now), pad_lib.pad(o.api, oh, reqs, now)
                assert np.array_equal(g[0], r[0]) and np.array_equal(g[1], r[1])
                stamped += len(_tcc_values(tr, r[0], r[1]))
                reqs = pad_lib.make_reqs(tr.ndts, seed=32, frac=0.4)
                g = pad_lib.pad(eng.api, eng.h, reqs, now, blank=True)
                r = pad_lib.pad(o.api, oh, reqs, now, blank=True)
                assert np.array_equal(g[0], r[0]) and np.array_equal(g[1], r[1])
            if b == 1:  # NACK -> RTX
                nacks = rtx_lib.make_nacks(o.api, oh, tr, seed=33)
                g = rtx_lib.rtx_lookup(eng.api, eng.h, nacks, now)
                r = rtx_lib.rtx_lookup(o.api, oh, nacks, now)
                assert len(g) == len(r) > 10
                idx = rtx_lib.packet_index(tr, b + 1)
                go, gw = rtx_lib.rtx_emit(eng.api, eng.h, tr, g, idx)
                oo, ow = rtx_lib.rtx_emit(o.api, oh, tr, r, idx)
                for f in oo.dtype.names:
                    assert np.array_equal(go[f], oo[f]), f
                assert np.array_equal(gw, ow)
                stamped += len(_tcc_values(tr, oo, ow))
        assert stamped > 500
        check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(tr.ndts))
    finally:
        o.destroy(oh)
        eng.close()


def test_transport_bound_between_runs(pkg, workload, abi):
    """transport-cc DownTracks forward on their own counters
    (no transport at the first run, so no transport counters exist yet), then
    are bound to transports and send padding, blank frames and RTX before the
    next lkf_run: the transports' counters must exist by then (stamped packets
    equal the oracle's) and the next batches continue from them."""
    tr = workload.Trace(2, duration_s=3.0, batch_s=1.0, rooms=2, seed=18, twcc=1)
    o = load_oracle()
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        stamped = 0
        for b in range(tr.nbatches):
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            eng.submit(pk, n, ar, alen)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen)
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            assert np.array_equal(grec, orec) and np.array_equal(gar, oar), b
            stamped += len(_tcc_values(tr, orec, oar))
            if b == 0:  # bind, then padding, blank frames and RTX before the next run
                tg = srtp_lib.bind_transports(pkg, eng.api, eng.h, tr, seed=4)
                to = srtp_lib.bind_transports(pkg, o.api, oh, tr, seed=4)
                assert sorted(tg) == sorted(to)
                now = EPOCH + 10**9
                reqs = pad_lib.make_reqs(tr.ndts, seed=41, frac=0.5)
                g, r = pad_lib.pad(eng.api, eng.h, reqs, now), pad_lib.pad(o.api, oh, reqs, now)
                assert np.array_equal(g[0], r[0]) and np.array_equal(g[1], r[1])
                assert len(_tcc_values(tr, r[0], r[1])) > 0
                reqs = pad_lib.make_reqs(tr.ndts, seed=42, frac=0.5)
                g = pad_lib.pad(eng.api, eng.h, reqs, now, blank=True)
                r = pad_lib.pad(o.api, oh, reqs, now, blank=True)
                assert np.array_equal(g[0], r[0]) and np.array_equal(g[1], r[1])
                nacks = rtx_lib.make_nacks(o.api, oh, tr, seed=43)
                g = rtx_lib.rtx_lookup(eng.api, eng.h, nacks, now)
                r = rtx_lib.rtx_lookup(o.api, oh, nacks, now)
                assert len(g) == len(r) > 5
                idx = rtx_lib.packet_index(tr, 1)
                go, gw = rtx_lib.rtx_emit(eng.api, eng.h, tr, g, idx)
                oo, ow = rtx_lib.rtx_emit(o.api, oh, tr, r, idx)
                for f in oo.dtype.names:
                    assert np.array_equal(go[f], oo[f]), f
                assert np.array_equal(gw, ow)
        assert stamped > 100
        check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(tr.ndts))
        rec = pkg.debug_check(reset=True)  # (a refused device -> host copy counts too)
        assert rec is None or rec[0] == 0, rec
    finally:
        o.destroy(oh)
        eng.close()
