"""Drop-in boundary calls mid-trace, engine vs oracle:

* state export / import on transceiver reuse: MediaTrackSubscriptions
  (mediatracksubscriptions.go:159-167) reads the old DownTrack's
  DownTrackState and seeds the new one's Forwarder (forwarder.go:340-375,
  rtpmunger.go:115-133, codecmunger/vp8.go:87-109) — here lkf_get_state,
  lkf_remove_downtrack, lkf_add_downtrack, lkf_seed_state between batches;
* lkf_remove_downtrack of live DownTracks between batches;
* lkf_remove_track (WebRTCReceiver.closeTracks + Buffer.Close) on the raw
  ingest path: the closed streams' datagrams are not processed, the track's
  DownTracks stop, its microphone leaves the speaker ranking.

Every output record, wire byte, counter, flow, RTCP NACK, speaker list and
exported Forwarder state must be identical."""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle
from tests.test_parity_gpu import check_sender_stats
from tests.test_ingress_gpu import check_nacks

pytestmark = pytest.mark.gpu

EPOCH = 1700000000 * 10**9


def _compare_batch(pkg, abi, eng, o, oh, b):
    gs = eng.stats()
    ost = abi.lkf_stats()
    o.api["get_stats"](oh, C.byref(ost))
    assert gs == ost.as_dict(), (b, gs, ost.as_dict())
    grec, gar = eng.drain()
    orec, oar = pkg.drain_arrays(o.api, oh)
    assert len(grec) == len(orec), (b, len(grec), len(orec))
    for f in abi.OUT_DTYPE.names:
        assert np.array_equal(grec[f], orec[f]), (b, f)
    assert np.array_equal(gar, oar), b
    return len(grec)


def _states(abi, api, h, ndts):
    out = []
    for dt in range(ndts):
        s = abi.lkf_fwd_state()
        assert api["get_state"](h, dt, C.byref(s)) == 0
        out.append(s.as_tuple())
    return out


def _reuse(abi, trace, api, h, dts, n0, orig):
    """Transceiver reuse of each DownTrack in dts: export, remove, add a new
    DownTrack with the same parameters (handle n0 + i; orig maps a handle to
    its trace DownTrack), seed it, give the video ones an allocation at the
    batch start.  Returns the exported states."""
    states = []
    for i, d in enumerate(dts):
        s = abi.lkf_fwd_state()
        assert api["get_state"](h, d, C.byref(s)) == 0
        states.append(s.as_tuple())
        assert api["remove_downtrack"](h, d) == 0
        p = trace.downtracks[orig[d]]
        nh = api["add_downtrack"](h, C.byref(p))
        assert nh == n0 + i, (nh, n0 + i)
        assert api["seed_state"](h, nh, C.byref(s)) == 0
        assert api["sender_stats_seed"](h, nh, d) == 0  # DownTrack.SeedState: rtpStats.Seed (downtrack.go:1051-1055)
        if trace.tracks[p.track].kind == abi.LKF_KIND_VIDEO:
            assert api["ctl"](h, nh, abi.LKF_CTL_SET_ALLOCATION, 2, 2, 2, 0, 0) == 0
    return states


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=11), dict(config=5, rooms=4, svc_dd=0, seed=12),
                                 dict(config=5, rooms=4, svc_dd=1, seed=13)])
def test_state_roundtrip_transceiver_reuse(pkg, workload, abi, cfg):
    o = load_oracle()
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=5.0, batch_s=1.0, **kw)
    eng = pkg.Engine.for_trace(tr, extra_dts=tr.ndts)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        n = tr.ndts
        orig = {d: d for d in range(n)}
        reused = list(range(1, n, 5))
        seeded = 0
        for b in range(tr.nbatches):
            if b in (2, 4):  # between batches, on both sides
                gst = _reuse(abi, tr, eng.api, eng.h, reused, n, orig)
                ost = _reuse(abi, tr, o.api, oh, reused, n, orig)
                assert gst == ost, b  # the exported states agree (bit-exact)
                seeded += sum(1 for s in gst if s[0])
                for i, d in enumerate(reused):
                    orig[n + i] = orig[d]
                reused = list(range(n, n + len(reused)))  # the next reuse takes the new DownTracks
                n += len(gst)
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, npk, ar, alen = tr.batch(b)
            dd = tr.batch_dd(b)[0] if tr.has_dd() else None
            eng.submit(pk, npk, ar, alen, dd)
            eng.run()
            eng.sync()
            o.run(oh, pk, npk, ar, alen, dd)
            _compare_batch(pkg, abi, eng, o, oh, b)
        assert seeded > 0
        assert _states(abi, eng.api, eng.h, n) == _states(abi, o.api, oh, n)
        gsum, osum = pkg.downtrack_summaries(eng.api, eng.h), pkg.downtrack_summaries(o.api, oh)
        for f in abi.DT_SUMMARY_DTYPE.names:
            assert np.array_equal(gsum[f], osum[f]), f
        ss = check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(n))
        assert int(ss["initialized"][tr.ndts:].sum()) > 0  # seeded statistics carried on
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


def test_seed_state_started_roundtrip(pkg, workload, abi):
    """A state seeded into a fresh DownTrack reads back identically (and a
    not-started state seeds nothing, forwarder.go:360-362)."""
    o = load_oracle()
    tr = workload.Trace(2, duration_s=2.0, batch_s=1.0, rooms=2, seed=17)
    eng = pkg.Engine.for_trace(tr, extra_dts=tr.ndts)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        workload.queue_events(eng.api, eng.h, tr, 0)
        pk, npk, ar, alen = tr.batch(0)
        eng.submit(pk, npk, ar, alen)
        eng.run()
        eng.sync()
        for d in range(0, tr.ndts, 3):
            s = abi.lkf_fwd_state()
            assert eng.api["get_state"](eng.h, d, C.byref(s)) == 0
            nh = eng.api["add_downtrack"](eng.h, C.byref(tr.downtracks[d]))
            assert eng.api["seed_state"](eng.h, nh, C.byref(s)) == 0
            t = abi.lkf_fwd_state()
            assert eng.api["get_state"](eng.h, nh, C.byref(t)) == 0
            assert t.as_tuple() == s.as_tuple(), d
            # the oracle agrees on the seeded state too
            oh_h = o.api["add_downtrack"](oh, C.byref(tr.downtracks[d]))
            assert oh_h == nh
            assert o.api["seed_state"](oh, oh_h, C.byref(s)) == 0
            u = abi.lkf_fwd_state()
            assert o.api["get_state"](oh, oh_h, C.byref(u)) == 0
            assert u.as_tuple() == s.as_tuple(), d
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=19), dict(config=4, participants=200, rooms=1)])
def test_remove_downtrack_mid_trace(pkg, workload, abi, cfg):
    o = load_oracle()
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=4.0, batch_s=0.5, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        rng = np.random.default_rng(5)
        removed = set()
        for b in range(tr.nbatches):
            if b in (2, 5):
                for d in rng.choice(tr.ndts, size=max(1, tr.ndts // 6), replace=False):
                    assert eng.api["remove_downtrack"](eng.h, int(d)) == 0
                    assert o.api["remove_downtrack"](oh, int(d)) == 0
                    removed.add(int(d))
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, npk, ar, alen = tr.batch(b)
            eng.submit(pk, npk, ar, alen)
            eng.run()
            eng.sync()
            o.run(oh, pk, npk, ar, alen)
            grec, _ = eng.drain()
            if b >= 5:
                assert not (set(grec["dt"].tolist()) & removed), b
            # (compare after the check: _compare_batch drains again)
            _compare_batch(pkg, abi, eng, o, oh, b)
        assert _states(abi, eng.api, eng.h, tr.ndts) == _states(abi, o.api, oh, tr.ndts)
        gsum, osum = pkg.downtrack_summaries(eng.api, eng.h), pkg.downtrack_summaries(o.api, oh)
        for f in abi.DT_SUMMARY_DTYPE.names:
            assert np.array_equal(gsum[f], osum[f]), f
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


def test_remove_track_ingest(pkg, workload, abi):
    """lkf_remove_track between raw ingests: a video track and a microphone
    track of one room close (flows NOT_HANDLED, no NACKs, no output for their
    DownTracks, the microphone leaves the speaker list)."""
    o = load_oracle()
    tr = workload.Trace(2, duration_s=3.0, batch_s=0.5, rooms=3, loss=0.05, reorder=0.03, seed=23)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        for api, h in ((eng.api, eng.h), (o.api, oh)):
            workload.load_topology(api, h, tr)
            workload.load_streams(api, h, tr)
        video = next(t for t in range(tr.ntracks) if tr.tracks[t].kind == abi.LKF_KIND_VIDEO)
        mic = next(t for t in range(tr.ntracks) if tr.tracks[t].is_mic)
        gone = set()
        for b in range(tr.nbatches):
            if b == 2:
                for t in (video, mic):
                    assert eng.api["remove_track"](eng.h, t) == 0
                    assert o.api["remove_track"](oh, t) == 0
                    gone.add(t)
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            rp, n, ar, alen = tr.batch_raw(b)
            eng.ingest(rp, n, ar, alen)
            assert o.api["ingest"](oh, rp, n, ar, alen) == 0
            gf, of = eng.flows(), pkg.flows_array(o.api, oh)
            for f in ("ext_sn", "ext_ts", "loss_start", "loss_end", "pkt", "flags"):
                assert np.array_equal(gf[f], of[f]), (b, f)
            check_nacks(pkg, eng, o, oh, b)
            n_in = C.c_uint32()
            assert o.api["ingested"](oh, None, 0, C.byref(n_in)) in (0, -28)
            buf = (abi.lkf_pkt * max(1, n_in.value))()
            assert o.api["ingested"](oh, buf, n_in.value, C.byref(n_in)) == 0
            eng.run()
            eng.sync()
            o.run(oh, C.cast(buf, C.POINTER(abi.lkf_pkt)) if n_in.value else None, n_in.value, ar, alen)
            _compare_batch(pkg, abi, eng, o, oh, b)
            now = EPOCH + (b + 1) * 10**9
            gsp, osp = eng.speakers(now), pkg.speakers_array(o.api, oh, now)
            assert len(gsp) == len(osp), b
            for f in ("room", "participant", "level", "active"):
                assert np.array_equal(gsp[f], osp[f]), (b, f)
        for s in range(tr.nstreams):
            assert eng.stream_stats(s) == pkg.stream_stats(o.api, oh, s), s
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()
