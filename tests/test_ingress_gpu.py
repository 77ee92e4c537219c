"""Bit-exact parity of the GPU ingress path and speaker ranking vs the CPU oracle.

Raw datagrams (with loss, reordering, audio-level extensions, VP8 payloads)
go through lkf_ingest (Buffer.calc on the GPU) and orc_ingest (the oracle's
restatement); the per-datagram flow records, the ExtPacket batches produced,
the TWCC responder pushes (processHeaderExtensions), the forwarded output of
that batch, every stream's RTPStatsReceiver counters
and the per-room active-speaker lists must be identical.
"""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle

pytestmark = pytest.mark.gpu

EPOCH = 1700000000 * 10**9


def _ingested(api, h, abi):
    n = C.c_uint32()
    rc = api["ingested"](h, None, 0, C.byref(n))
    assert rc in (0, -28)
    arr = (abi.lkf_pkt * max(1, n.value))()
    assert api["ingested"](h, arr, n.value, C.byref(n)) == 0
    return C.string_at(arr, 64 * n.value) if n.value else b""


def _ingested_dd(api, h, abi):
    n = C.c_uint32()
    rc = api["ingested_dd"](h, None, 0, C.byref(n))
    assert rc in (0, -28)
    sz = C.sizeof(abi.lkf_pkt_dd)
    buf = C.create_string_buffer(max(1, n.value) * sz)
    assert api["ingested_dd"](h, buf, n.value, C.byref(n)) == 0
    return buf.raw[: sz * n.value]


def check_nacks(pkg, eng, o, oh, b):
    """The batch's RTCP NACKs (Buffer.doNACKs per datagram) must be identical."""
    gr, gp = pkg.nacks_arrays(eng.api, eng.h)
    orr, op = pkg.nacks_arrays(o.api, oh)
    assert len(gr) == len(orr), (b, len(gr), len(orr))
    for f in abi_fields(gr):
        if not np.array_equal(gr[f], orr[f]):
            bad = np.nonzero(gr[f] != orr[f])[0][:5]
            raise AssertionError("batch %d NACK field %s differs at %s: gpu %s orc %s" % (b, f, bad, gr[bad], orr[bad]))
    assert np.array_equal(gp, op), b
    return len(gr), int(gr["num_nacked"].sum()) if len(gr) else 0


def abi_fields(a):
    return [f for f in a.dtype.names if f != "reserved"]


def run_ingress_parity(pkg, workload, abi, trace, speakers=True, rtt_changes=None):
    """rtt_changes: {batch: [(stream, rtt_ms), ...]} applied (Buffer.SetRTT)
    before that batch's ingest on both sides."""
    o = load_oracle()
    eng = pkg.Engine.for_trace(trace)
    oh = o.create(500)
    try:
        for api, h in ((eng.api, eng.h), (o.api, oh)):
            workload.load_topology(api, h, trace)
            workload.load_streams(api, h, trace)
        total_fwd = 0
        nack_pkts = 0
        twcc_pushes = 0
        for b in range(trace.nbatches):
            for sid, rtt in (rtt_changes or {}).get(b, []):
                assert eng.api["stream_set_rtt"](eng.h, sid, rtt) == 0
                assert o.api["stream_set_rtt"](oh, sid, rtt) == 0
            workload.queue_events(eng.api, eng.h, trace, b)
            workload.queue_events(o.api, oh, trace, b)
            rp, n, ar, alen = trace.batch_raw(b)
            eng.ingest(rp, n, ar, alen)
            assert o.api["ingest"](oh, rp, n, ar, alen) == 0
            nack_pkts += check_nacks(pkg, eng, o, oh, b)[0]
            gf = eng.flows()
            of = pkg.flows_array(o.api, oh)
            assert len(gf) == len(of) == n
            for f in ("ext_sn", "ext_ts", "loss_start", "loss_end", "pkt", "flags"):
                if not np.array_equal(gf[f], of[f]):
                    bad = np.nonzero(gf[f] != of[f])[0][:5]
                    raise AssertionError("batch %d flow field %s differs at %s: gpu %s orc %s" % (
                        b, f, bad, gf[bad], of[bad]))
            gt, ot = pkg.twcc_words(eng.api, eng.h), pkg.twcc_words(o.api, oh)
            assert len(gt) == len(ot) == n
            if not np.array_equal(gt, ot):
                bad = np.nonzero(gt != ot)[0][:5]
                raise AssertionError("batch %d TWCC pushes differ at %s: gpu %s orc %s" % (b, bad, gt[bad], ot[bad]))
            twcc_pushes += int(np.count_nonzero(gt & abi.LKF_TWCC_PUSH))
            gp = _ingested(eng.api, eng.h, abi)
            op = _ingested(o.api, oh, abi)
            if gp != op:
                g = np.frombuffer(gp, np.uint8).reshape(-1, 64)
                o_ = np.frombuffer(op, np.uint8).reshape(-1, 64)
                bad = np.nonzero((g != o_).any(1))[0] if len(g) == len(o_) else []
                raise AssertionError("batch %d ExtPacket batches differ (%d vs %d) first rows %s" % (
                    b, len(g), len(o_), list(bad[:5])))
            gd = _ingested_dd(eng.api, eng.h, abi)
            od = _ingested_dd(o.api, oh, abi)
            assert gd == od, "batch %d ExtPacket dependency descriptors differ" % b
            # forward the ingested batch on both sides
            eng.run()
            eng.sync()
            m = len(op) // 64
            if m:
                o.run(oh, C.cast(C.c_char_p(op), C.POINTER(abi.lkf_pkt)), m, ar, alen)
            else:
                o.run(oh, None, 0, ar, alen)
            gs = eng.stats()
            ost = abi.lkf_stats()
            o.api["get_stats"](oh, C.byref(ost))
            assert gs == ost.as_dict(), (b, gs, ost.as_dict())
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            assert len(grec) == len(orec)
            for f in abi.OUT_DTYPE.names:
                assert np.array_equal(grec[f], orec[f]), (b, f)
            assert np.array_equal(gar, oar), b
            total_fwd += gs["forwarded"]
            if speakers:
                now = EPOCH + (b + 1) * 10**9
                gsp = eng.speakers(now)
                osp = pkg.speakers_array(o.api, oh, now)
                assert len(gsp) == len(osp), (b, len(gsp), len(osp))
                for f in ("room", "participant", "level", "active"):
                    assert np.array_equal(gsp[f], osp[f]), (b, f, gsp, osp)
        for s in range(trace.nstreams):
            assert eng.stream_stats(s) == pkg.stream_stats(o.api, oh, s), s
        run_ingress_parity.nack_pkts = nack_pkts
        run_ingress_parity.twcc_pushes = twcc_pushes
        return total_fwd
    finally:
        eng.close()
        o.destroy(oh)


def test_ingress_config2_loss_reorder(pkg, workload, abi):
    tr = workload.Trace(2, duration_s=3.0, batch_s=0.5, rooms=3, loss=0.05, reorder=0.03, seed=21)
    assert run_ingress_parity(pkg, workload, abi, tr) > 0
    assert run_ingress_parity.twcc_pushes > 1000  # every video datagram carries transport-cc


def test_ingress_config5_vp9(pkg, workload, abi):
    """VP9 SVC datagrams: VP9 descriptor parse, key frames, SID dispatch, then forwarding."""
    tr = workload.Trace(5, duration_s=3.0, batch_s=0.5, rooms=4, loss=0.05, reorder=0.03, seed=31, svc_dd=0)
    assert run_ingress_parity(pkg, workload, abi, tr) > 0


def test_ingress_config5_dd(pkg, workload, abi):
    """AV1 and VP9 publishers with dependency descriptors: the per-stream
    DependencyDescriptorParser (structures, frame-number wrap, frame integrity,
    active decode targets) on the GPU, then the DD selector on its output."""
    tr = workload.Trace(5, duration_s=3.0, batch_s=0.5, rooms=4, seed=41)
    assert tr.has_dd()
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False) > 0


def test_ingress_config5_dd_loss_reorder(pkg, workload, abi):
    tr = workload.Trace(5, duration_s=3.0, batch_s=0.25, rooms=3, loss=0.06, reorder=0.04, seed=43)
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False) > 0


def test_ingress_config5_dd_wide(pkg, workload, abi):
    """The wide descriptor (9 chains, 17-18 frame diffs) through the stream
    parser and then the selector (tests/test_dd_wide_cpu.py)."""
    tr = workload.Trace(5, duration_s=3.0, batch_s=0.5, rooms=4, loss=0.04, reorder=0.03, seed=63, svc_dd=2)
    assert tr.has_dd()
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False) > 0


def test_ingress_config5_dd_burst(pkg, workload, abi):
    """The burst workload (svc_dd = 3: chains waiting on dozens of frames)
    through the stream parser and then the selector."""
    tr = workload.Trace(5, duration_s=4.0, batch_s=0.5, rooms=4, seed=94, svc_dd=3)
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False) > 0


def test_ingress_h264_keyframes(pkg, workload, abi):
    """H.264 simulcast publishers: IsH264KeyFrame over single NALU / STAP-A /
    STAP-B / FU-A SPS packets (and truncated aggregates) on the GPU."""
    tr = workload.Trace(2, duration_s=3.0, batch_s=0.5, rooms=3, loss=0.04, reorder=0.03, seed=47, h264=1)
    assert run_ingress_parity(pkg, workload, abi, tr) > 0


def test_ingress_config1(pkg, workload, abi):
    tr = workload.Trace(1, duration_s=3.0, batch_s=1.0)
    assert run_ingress_parity(pkg, workload, abi, tr) > 0


def test_ingress_config3_speakers(pkg, workload, abi):
    """configs[2] shape: 50-participant audio-heavy rooms, speaker ranking every batch (400 ms)."""
    tr = workload.Trace(3, duration_s=4.0, batch_s=0.4, rooms=2)
    assert run_ingress_parity(pkg, workload, abi, tr) > 0


def test_ingress_nack_config2_full(pkg, workload, abi):
    """configs[1] at its benched size (100 rooms x 10 participants, 2 % loss,
    1 % reorder) through 100-ms ingest ticks: every Buffer's NackQueue
    (Remove on arrival, Push of loss ranges, Pairs with the RTT backoff and
    five tries) on the GPU, the RTCP NACK of every datagram and its pairs
    identical to the oracle's; RTTs change mid-trace (Buffer.SetRTT)."""
    tr = workload.Trace(2, duration_s=2.0, batch_s=0.1, rooms=100)
    rtt = {5: [(s, 20 + (7 * s) % 200) for s in range(0, tr.nstreams, 3)],
           12: [(s, 0) for s in range(0, tr.nstreams, 5)] + [(1, 400)]}
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False, rtt_changes=rtt) > 0
    assert run_ingress_parity.nack_pkts > 1000


def test_ingress_nack_heavy_loss(pkg, workload, abi):
    """Loss bursts and deep reordering: queues at CacheSize, purges after the
    fifth try, removals of NACKed SNs that arrive late."""
    tr = workload.Trace(2, duration_s=3.0, batch_s=0.05, rooms=4, loss=0.25, reorder=0.1, seed=77)
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False) > 0
    assert run_ingress_parity.nack_pkts > 100


@pytest.mark.parametrize("loss,reorder,batch_s,seed", [(0.02, 0.01, 1.0, 5), (0.06, 0.04, 1.0, 6), (0.3, 0.1, 1.0, 7),
                                                       (0.05, 0.03, 0.01, 8)])
def test_ingress_nack_lane_parallel(pkg, workload, abi, loss, reorder, batch_s, seed):
    """Round 6: k_ing_nack decides each queue entry's nacks on a lane of its
    own where that is exact (no capacity eviction possible, distinct SNs,
    arrivals in order) and falls back to the serial form per stream
    otherwise.  1-s ingests as the bench runs them (the lane-parallel form on
    nearly every stream), heavy loss (queues reach CacheSize: the serial form
    on many streams, both forms in one launch), and 10-ms ticks; every RTCP
    NACK, its pairs and the per-stream receiver statistics (nacks included)
    equal the oracle's."""
    tr = workload.Trace(2, duration_s=4.0 if batch_s >= 1.0 else 0.6, batch_s=batch_s, rooms=12, loss=loss,
                        reorder=reorder, seed=seed)
    rtt = {1: [(s, 30 + (11 * s) % 300) for s in range(0, tr.nstreams, 2)]}
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False, rtt_changes=rtt) > 0
    assert run_ingress_parity.nack_pkts > 10


def test_ingress_config3_bench_size(pkg, workload, abi):
    """configs[2] at the per-GPU size bench.py runs (125 rooms x 50
    participants, 6,875 streams, ~16 M tuples per 1-s batch): raw datagrams
    through Buffer.calc (stream kernel, buckets, NACK queues) and the
    forwarding, the speaker ranking after every batch, and every stream's
    RTPStatsReceiver — counters, timing, gap histogram and jitter — equal to
    the oracle's."""
    tr = workload.Trace(3, duration_s=2.0, batch_s=1.0, rooms=125)
    assert run_ingress_parity(pkg, workload, abi, tr) > 0


def test_ingress_config5_dd_heavy_loss_small_batches(pkg, workload, abi):
    """DD streams through the run path under heavy loss and deep reordering
    with 50-ms ingests: runs cut by reorders, descriptors that attach a
    structure (key frames) at any lane of a chunk, lost first / last packets
    of frames (frame integrity), all against the oracle's serial parser."""
    tr = workload.Trace(5, duration_s=3.0, batch_s=0.05, rooms=4, loss=0.2, reorder=0.1, seed=59)
    assert tr.has_dd()
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False) > 0


def test_ingress_config5_bench_size(pkg, workload, abi):
    """configs[4] at the per-GPU size bench.py runs (2,000 rooms x 5
    participants, VP9/AV1 L3T3 with dependency descriptors): raw datagrams
    through Buffer.calc with the DD parser in the stream wave's runs, then the
    SVC / DD forwarding, identical to the oracle."""
    tr = workload.Trace(5, duration_s=2.0, batch_s=1.0, rooms=2000)
    assert tr.has_dd()
    assert run_ingress_parity(pkg, workload, abi, tr, speakers=False) > 0


def test_empty_ingest_after_ingest(pkg, workload, abi):
    """an empty ingest after a full one produces an empty
    ExtPacket batch (lkf_ingested returns 0 records), forwards nothing, and
    the next full ingest continues as the oracle does; a second host ingest
    into the same batch context before lkf_run (its datagram copies overwrite
    what the first one's NACK queues and bucket copies read) leaves the
    receivers' state equal to the oracle's."""
    trace = workload.Trace(2, duration_s=3.0, batch_s=1.0, rooms=2, seed=23)
    o = load_oracle()
    eng = pkg.Engine.for_trace(trace)
    oh = o.create(500)
    try:
        for api, h in ((eng.api, eng.h), (o.api, oh)):
            workload.load_topology(api, h, trace)
            workload.load_streams(api, h, trace)
        for b in range(trace.nbatches):
            workload.queue_events(eng.api, eng.h, trace, b)
            workload.queue_events(o.api, oh, trace, b)
            rp, n, ar, alen = trace.batch_raw(b)
            if b == 1:  # a full ingest, then (same context, no run) another full ingest
                eng.ingest(rp, n // 2, ar, alen)
                assert o.api["ingest"](oh, rp, n // 2, ar, alen) == 0
                eng.ingest(C.cast(C.cast(rp, C.c_void_p).value + (n // 2) * C.sizeof(abi.lkf_raw_pkt),
                                  C.POINTER(abi.lkf_raw_pkt)), n - n // 2, ar, alen)
                assert o.api["ingest"](oh, C.cast(C.cast(rp, C.c_void_p).value + (n // 2) *
                                                  C.sizeof(abi.lkf_raw_pkt), C.POINTER(abi.lkf_raw_pkt)),
                                       n - n // 2, ar, alen) == 0
            else:
                eng.ingest(rp, n, ar, alen)
                assert o.api["ingest"](oh, rp, n, ar, alen) == 0
            gp, op = _ingested(eng.api, eng.h, abi), _ingested(o.api, oh, abi)
            assert gp == op and len(gp) > 0, b
            if b == 0:  # an empty ingest replaces the batch: nothing to forward
                eng.ingest(rp, 0, ar, 0)
                assert o.api["ingest"](oh, rp, 0, ar, 0) == 0
                assert _ingested(eng.api, eng.h, abi) == b"" == _ingested(o.api, oh, abi)
                op = b""
            eng.run()
            eng.sync()
            m = len(op) // 64
            if m:
                o.run(oh, C.cast(C.c_char_p(op), C.POINTER(abi.lkf_pkt)), m, ar, alen)
            else:
                o.run(oh, None, 0, ar, alen)
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            assert np.array_equal(grec, orec) and np.array_equal(gar, oar), b
            if b == 0:
                assert len(grec) == 0
        for s in range(trace.nstreams):
            assert eng.stream_stats(s) == pkg.stream_stats(o.api, oh, s), s
    finally:
        eng.close()
        o.destroy(oh)
