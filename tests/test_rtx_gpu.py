"""NACK -> RTX parity, engine vs oracle (lkf_rtx_lookup + lkf_rtx_emit).

After forwarding the same batches on both, the same NACK lists (hundreds of
DownTracks, repeats, out-of-window SNs, deficient DownTracks) must give the
same sequencer records — then the same records again with their NACK counts
advanced — and the same retransmitted wire packets, byte for byte."""
import numpy as np
import pytest

from tests import rtx_lib
from tests.oracle_lib import load as load_oracle
from tests.test_parity_gpu import check_sender_stats

pytestmark = pytest.mark.gpu
EPOCH = 1700000000 * 10**9


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=4, seed=9), dict(config=1, seed=4), dict(config=3, rooms=2),
                                 dict(config=5, rooms=4, svc_dd=1, seed=14)])
def test_rtx_lookup_and_emit_match_oracle(pkg, workload, cfg):
    o = load_oracle()
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=3.0, batch_s=1.0, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    nb = 3
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        for b in range(nb):
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            dd = tr.batch_dd(b)[0] if tr.has_dd() else None
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen, dd)
        idx = rtx_lib.packet_index(tr, nb)
        nacks = rtx_lib.make_nacks(o.api, oh, tr, seed=5)
        assert len(nacks) > 50
        for step, dt_ns in enumerate((500 * 10**6, 1500 * 10**6, 1510 * 10**6, 3 * 10**9, 4 * 10**9)):
            now = EPOCH + nb * 10**9 + dt_ns
            g = rtx_lib.rtx_lookup(eng.api, eng.h, nacks, now)
            r = rtx_lib.rtx_lookup(o.api, oh, nacks, now)
            assert len(g) == len(r), (step, len(g), len(r))
            for f in r.dtype.names:
                assert np.array_equal(g[f], r[f]), (step, f)
            if step == 0:
                assert len(r) > 20
                go, gw = rtx_lib.rtx_emit(eng.api, eng.h, tr, g, idx)
                oo, ow = rtx_lib.rtx_emit(o.api, oh, tr, r, idx)
                assert len(go) == len(oo) > 0
                for f in oo.dtype.names:
                    assert np.array_equal(go[f], oo[f]), f
                assert np.array_equal(gw, ow)
                if tr.has_dd():  # RTX of a DD DownTrack carries the sequencer's ddBytes (downtrack.go:1684)
                    assert rtx_lib.count_dd_elements(tr, oo, ow) > 0
                # RTPStatsSender.Update of the retransmissions (duplicates / out of order)
                ss = check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(tr.ndts))
                assert int(ss["packets_duplicate"].sum()) > 0
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


def test_rtx_lookup_rejects_split_lists(pkg, workload):
    tr = workload.Trace(1, duration_s=1.0, batch_s=1.0)
    eng = pkg.Engine.for_trace(tr)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        nacks = np.array([(0, 1, 0), (1, 2, 0), (0, 3, 0)], dtype=pkg.abi.NACK_DTYPE)
        out = np.zeros(3, dtype=pkg.abi.RTX_DTYPE)
        import ctypes as C
        k = C.c_uint32()
        rc = eng.api["rtx_lookup"](eng.h, nacks.ctypes.data, 3, 0, out.ctypes.data, 3, C.byref(k))
        assert rc == -34  # LKF_EORDER: DownTrack 0's NACKs are split
    finally:
        eng.close()
        tr.close()


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=11, loss=0.02, reorder=0.01),
                                 dict(config=5, rooms=3, svc_dd=1, seed=15)])
def test_rtx_from_bucket_matches_oracle(pkg, workload, abi, cfg):
    """Raw datagrams ingested on both sides fill the receivers' buckets (the
    GPU's in HBM: k_bkt_add / k_bkt_store); the retransmissions read from them
    (lkf_rtx_emit_bucket: k_bkt_read + k_rtx) must equal the oracle's bucket
    restatement's, records and wire bytes."""
    import ctypes as C
    o = load_oracle()
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=3.0, batch_s=1.0, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    nb = 3
    try:
        for api, h in ((eng.api, eng.h), (o.api, oh)):
            workload.load_topology(api, h, tr)
            workload.load_streams(api, h, tr)

        def run_eng(b, pk, n, ar, alen):
            eng.run()
            eng.sync()

        def run_orc(b, pk, n, ar, alen):  # (the ingest's DD side array stays with the oracle, as in test_ingress_gpu)
            o.run(oh, pk if n else None, n, ar, alen)

        for b in range(nb):  # interleaved: the engine's ingest feeds its next run
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            rp, n, ar, alen = tr.batch_raw(b)
            eng.ingest(rp, n, ar, alen)
            assert o.api["ingest"](oh, rp, n, ar, alen) == 0
            assert np.array_equal(eng.flows()["flags"], pkg.flows_array(o.api, oh)["flags"]), b
            k = C.c_uint32()
            assert o.api["ingested"](oh, None, 0, C.byref(k)) in (0, -28)
            arr = (abi.lkf_pkt * max(1, k.value))()
            assert o.api["ingested"](oh, arr, k.value, C.byref(k)) == 0
            run_eng(b, None, 0, ar, alen)
            run_orc(b, arr, k.value, ar, alen)
        nacks = rtx_lib.make_nacks(o.api, oh, tr, seed=7)
        now = EPOCH + nb * 10**9 + 5 * 10**8
        g = rtx_lib.rtx_lookup(eng.api, eng.h, nacks, now)
        r = rtx_lib.rtx_lookup(o.api, oh, nacks, now)
        assert len(g) == len(r) > 20
        go, gw = rtx_lib.rtx_emit_bucket(eng.api, eng.h, g)
        oo, ow = rtx_lib.rtx_emit_bucket(o.api, oh, r)
        assert len(go) == len(oo) > 10, (len(go), len(oo))
        for f in oo.dtype.names:
            assert np.array_equal(go[f], oo[f]), f
        assert np.array_equal(gw, ow)
        check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(tr.ndts))
    finally:
        o.destroy(oh)
        eng.close()


def test_bucket_too_old_and_wrap_match_oracle(pkg, workload, abi):
    """The bucket edge cases on the GPU (k_bkt_add / k_bkt_store) against the
    oracle: a 5-s batch wraps the audio rings inside the batch (the earlier
    writer of a reused slot is not stored), and two datagrams arrive later
    than their bucket's window (too old: no ExtPacket).  Flows, ExtPackets and
    the retransmissions read back from the buckets must be identical."""
    import ctypes as C
    from tests import bucket_lib
    o = load_oracle()
    tr = workload.Trace(2, duration_s=5.0, batch_s=5.0, rooms=2, seed=3, loss=0.0, reorder=0.0)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        for api, h in ((eng.api, eng.h), (o.api, oh)):
            workload.load_topology(api, h, tr)
            workload.load_streams(api, h, tr)
        workload.queue_events(eng.api, eng.h, tr, 0)
        workload.queue_events(o.api, oh, tr, 0)
        arr, n, ar, alen, moved = bucket_lib.late_batch(tr)
        assert len(moved) == 2
        eng.ingest(arr, n, ar, alen)
        assert o.api["ingest"](oh, arr, n, ar, alen) == 0
        gf, of = eng.flows(), pkg.flows_array(o.api, oh)
        for f in ("ext_sn", "ext_ts", "pkt", "flags"):
            assert np.array_equal(gf[f], of[f]), f
        late = (of["flags"] & abi.LKF_FLOW_OUT_OF_ORDER) != 0
        ok = (of["flags"] & (abi.LKF_FLOW_BUCKET | abi.LKF_FLOW_DUPLICATE | abi.LKF_FLOW_PADDING)) == 0
        assert int(np.count_nonzero(late & ok)) == 2
        k = C.c_uint32()
        assert o.api["ingested"](oh, None, 0, C.byref(k)) in (0, -28)
        pk = (abi.lkf_pkt * max(1, k.value))()
        assert o.api["ingested"](oh, pk, k.value, C.byref(k)) == 0
        eng.run()
        eng.sync()
        o.run(oh, pk, k.value, ar, alen)
        nacks = rtx_lib.make_nacks(o.api, oh, tr, seed=8)
        now = EPOCH + 6 * 10**9
        g = rtx_lib.rtx_lookup(eng.api, eng.h, nacks, now)
        r = rtx_lib.rtx_lookup(o.api, oh, nacks, now)
        assert len(g) == len(r) > 20
        go, gw = rtx_lib.rtx_emit_bucket(eng.api, eng.h, g)
        oo, ow = rtx_lib.rtx_emit_bucket(o.api, oh, r)
        assert len(go) == len(oo) > 10
        for f in oo.dtype.names:
            assert np.array_equal(go[f], oo[f]), f
        assert np.array_equal(gw, ow)
    finally:
        o.destroy(oh)
        eng.close()
