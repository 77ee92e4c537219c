"""Control calls overlapping queued runs, engine vs oracle.

The other GPU tests call lkf_sync before every control call; here padding,
blank frames, NACK lookups and RTX emission (host-sourced and bucket-sourced)
are issued right behind several queued 10-ms runs with no sync in between.
A 10-ms batch's sender statistics (RTPStatsSender.Update per forwarded
tuple) run on the emit stream after emit (k_sender_stats_thread), while the
control calls' own sendingPacket updates run on the sender stream: the engine
must order the latter after the former (engine.cpp sender_after_queued), or
one set of updates to the same DownTrack's statistics is lost or reordered.
Every output and, at the end, every DownTrack's sender statistics must equal
the oracle's, which runs the same calls in the same order serially."""
import ctypes as C

import numpy as np
import pytest

from tests import pad_lib, rtx_lib
from tests.oracle_lib import load as load_oracle
from tests.test_parity_gpu import check_sender_stats

pytestmark = pytest.mark.gpu
EPOCH = 1700000000 * 10**9


def _same(g, o, what):
    go, gw = g[0], g[1]
    oo, ow = o[0], o[1]
    assert len(go) == len(oo), (what, len(go), len(oo))
    for f in oo.dtype.names:
        assert np.array_equal(go[f], oo[f]), (what, f)
    assert np.array_equal(gw, ow), what


def test_control_calls_behind_queued_short_runs(pkg, workload):
    o = load_oracle()
    tr = workload.Trace(2, duration_s=0.8, batch_s=0.01, rooms=4, seed=21)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    nb = tr.nbatches
    state = {"b": 0}

    def queue(k):  # k runs on both sides; the engine's are only enqueued
        for _ in range(k):
            b = state["b"]
            if b >= nb:
                return
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            eng.submit(pk, n, ar, alen)
            eng.run()
            o.run(oh, pk, n, ar, alen)
            state["b"] = b + 1

    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        queue(12)  # Forwarders start
        step, calls = 0, {"pad": 0, "blank": 0, "rtx": 0}
        while state["b"] < nb:
            queue(5)
            now = EPOCH + int(state["b"] * 0.01 * 1e9)
            kind = ("pad", "blank", "rtx")[step % 3]
            if kind in ("pad", "blank"):
                reqs = pad_lib.make_reqs(tr.ndts, seed=100 + step, frac=0.3, max_bytes=1200)
                g = pad_lib.pad(eng.api, eng.h, reqs, now, blank=kind == "blank")
                r = pad_lib.pad(o.api, oh, reqs, now, blank=kind == "blank")
                _same(g, r, (kind, step))
                calls[kind] += len(r[0])
            else:
                nacks = rtx_lib.make_nacks(o.api, oh, tr, seed=200 + step, max_dts=120, per_dt=4)
                g = rtx_lib.rtx_lookup(eng.api, eng.h, nacks, now)
                r = rtx_lib.rtx_lookup(o.api, oh, nacks, now)
                assert len(g) == len(r), (step, len(g), len(r))
                for f in r.dtype.names:
                    assert np.array_equal(g[f], r[f]), (step, f)
                queue(3)  # more runs between the lookup and the emission
                idx = rtx_lib.packet_index(tr, state["b"])
                _same(rtx_lib.rtx_emit(eng.api, eng.h, tr, g, idx), rtx_lib.rtx_emit(o.api, oh, tr, r, idx),
                      ("rtx", step))
                calls["rtx"] += len(r)
            step += 1
        eng.sync()
        assert calls["pad"] > 0 and calls["blank"] > 0 and calls["rtx"] > 0, calls
        ss = check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(tr.ndts))
        assert int(ss["packets_padding"].sum()) > 0 and int(ss["packets_duplicate"].sum()) > 0
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


def test_bucket_rtx_behind_queued_ingest_runs(pkg, workload, abi):
    """The same for the ingest path: raw 10-ms batches ingested and forwarded
    without a sync, then NACK lookups and lkf_rtx_emit_bucket (the sources read
    from the GPU buckets, whose copies run on the sender stream) right behind
    them."""
    o = load_oracle()
    tr = workload.Trace(2, duration_s=0.6, batch_s=0.01, rooms=3, seed=23, loss=0.02, reorder=0.01)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    nb = tr.nbatches
    state = {"b": 0}

    def queue(k):
        for _ in range(k):
            b = state["b"]
            if b >= nb:
                return
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            rp, n, ar, alen = tr.batch_raw(b)
            eng.ingest(rp, n, ar, alen)
            eng.run()
            assert o.api["ingest"](oh, rp, n, ar, alen) == 0
            k2 = C.c_uint32()
            assert o.api["ingested"](oh, None, 0, C.byref(k2)) in (0, -28)
            arr = (abi.lkf_pkt * max(1, k2.value))()
            assert o.api["ingested"](oh, arr, k2.value, C.byref(k2)) == 0
            o.run(oh, arr if k2.value else None, k2.value, ar, alen)
            state["b"] = b + 1

    try:
        for api, h in ((eng.api, eng.h), (o.api, oh)):
            workload.load_topology(api, h, tr)
            workload.load_streams(api, h, tr)
        queue(12)
        step, sent = 0, 0
        while state["b"] < nb:
            queue(6)
            now = EPOCH + int(state["b"] * 0.01 * 1e9)
            nacks = rtx_lib.make_nacks(o.api, oh, tr, seed=300 + step, max_dts=100, per_dt=4)
            g = rtx_lib.rtx_lookup(eng.api, eng.h, nacks, now)
            r = rtx_lib.rtx_lookup(o.api, oh, nacks, now)
            assert len(g) == len(r), (step, len(g), len(r))
            queue(2)
            _same(rtx_lib.rtx_emit_bucket(eng.api, eng.h, g), rtx_lib.rtx_emit_bucket(o.api, oh, r), ("bucket", step))
            sent += len(r)
            step += 1
        eng.sync()
        assert sent > 0
        check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(tr.ndts))
    finally:
        o.destroy(oh)
        eng.close()
