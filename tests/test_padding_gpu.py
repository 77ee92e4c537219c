"""Padding and blank frames, engine vs oracle.

Batches are forwarded, then WritePaddingRTP runs on most DownTracks (mixed
gates, byte budgets, forced markers, Forwarders that have not started), more
batches follow, then blank-frame ticks, more batches and NACK lookups.  The
padding and blank-frame packets, the bytes WritePaddingRTP reports, every
later batch (the munger's RangeMap.DecValue carries the SN offset on), the
Forwarder state, the sendingPacket totals and the sequencer lookups (padding
SNs are excluded by pushPadding's RangeMap) must all be identical."""
import ctypes as C

import numpy as np
import pytest

from tests import pad_lib, rtx_lib
from tests.oracle_lib import load as load_oracle
from tests.test_parity_gpu import check_sender_stats

pytestmark = pytest.mark.gpu
EPOCH = 1700000000 * 10**9


def _same(a, b, what):
    assert len(a) == len(b), (what, len(a), len(b))
    for f in a.dtype.names:
        assert np.array_equal(a[f], b[f]), (what, f)


def _state(api, h, dt, abi):
    st = abi.lkf_fwd_state()
    assert api["get_state"](h, dt, C.byref(st)) == 0
    return st.as_tuple()


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=4, seed=3), dict(config=1, seed=2),
                                 dict(config=2, rooms=3, seed=11, h264=1), dict(config=5, rooms=6, svc_dd=1)])
def test_padding_and_blank_frames_match_oracle(pkg, workload, cfg):
    o = load_oracle()
    abi = pkg.abi
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=6.0, batch_s=1.0, **kw)
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    # pad before batch 0 (Forwarders not started: maybeStart), after 1 and 3; blank after 2 and 4
    plan = {0: "pad", 2: "pad", 3: "blank", 4: "pad", 5: "blank"}
    sent_any = 0
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        for b in range(tr.nbatches):
            now = EPOCH + b * 10**9 - 10**6
            if b in plan:
                blank = plan[b] == "blank"
                reqs = pad_lib.make_reqs(tr.ndts, seed=100 + b, frac=0.7)
                if b == 0:
                    reqs["flags"] |= abi.PAD_ON_MUTE  # before anything is forwarded only paddingOnMute sends
                go, gw, gs = pad_lib.pad(eng.api, eng.h, reqs, now, blank)
                oo, ow, os_ = pad_lib.pad(o.api, oh, reqs, now, blank)
                _same(go, oo, (b, plan[b]))
                assert np.array_equal(gw, ow), (b, plan[b], "wire")
                if not blank:
                    assert np.array_equal(gs, os_), (b, "bytes_sent")
                sent_any += len(oo)
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            dd = tr.batch_dd(b)[0] if tr.has_dd() else None
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            eng.sync()
            o.run(oh, pk, n, ar, alen, dd)
            grec, gar = eng.drain()
            orec, oar = pkg.drain_arrays(o.api, oh)
            _same(grec, orec, (b, "batch"))
            assert np.array_equal(gar, oar), (b, "batch wire")
        assert sent_any > 50
        for dt in range(tr.ndts):
            assert _state(eng.api, eng.h, dt, abi) == _state(o.api, oh, dt, abi), dt
        _same(pkg.downtrack_summaries(eng.api, eng.h), pkg.downtrack_summaries(o.api, oh), "summaries")
        # RTPStatsSender after forwarded packets, padding and blank frames (sendingPacket isPadding)
        ss = check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(tr.ndts))
        assert int(ss["packets_padding"].sum()) > 0
        nacks = rtx_lib.make_nacks(o.api, oh, tr, seed=7, per_dt=12)
        now = EPOCH + tr.nbatches * 10**9 + 5 * 10**8
        _same(rtx_lib.rtx_lookup(eng.api, eng.h, nacks, now), rtx_lib.rtx_lookup(o.api, oh, nacks, now), "rtx")
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()


def test_padding_rejects_repeated_downtrack(pkg, workload):
    tr = workload.Trace(1, duration_s=1.0, batch_s=1.0)
    eng = pkg.Engine.for_trace(tr)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        reqs = pad_lib.make_reqs(tr.ndts, seed=1, frac=0.2)
        reqs = np.concatenate([reqs, reqs[:1]])
        k, al = C.c_uint32(), C.c_uint64()
        rc = eng.api["padding"](eng.h, reqs.ctypes.data, len(reqs), 0, None, None, 0, 0, C.byref(k), C.byref(al), None)
        assert rc == -22  # LKF_EINVAL
    finally:
        eng.close()
        tr.close()
