"""SRTP protect parity, engine (k_srtp_protect) vs oracle (oracle/srtp_oracle.h).

The same batches, transports (one per (room, subscriber), every seventh
DownTrack unbound) and send times on both; every protected packet — header
with its abs-send-time stamped, AES-CM ciphertext, HMAC-SHA1 tag — must be
identical (AES-CM ciphertext and HMAC-SHA1 tag, or AEAD_AES_128_GCM
ciphertext and GCM tag for the GCM transports), over several batches (rollover bases carried; seed 5 has DownTracks
whose munged sequence numbers wrap), with a pipelined variant that protects
each run before the previous one has been drained."""
import numpy as np
import pytest

from tests import srtp_lib
from tests.oracle_lib import load as load_oracle

pytestmark = pytest.mark.gpu
EPOCH = 1700000000 * 10**9


def _compare(pkg, eng, o, oh, b, bound):
    """Every record's protected packet (out_len + 10 bytes when its DownTrack
    is bound to a transport) byte for byte; returns the protected count."""
    grec, _ = eng.drain()
    orec, _ = pkg.drain_arrays(o.api, oh)
    assert len(grec) == len(orec)
    assert np.array_equal(grec["out_off"], orec["out_off"])
    gp = pkg.drain_protected(eng.api, eng.h)
    op = pkg.drain_protected(o.api, oh)
    assert len(gp) == len(op)
    n_prot = 0
    for i in range(len(orec)):
        r = orec[i]
        off = int(r["out_off"]) + 16 * i
        d = int(r["dt"])
        ln = int(r["out_len"]) + ((16 if bound[d][3] == srtp_lib.GCM else 10) if d in bound else 0)
        if not np.array_equal(gp[off:off + ln], op[off:off + ln]):
            bad = int(np.nonzero(gp[off:off + ln] != op[off:off + ln])[0][0])
            raise AssertionError("batch %d record %d (dt %d sn %d len %d) differs at byte %d" % (
                b, i, int(r["dt"]), int(r["ext_sn"]), ln, bad))
        n_prot += ln > int(r["out_len"])
    return n_prot


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=2, seed=5), dict(config=1, seed=4, batch_s=0.05),
                                 dict(config=2, rooms=2, seed=5, gcm_every=2),
                                 dict(config=1, seed=4, batch_s=0.05, gcm_every=1)])
def test_protect_matches_oracle(pkg, workload, cfg):
    kw = dict(cfg)
    bs = kw.pop("batch_s", 1.0)
    ge = kw.pop("gcm_every", 0)
    tr = workload.Trace(kw.pop("config"), duration_s=4.0 if bs == 1.0 else 1.0, batch_s=bs, **kw)
    o = load_oracle()
    eng = pkg.Engine.for_trace(tr)
    oh = o.create(500)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        tg = srtp_lib.bind_transports(pkg, eng.api, eng.h, tr, seed=5, gcm_every=ge)
        to = srtp_lib.bind_transports(pkg, o.api, oh, tr, seed=5, gcm_every=ge)
        assert sorted(tg) == sorted(to)
        n_prot = 0
        for b in range(tr.nbatches):
            workload.queue_events(eng.api, eng.h, tr, b)
            workload.queue_events(o.api, oh, tr, b)
            pk, n, ar, alen = tr.batch(b)
            eng.submit(pk, n, ar, alen)
            eng.run()
            send = EPOCH + b * 10**9 + 987654321
            assert eng.api["protect"](eng.h, send) == 0
            eng.sync()
            o.run(oh, pk, n, ar, alen)
            assert o.api["protect"](oh, send) == 0
            n_prot += _compare(pkg, eng, o, oh, b, tg)
        assert n_prot > 100
    finally:
        o.destroy(oh)
        eng.close()
