"""The TWCC responder's input at ingress (Buffer.processHeaderExtensions,
pkg/sfu/buffer/buffer.go:569-576): for every datagram that unmarshals, on a
stream with a negotiated transport-cc id, whose header carries that element,
twcc.Responder.Push(BigEndian.Uint16(ext[0:2]), arrival, marker).

The oracle's words (orc_ingest_twcc) are checked against an independent
parse of the raw datagrams here (RFC 8285 one- and two-byte extension blocks,
first element with the id), on traces with loss and reordering (out-of-order
and duplicate datagrams still push) and DD tracks (two-byte blocks).  The
Responder itself (mediatransportutil twcc, RTCP TransportLayerCC building) is
outside the path; parity unpinned beyond the call's arguments."""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle

TWCC_ID = 5  # the synthetic streams' transport-cc id


def ext_element(pkt, want):
    """Payload of the first header-extension element with id `want`, or None."""
    if len(pkt) < 12 or not (pkt[0] & 0x10):
        return None
    x = 12 + 4 * (pkt[0] & 15)
    if len(pkt) < x + 4:
        return None
    prof = (pkt[x] << 8) | pkt[x + 1]
    end = x + 4 + 4 * ((pkt[x + 2] << 8) | pkt[x + 3])
    p = x + 4
    if prof not in (0xBEDE, 0x1000):
        return None
    while p < end:
        if pkt[p] == 0:
            p += 1
            continue
        if prof == 0xBEDE:
            i, ln, d = pkt[p] >> 4, (pkt[p] & 15) + 1, p + 1
            if i == 15:
                break
        else:
            i, ln, d = pkt[p], pkt[p + 1], p + 2
        if i == want:
            return bytes(pkt[d:d + ln])
        p = d + ln
    return None


@pytest.mark.parametrize("kw", [dict(config=2, duration_s=2.0, rooms=2, loss=0.05, reorder=0.05, seed=3),
                                dict(config=5, duration_s=2.0, rooms=2, seed=4)])
def test_oracle_twcc_pushes(kw, pkg, workload, abi):
    o = load_oracle()
    tr = workload.Trace(**kw)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        workload.load_streams(o.api, h, tr)
        pushes = markers = 0
        for b in range(tr.nbatches):
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](h, rp, n, ar, alen) == 0
            got = pkg.twcc_words(o.api, h)
            assert len(got) == n
            arena = C.string_at(ar, alen) if alen else b""
            want = np.zeros(n, dtype=np.uint32)
            for i in range(n):
                pkt = arena[rp[i].off:rp[i].off + rp[i].len]
                e = ext_element(pkt, TWCC_ID)
                if e is not None and len(e) >= 2:
                    want[i] = abi.LKF_TWCC_PUSH | (abi.LKF_TWCC_MARKER if pkt[1] & 0x80 else 0) | (e[0] << 8) | e[1]
            assert np.array_equal(got, want), (b, np.nonzero(got != want)[0][:5])
            pushes += int(np.count_nonzero(got))
            markers += int(np.count_nonzero(got & abi.LKF_TWCC_MARKER))
        assert pushes > 500 and markers > 10
    finally:
        o.destroy(h)


def test_oracle_transport_cc_numbering(pkg, workload, abi):
    """The oracle's TWCC interceptor restatement: per transport, the records of
    its transport-cc DownTracks carry consecutive sequence numbers in output
    (send) order across batches; abs-send-time subscribers carry none; an
    unbound DownTrack counts on its own."""
    import ctypes as C

    from tests import srtp_lib
    from tests.oracle_lib import load as load_oracle
    from tests.test_twcc_send_gpu import _tcc_values
    o = load_oracle()
    tr = workload.Trace(2, duration_s=3.0, batch_s=1.0, rooms=2, seed=8, twcc=1)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        tmap = srtp_lib.bind_transports(pkg, o.api, h, tr, seed=6)
        nxt = {}
        seen = 0
        for b in range(tr.nbatches):
            workload.queue_events(o.api, h, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(h, pk, n, ar, alen)
            rec, arr = pkg.drain_arrays(o.api, h)
            for d, v in _tcc_values(tr, rec, arr):
                key = ("t", tmap[d][0]) if d in tmap else ("d", d)
                assert v == nxt.get(key, 0) & 0xFFFF, (b, d, v, nxt.get(key))
                nxt[key] = nxt.get(key, 0) + 1
                seen += 1
            for r in rec:  # an abs-send-time subscriber's packet keeps its 20-B header (no element added)
                p = tr.downtracks[int(r["dt"])]
                if p.ext_abs_send_time and not p.ext_dd:
                    w = arr[int(r["out_off"]):int(r["out_off"]) + 16]
                    assert (int(w[14]) << 8 | int(w[15])) == 1, "one-word extension block"
        assert seen > 1000
        assert any(k[0] == "d" for k in nxt) and any(k[0] == "t" for k in nxt)
    finally:
        o.destroy(h)
        tr.close()
