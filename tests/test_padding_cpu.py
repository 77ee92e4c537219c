"""Padding / blank frames on the CPU oracle (the checker of the GPU path):
the wire layout of WritePaddingRTP (downtrack.go:797-855) and
writeBlankFrameRTP (:1358-1393), SN continuity through the munger's
RangeMap.DecValue (rtpmunger.go:336), and NACKs for padding SNs dropped by
the sequencer's exclusion range (sequencer.go:211-261; the exclusion logic
itself is pinned by the sequencer_test.go KATs in oracle/kat_sfu.inc)."""
import ctypes as C

import numpy as np

from tests import pad_lib
from tests.oracle_lib import load as load_oracle

EPOCH = 1700000000 * 10**9
VP8_KEY_8x8 = bytes([0x10, 0x02, 0x00, 0x9d, 0x01, 0x2a, 0x08, 0x00, 0x08, 0x00, 0x00, 0x47, 0x08, 0x85, 0x85, 0x88,
                     0x85, 0x84, 0x88, 0x02, 0x02, 0x00, 0x0c, 0x0d, 0x60, 0x00, 0xfe, 0xff, 0xab, 0x50, 0x80])


def _run(o, oh, tr, workload, b):
    workload.queue_events(o.api, oh, tr, b)
    pk, n, ar, alen = tr.batch(b)
    o.run(oh, pk, n, ar, alen)


def test_padding_wire_and_continuity(pkg, workload):
    o = load_oracle()
    abi = pkg.abi
    tr = workload.Trace(2, duration_s=3.0, batch_s=1.0, rooms=2, seed=5)
    oh = o.create(500)
    try:
        workload.load_topology(o.api, oh, tr)
        _run(o, oh, tr, workload, 0)
        _run(o, oh, tr, workload, 1)
        before = {}
        for dt in range(tr.ndts):
            st = abi.lkf_fwd_state()
            o.api["get_state"](oh, dt, C.byref(st))
            before[dt] = (st.ext_last_sn, st.ext_last_ts)
        reqs = pad_lib.make_reqs(tr.ndts, seed=3, frac=1.0)
        reqs["flags"] = abi.PAD_WRITABLE | abi.PAD_RR_SEEN | abi.PAD_FORCE_MARKER
        reqs["bytes_to_send"] = 1000  # ceil(1000 / 275) = 4 packets
        now = EPOCH + 2 * 10**9 - 10**6
        out, wire, sent = pad_lib.pad(o.api, oh, reqs, now)
        video = {int(r["dt"]) for r in out}
        assert video and len(out) == 4 * len(video)
        for i, r in zip(range(len(reqs)), reqs):
            assert sent[i] == (4 * 267 if int(r["dt"]) in video else 0)
        padded = {}
        for r in out:
            dt = int(r["dt"])
            last_sn, last_ts = before[dt]
            k = padded.setdefault(dt, 0)
            assert r["ext_sn"] == last_sn + 1 + k and r["ext_ts"] == last_ts
            padded[dt] = k + 1
            pkt = bytes(wire[r["out_off"]:r["out_off"] + r["out_len"]])
            ext = 8 if pkt[0] & 0x10 else 0
            assert pkt[0] & 0x20 and not pkt[1] & 0x80 and r["out_len"] == 12 + ext + 255
            assert pkt[-1] == 255 and not any(pkt[12 + ext:-1])
        # the next batch continues after the padding SNs, and NACKs for them find nothing
        _run(o, oh, tr, workload, 2)
        rec, _ = pkg.drain_arrays(o.api, oh)
        firsts = [(int(rec[rec["dt"] == dt]["ext_sn"][0]), before[dt][0] + 5) for dt in video if (rec["dt"] == dt).any()]
        assert firsts  # (a loss gap or a late out-of-order packet may come first)
        assert sum(f == e for f, e in firsts) * 2 > len(firsts)
        dt = sorted(video)[0]
        sns = (C.c_uint16 * 4)(*[int(before[dt][0] + 1 + k) & 0xFFFF for k in range(4)])
        meta = (abi.lkf_seq_meta * 4)()
        k = C.c_uint32()
        assert o.api["seq_lookup"](oh, dt, sns, 4, now + 10**9, meta, C.byref(k)) == 0
        assert k.value == 0
    finally:
        o.destroy(oh)
        tr.close()


def test_blank_frames_payloads(pkg, workload):
    o = load_oracle()
    tr = workload.Trace(2, duration_s=2.0, batch_s=1.0, rooms=1, seed=8)
    oh = o.create(500)
    try:
        workload.load_topology(o.api, oh, tr)
        _run(o, oh, tr, workload, 0)
        _run(o, oh, tr, workload, 1)
        reqs = pad_lib.make_reqs(tr.ndts, seed=4, frac=1.0)
        reqs["flags"] = pkg.abi.PAD_WRITABLE
        out, wire, _ = pad_lib.pad(o.api, oh, reqs, EPOCH + 2 * 10**9, blank=True)
        assert len(out) >= len(reqs) // 2
        kinds = set()
        for r in out:
            pkt = bytes(wire[r["out_off"]:r["out_off"] + r["out_len"]])
            assert pkt[1] & 0x80 and not pkt[0] & 0x20  # marker, no padding
            body = pkt[12 + (8 if pkt[0] & 0x10 else 0):]
            if body.endswith(VP8_KEY_8x8):
                kinds.add("vp8")
                assert 1 <= len(body) - 31 <= 6  # the VP8 padding descriptor (vp8.go:304-363)
            else:
                assert body == bytes([0xf8, 0xff, 0xfe]) + bytes(77)  # OpusSilenceFrame
                kinds.add("opus")
        assert kinds == {"vp8", "opus"}
    finally:
        o.destroy(oh)
        tr.close()
