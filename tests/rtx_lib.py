"""NACK -> RTX helpers shared by the CPU (oracle) and GPU (engine vs oracle) tests.

NACK lists are drawn around each DownTrack's last forwarded sequence number
(plus a duplicate, a future and a too-old SN per list); the source packet of
an RTX record — what Receiver.ReadRTP(layer, source_sn) returns from the
bucket — is the raw RTP packet of the trace with that (track, layer, SN)."""
import ctypes as C
import importlib

import numpy as np

abi = importlib.import_module("livekit-server_amd.abi")


def packet_index(trace, upto):
    """(track, layer, sn16) -> raw RTP bytes, for batches [0, upto)."""
    idx = {}
    for b in range(upto):
        pk, n, ar, alen = trace.batch(b)
        if not n:
            continue
        arena = C.string_at(ar, alen)
        for i in range(n):
            p = pk[i]
            idx[(p.track, p.layer, p.ext_sn & 0xFFFF)] = arena[p.arena_off:p.arena_off + p.payload_off + p.payload_len]
    return idx


def make_nacks(api, h, trace, seed, max_dts=300, per_dt=6):
    rng = np.random.default_rng(seed)
    dts = rng.choice(trace.ndts, size=min(trace.ndts, max_dts), replace=False)
    rows = []
    for dt in dts:
        st = abi.lkf_fwd_state()
        assert api["get_state"](h, int(dt), C.byref(st)) == 0
        if not st.started:
            continue
        last = st.ext_last_sn & 0xFFFF
        sns = [(last - int(k)) & 0xFFFF for k in rng.integers(0, 400, per_dt)]
        sns.append(sns[0])                 # repeated in one list: the second is suppressed (RTT)
        sns.append((last + 7) & 0xFFFF)    # ahead of the highest
        sns.append((last - 40000) & 0xFFFF)  # outside the window
        rows += [(int(dt), s, 0) for s in sns]
    return np.array(rows, dtype=abi.NACK_DTYPE)


def rtx_lookup(api, h, nacks, now_ns):
    out = np.zeros(max(1, len(nacks)), dtype=abi.RTX_DTYPE)
    k = C.c_uint32()
    rc = api["rtx_lookup"](h, nacks.ctypes.data, len(nacks), now_ns, out.ctypes.data, len(out), C.byref(k))
    assert rc == 0, rc
    return out[:k.value]


def rtx_emit(api, h, trace, rtx, idx):
    n = len(rtx)
    src = (abi.lkf_raw_pkt * max(1, n))()
    blob = bytearray()
    for i in range(n):
        track = trace.downtracks[int(rtx["dt"][i])].track
        raw = idx.get((track, int(rtx["layer"][i]), int(rtx["source_sn"][i])), b"")
        src[i].off = len(blob)
        src[i].len = len(raw)
        blob += raw
        blob += bytes((-len(blob)) % 16)
    arena = (C.c_uint8 * max(1, len(blob))).from_buffer_copy(bytes(blob) or b"\0")
    out = np.zeros(max(1, n), dtype=abi.OUT_DTYPE)
    cap = len(blob) + 320 * n + 64  # (+ CSRCs and the pacer's extension block, a DD up to 255 B)
    wire = np.zeros(cap, dtype=np.uint8)
    k = C.c_uint32()
    ol = C.c_uint64()
    rc = api["rtx_emit"](h, rtx.ctypes.data, n, src, arena, len(blob), out.ctypes.data, wire.ctypes.data, cap,
                         C.byref(k), C.byref(ol))
    assert rc == 0, rc
    return out[:k.value], wire[:ol.value]


def rtx_emit_bucket(api, h, rtx, cap_per=1700):
    """lkf_rtx_emit_bucket: the sources read from the receivers' buckets."""
    n = len(rtx)
    out = np.zeros(max(1, n), dtype=abi.OUT_DTYPE)
    cap = cap_per * n + 64
    wire = np.zeros(cap, dtype=np.uint8)
    k = C.c_uint32()
    ol = C.c_uint64()
    rc = api["rtx_emit_bucket"](h, rtx.ctypes.data, n, out.ctypes.data, wire.ctypes.data, cap, C.byref(k),
                                C.byref(ol))
    assert rc == 0, rc
    return out[:k.value], wire[:ol.value]


def ingest_forward(api, h, trace, workload, nb, run):
    """Raw datagrams through lkf_ingest (the buckets fill), then the ingested
    ExtPackets forwarded: run(b, ingested lkf_pkt bytes, count, arena, len)."""
    for b in range(nb):
        workload.queue_events(api, h, trace, b)
        rp, n, ar, alen = trace.batch_raw(b)
        assert api["ingest"](h, rp, n, ar, alen) == 0
        k = C.c_uint32()
        rc = api["ingested"](h, None, 0, C.byref(k))
        assert rc in (0, -28)
        arr = (abi.lkf_pkt * max(1, k.value))()
        assert api["ingested"](h, arr, k.value, C.byref(k)) == 0
        run(b, arr, k.value, ar, alen)


def wire_by_rtx(out, wire):
    """RTX index (lkf_out.pkt) -> its wire packet."""
    return {int(r["pkt"]): bytes(wire[int(r["out_off"]):int(r["out_off"]) + int(r["out_len"])]) for r in out}


def count_dd_elements(trace, out, wire):
    """RTX packets whose extension block carries the DownTrack's DD element."""
    k = 0
    for r in out:
        dd_id = int(trace.downtracks[int(r["dt"])].ext_dd)
        w = wire[int(r["out_off"]):int(r["out_off"]) + int(r["out_len"])]
        if not dd_id or not (int(w[0]) & 0x10):
            continue
        h = 12 + 4 * (int(w[0]) & 0xF)
        prof = (int(w[h]) << 8) | int(w[h + 1])
        words = (int(w[h + 2]) << 8) | int(w[h + 3])
        q, end = h + 4, h + 4 + 4 * words
        while q < end:
            if prof == 0xBEDE:
                if w[q] == 0:
                    q += 1
                    continue
                eid, ln = int(w[q]) >> 4, (int(w[q]) & 0xF) + 1
                q += 1
            else:
                if w[q] == 0:
                    q += 1
                    continue
                eid, ln = int(w[q]), int(w[q + 1])
                q += 2
            if eid == dd_id:
                k += 1
                break
            q += ln
    return k
