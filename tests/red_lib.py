"""RED helpers shared by the CPU (oracle) and GPU (engine vs oracle) tests:
drive lkf_red_encode / lkf_red_decode (or the oracle's orc_red_*) over the
Opus tracks of a synthetic trace's ExtPacket batches."""
import ctypes as C
import importlib

import numpy as np

abi = importlib.import_module("livekit-server_amd.abi")
PKT_DTYPE = np.dtype((np.void, 64))


def opus_map(trace):
    m = np.full(trace.ntracks, -1, dtype=np.int32)
    for t in range(trace.ntracks):
        if trace.tracks[t].kind == 0:
            m[t] = t  # the RED view is labelled with the source track (a test choice)
    return m


def batch_arrays(trace, b):
    pk, n, ar, alen = trace.batch(b)
    pkts = np.frombuffer(C.string_at(pk, max(1, n) * 64), dtype=np.uint8)[:n * 64].copy()
    arena = np.frombuffer(C.string_at(ar, alen), dtype=np.uint8).copy() if alen else np.zeros(1, np.uint8)
    return pkts, n, arena, alen


def red(api, h, fn, pkts, n, arena, alen, m):
    """-> (lkf_pkt bytes [k*64], k, arena bytes)"""
    cap = 3 * max(1, n)
    out = np.zeros(cap * 64, dtype=np.uint8)
    acap = 3 * (int(alen) + 1600 * max(1, n)) + 64
    oar = np.zeros(acap, dtype=np.uint8)
    k, ol = C.c_uint32(), C.c_uint64()
    rc = api[fn](h, pkts.ctypes.data, n, arena.ctypes.data, alen, m.ctypes.data, len(m), out.ctypes.data, cap,
                 oar.ctypes.data, acap, C.byref(k), C.byref(ol))
    assert rc == 0, (fn, rc)
    return out[:k.value * 64], k.value, oar[:ol.value]


def drop(pkts, n, keep):
    """the packets whose mask entry is set (descriptors only: the arena is shared)"""
    v = pkts.reshape(n, 64)[keep]
    return v.reshape(-1).copy(), int(keep.sum())


def fields(pkts, k):
    """(ext_sn, ext_ts, track, payload_off, payload_len, hdr1) arrays of an lkf_pkt byte array"""
    v = pkts.reshape(k, 64)
    sn = v[:, 0:8].copy().view("<u8")[:, 0]
    ts = v[:, 8:16].copy().view("<u8")[:, 0]
    arena_off = v[:, 24:28].copy().view("<u4")[:, 0]
    track = v[:, 28:32].copy().view("<u4")[:, 0]
    poff = v[:, 36:38].copy().view("<u2")[:, 0]
    plen = v[:, 38:40].copy().view("<u2")[:, 0]
    return dict(ext_sn=sn, ext_ts=ts, arena_off=arena_off, track=track, payload_off=poff, payload_len=plen,
                hdr1=v[:, 41].copy())
