"""Padding / blank-frame helpers shared by the CPU (oracle) and GPU (engine vs
oracle) tests: request lists over many DownTracks with the DownTrack facts the
engine does not track (writable, RTCP RR seen, paddingOnMute, forceMarker)
varied, and Forwarder.maybeStart's random start drawn from the reference's
ranges (forwarder.go:1774-1775)."""
import ctypes as C
import importlib

import numpy as np

abi = importlib.import_module("livekit-server_amd.abi")


def make_reqs(ndts, seed, frac=0.6, max_bytes=3000):
    rng = np.random.default_rng(seed)
    dts = rng.choice(ndts, size=max(1, int(ndts * frac)), replace=False)
    r = np.zeros(len(dts), dtype=abi.PAD_REQ_DTYPE)
    r["dt"] = dts
    r["bytes_to_send"] = rng.integers(0, max_bytes, len(dts))
    fl = np.full(len(dts), abi.PAD_WRITABLE | abi.PAD_RR_SEEN, dtype=np.uint32)
    u = rng.random(len(dts))
    fl[u < 0.10] &= ~np.uint32(abi.PAD_WRITABLE)   # closed / not bound
    fl[(u >= 0.10) & (u < 0.20)] &= ~np.uint32(abi.PAD_RR_SEEN)  # no receiver report yet
    fl[(u >= 0.20) & (u < 0.35)] |= abi.PAD_ON_MUTE
    fl[(u >= 0.35) & (u < 0.55)] |= abi.PAD_FORCE_MARKER
    r["flags"] = fl
    r["start_sn"] = rng.integers(1 << 15, (1 << 15) + (1 << 14), len(dts))
    r["start_ts"] = rng.integers(1 << 31, (1 << 31) + (1 << 30), len(dts), dtype=np.uint64).astype(np.uint32)
    return r


def pad(api, h, reqs, now_ns, blank=False):
    """-> (records, wire bytes, bytes_sent per request or None)"""
    n = len(reqs)
    cap = max(1, int(sum(2 if blank else (int(b) + 274) // 275 for b in reqs["bytes_to_send"])))
    out = np.zeros(cap, dtype=abi.OUT_DTYPE)
    arena = np.zeros(cap * 288 + 64, dtype=np.uint8)
    k = C.c_uint32()
    al = C.c_uint64()
    if blank:
        rc = api["blank_frames"](h, reqs.ctypes.data, n, now_ns, out.ctypes.data, arena.ctypes.data, cap, len(arena),
                                 C.byref(k), C.byref(al))
        sent = None
    else:
        sent = np.zeros(max(1, n), dtype=np.uint32)
        rc = api["padding"](h, reqs.ctypes.data, n, now_ns, out.ctypes.data, arena.ctypes.data, cap, len(arena),
                            C.byref(k), C.byref(al), sent.ctypes.data)
        sent = sent[:n]
    assert rc == 0, rc
    return out[:k.value], arena[:al.value], sent
