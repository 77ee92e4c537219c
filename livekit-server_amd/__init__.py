"""lkfwd — MI355X-native batched RTP forwarding engine (livekit-server SFU hot path).

The product is ``lib/liblkfwd.so`` (gfx950 HIP kernels + C++ host engine,
C-ABI in ``include/lkfwd.h``).  This module is a thin ctypes loader used by the
tests and bench: it never computes anything itself and has no CPU fallback —
if the HIP library is missing or no GPU is present, it raises.

Import with ``importlib.import_module("livekit-server_amd")`` (the directory
name contains a hyphen).
"""
import ctypes as C
import os

import numpy as np

from . import abi

# LKF_LIB names another build of the engine in lib/ (liblkfwd_checked.so: the
# bounds-checked kernels of `make` target liblkfwd_checked.so)
LIB_PATH = os.path.join(abi.LIBDIR, os.environ.get("LKF_LIB", "liblkfwd.so"))
_lib = None


class EngineError(RuntimeError):
    pass


def load_library(path=None):
    """Loads liblkfwd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError("liblkfwd.so not built (%s): run __graft_entry__.build()" % p)
    lib = C.CDLL(p)
    v = C.c_void_p
    lib.lkf_create.restype = v
    lib.lkf_create.argtypes = [C.c_int, C.POINTER(abi.lkf_cfg)]
    lib.lkf_destroy.restype = None
    lib.lkf_destroy.argtypes = [v]
    lib.lkf_last_error.restype = C.c_char_p
    lib.lkf_last_error.argtypes = [v]
    lib.lkf_version.restype = C.c_char_p
    lib.lkf_version.argtypes = []
    lib.lkf_submit.restype = C.c_int
    lib.lkf_submit.argtypes = [v, v, C.c_uint32, v, C.c_uint64]
    lib.lkf_submit_device.restype = C.c_int
    lib.lkf_submit_device.argtypes = [v, v, C.c_uint32, v, C.c_uint64]
    lib.lkf_run.restype = C.c_int
    lib.lkf_run.argtypes = [v, v]
    lib.lkf_sync.restype = C.c_int
    lib.lkf_sync.argtypes = [v]
    lib.lkf_output_device.restype = C.c_int
    lib.lkf_output_device.argtypes = [v, C.POINTER(v), C.POINTER(C.c_uint64), C.POINTER(v), C.POINTER(C.c_uint64)]
    lib.lkf_last_timings.restype = C.c_int
    lib.lkf_last_timings.argtypes = [v, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
    lib.lkf_timing_window.restype = C.c_int
    lib.lkf_timing_window.argtypes = [v, C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                      C.POINTER(C.c_float)]
    lib.lkf_get_cumulative.restype = C.c_int
    lib.lkf_get_cumulative.argtypes = [v, C.POINTER(abi.lkf_stats), C.c_int]
    if hasattr(lib, "lkf_debug_check"):
        lib.lkf_debug_check.restype = C.c_int
        lib.lkf_debug_check.argtypes = [v, C.POINTER(C.c_uint64), C.c_int]
    lib.api = abi.bind_engine_api(lib, "lkf_")
    if path is None:
        _lib = lib
    return lib


def debug_check(reset=True):
    """Bounds-check record of a checked build (LKF_LIB=liblkfwd_checked.so):
    (violations, first site, its index, its capacity), or None for a product
    build."""
    lib = load_library()
    out = (C.c_uint64 * 4)()
    rc = lib.lkf_debug_check(None, out, 1 if reset else 0)
    if rc != 0:
        return None
    return tuple(int(x) for x in out)


def drain_arrays(api, h, nmax=None):
    """Reads the last batch's records + wire bytes into numpy arrays."""
    n = C.c_uint64()
    alen = C.c_uint64()
    rc = api["drain"](h, None, 0, None, 0, C.byref(n), C.byref(alen))
    if rc not in (0, -28):  # -28: ENOSPC for the size probe
        raise EngineError("drain probe rc=%d" % rc)
    recs = np.zeros(n.value, dtype=abi.OUT_DTYPE)
    arena = np.zeros(alen.value, dtype=np.uint8)
    rc = api["drain"](h, recs.ctypes.data, n.value, arena.ctypes.data, alen.value, C.byref(n), C.byref(alen))
    if rc != 0:
        msg = api["last_error"](h).decode() if "last_error" in api else ""
        raise EngineError("drain rc=%d (%d records, %d bytes): %s" % (rc, n.value, alen.value, msg))
    return recs, arena


def transport_params(master_key, master_salt, profile=abi.LKF_SRTP_AES128_CM_HMAC_SHA1_80):
    """lkf_transport_params from a DTLS-SRTP export: 16 key bytes and 14 salt
    bytes (12 for AEAD_AES_128_GCM)."""
    t = abi.lkf_transport_params()
    C.memmove(t.master_key, bytes(master_key), 16)
    C.memmove(t.master_salt, bytes(master_salt), len(master_salt))
    t.profile = profile
    return t


def drain_protected(api, h):
    """The last protected run's arena (record i's packet at out_off + 16 * i)."""
    n = C.c_uint64()
    rc = api["drain_protected"](h, None, 0, C.byref(n))
    if rc not in (0, -28):
        raise EngineError("drain_protected probe rc=%d" % rc)
    arena = np.zeros(n.value, dtype=np.uint8)
    rc = api["drain_protected"](h, arena.ctypes.data, n.value, C.byref(n))
    if rc != 0:
        raise EngineError("drain_protected rc=%d" % rc)
    return arena


def twcc_words(api, h):
    """Per-datagram TWCC responder push words (LKF_TWCC_*) of the last ingest."""
    n = C.c_uint32()
    rc = api["ingest_twcc"](h, None, 0, C.byref(n))
    if rc not in (0, -28):
        raise EngineError("ingest_twcc probe rc=%d" % rc)
    out = np.zeros(n.value, dtype=np.uint32)
    rc = api["ingest_twcc"](h, out.ctypes.data, n.value, C.byref(n))
    if rc != 0:
        raise EngineError("ingest_twcc rc=%d" % rc)
    return out


def flows_array(api, h):
    """Per-datagram outcomes (lkf_flow) of the last ingest as a numpy array."""
    n = C.c_uint32()
    rc = api["ingest_flows"](h, None, 0, C.byref(n))
    if rc not in (0, -28):
        raise EngineError("ingest_flows probe rc=%d" % rc)
    out = np.zeros(n.value, dtype=abi.FLOW_DTYPE)
    rc = api["ingest_flows"](h, out.ctypes.data, n.value, C.byref(n))
    if rc != 0:
        raise EngineError("ingest_flows rc=%d" % rc)
    return out


def nacks_arrays(api, h):
    """lkf_ingest_nacks: the last ingest's RTCP NACKs (RTCP_NACK_DTYPE) and
    their pairs (NACK_PAIR_DTYPE)."""
    n = C.c_uint32()
    npairs = C.c_uint32()
    rc = api["ingest_nacks"](h, None, 0, None, 0, C.byref(n), C.byref(npairs))
    if rc not in (0, -28):
        raise EngineError("ingest_nacks probe rc=%d" % rc)
    recs = np.zeros(n.value, dtype=abi.RTCP_NACK_DTYPE)
    pairs = np.zeros(npairs.value, dtype=abi.NACK_PAIR_DTYPE)
    rc = api["ingest_nacks"](h, recs.ctypes.data, n.value, pairs.ctypes.data, npairs.value, C.byref(n),
                             C.byref(npairs))
    if rc != 0:
        raise EngineError("ingest_nacks rc=%d" % rc)
    return recs, pairs


def speakers_array(api, h, now_ns):
    """Room.GetActiveSpeakers for every room at now_ns as a numpy array."""
    n = C.c_uint32()
    cap = 4096
    while True:
        out = np.zeros(cap, dtype=abi.SPEAKER_DTYPE)
        rc = api["speakers"](h, now_ns, out.ctypes.data, cap, C.byref(n))
        if rc == 0:
            return out[:n.value]
        if rc != -28:
            raise EngineError("speakers rc=%d" % rc)
        cap = n.value


def room_summaries_enqueue(api, h, now_ns, room_ids, spk_ptr, k, bwe_ptr, s, stream_ptr):
    """lkf_room_summaries_enqueue: the speaker and bandwidth records of the
    rooms `room_ids` (ascending) packed into device buffers spk int32
    [rows, k, 3] / bwe int64 [rows, s, 5] on the caller stream `stream_ptr`,
    without a host wait (rooms.pack_speakers / rooms.fold_summaries layout)."""
    ids = np.ascontiguousarray(np.asarray(room_ids, dtype=np.uint32))
    rc = api["room_summaries_enqueue"](h, now_ns, ids.ctypes.data, len(ids), spk_ptr, k, bwe_ptr, s, stream_ptr)
    if rc != 0:
        raise EngineError("room_summaries_enqueue rc=%d" % rc)


def downtrack_summaries(api, h):
    """lkf_downtrack_summaries: one DT_SUMMARY_DTYPE row per DownTrack handle."""
    n = C.c_uint32()
    rc = api["downtrack_summaries"](h, None, 0, C.byref(n))
    if rc not in (0, -28):
        raise EngineError("downtrack_summaries rc=%d" % rc)
    out = np.zeros(max(1, n.value), dtype=abi.DT_SUMMARY_DTYPE)
    rc = api["downtrack_summaries"](h, out.ctypes.data, n.value, C.byref(n))
    if rc != 0:
        raise EngineError("downtrack_summaries rc=%d" % rc)
    return out[:n.value]


def sender_stats(api, h, dts):
    """lkf_sender_stats_get for each DownTrack handle in `dts`: SENDER_STATS_DTYPE rows."""
    out = np.zeros(len(dts), dtype=abi.SENDER_STATS_DTYPE)
    for i, d in enumerate(dts):
        rc = api["sender_stats_get"](h, int(d), out[i:i + 1].ctypes.data)
        if rc != 0:
            raise EngineError("sender_stats_get(%d) rc=%d" % (d, rc))
    return out


def stream_stats(api, h, sid):
    st = abi.lkf_stream_stats()
    rc = api["stream_stats_get"](h, sid, C.byref(st))
    if rc != 0:
        raise EngineError("stream_stats_get rc=%d" % rc)
    return st.as_tuple()


class Engine:
    """One lkf_engine on one HIP device (one process per GPU)."""

    def __init__(self, device=0, max_tracks=1024, max_downtracks=16384, max_batch_pkts=1 << 16,
                 max_batch_arena=64 << 20, max_out_pkts=1 << 20, max_out_bytes=256 << 20,
                 max_batch_tuples=1 << 21, seq_size=500, lib_path=None):
        self.lib = load_library(lib_path)
        self.api = self.lib.api
        cfg = abi.lkf_cfg(max_tracks=max_tracks, max_downtracks=max_downtracks, max_batch_pkts=max_batch_pkts,
                          seq_size=seq_size, max_batch_arena=max_batch_arena, max_out_bytes=max_out_bytes,
                          max_out_pkts=max_out_pkts, max_batch_tuples=max_batch_tuples)
        self.h = self.lib.lkf_create(device, C.byref(cfg))
        if not self.h:
            raise EngineError("lkf_create failed on HIP device %d (no GPU or out of memory)" % device)

    @classmethod
    def for_trace(cls, trace, device=0, headroom=1.25, extra_dts=0, **kw):
        """Engine sized for a synthetic `workload.Trace` (extra_dts: DownTracks
        added beyond the trace's, e.g. re-subscriptions)."""
        mp = int(trace.max_batch_pkts * headroom) + 64
        return cls(device=device, max_tracks=trace.ntracks + 8, max_downtracks=trace.ndts + 8 + extra_dts,
                   max_batch_pkts=mp, max_batch_arena=int(trace.max_batch_arena * headroom) + 4096,
                   max_batch_tuples=int(trace.max_batch_tuples * headroom) + 1024,
                   max_out_pkts=int(trace.max_batch_tuples * headroom) + 1024,
                   max_out_bytes=int(trace.max_batch_out_bytes * headroom) + (1 << 20), **kw)

    def _chk(self, rc, what):
        if rc != 0:
            raise EngineError("%s rc=%d: %s" % (what, rc, self.lib.lkf_last_error(self.h).decode()))

    def submit(self, pkts, n, arena, arena_len, dd=None):
        """lkf_submit (+ lkf_submit_dd with the batch's lkf_pkt_dd side array)."""
        self._chk(self.lib.lkf_submit(self.h, C.cast(pkts, C.c_void_p), n, C.cast(arena, C.c_void_p), arena_len),
                  "submit")
        if dd is not None:
            self._chk(self.api["submit_dd"](self.h, C.cast(dd, C.c_void_p), n), "submit_dd")

    def submit_device(self, d_pkts, n, d_arena, arena_len):
        self._chk(self.lib.lkf_submit_device(self.h, d_pkts, n, d_arena, arena_len), "submit_device")

    def run(self, stream=None):
        self._chk(self.lib.lkf_run(self.h, stream), "run")

    def ingest(self, raws, n, raw, raw_len):
        """Buffer.calc over a raw batch; the ExtPackets become the next run's batch."""
        rc = self.api["ingest"](self.h, C.cast(raws, C.c_void_p), n, C.cast(raw, C.c_void_p), raw_len)
        if rc != 0:
            raise EngineError("lkf_ingest rc=%d: %s" % (rc, self.lib.lkf_last_error(self.h).decode()))

    def ingest_device(self, d_raws, n, d_raw, raw_len):
        """lkf_ingest with HBM-resident raw datagrams (no host sync)."""
        rc = self.api["ingest_device"](self.h, d_raws, n, d_raw, raw_len)
        if rc != 0:
            raise EngineError("lkf_ingest_device rc=%d: %s" % (rc, self.lib.lkf_last_error(self.h).decode()))

    def flows(self):
        return flows_array(self.api, self.h)

    def stream_stats(self, sid):
        return stream_stats(self.api, self.h, sid)

    def speakers(self, now_ns):
        return speakers_array(self.api, self.h, now_ns)

    def sync(self):
        self._chk(self.lib.lkf_sync(self.h), "sync")

    def stats(self):
        st = abi.lkf_stats()
        self._chk(self.api["get_stats"](self.h, C.byref(st)), "get_stats")
        return st.as_dict()

    def drain(self):
        return drain_arrays(self.api, self.h)

    def drain_run_into(self, age, out_ptr, cap, arena_ptr, arena_cap):
        """lkf_drain_run into caller buffers (e.g. pinned host memory) -> (records, bytes)."""
        n = C.c_uint64()
        alen = C.c_uint64()
        f = self.lib.lkf_drain_run
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        self._chk(f(self.h, age, out_ptr, cap, arena_ptr, arena_cap, C.byref(n), C.byref(alen)), "drain_run")
        return n.value, alen.value

    def drain_run_async(self, age, out_ptr, cap, arena_ptr, arena_cap):
        """lkf_drain_run_async into page-locked buffers: returns (records, bytes)
        once the copies are enqueued; drain_wait() before reading them."""
        n = C.c_uint64()
        alen = C.c_uint64()
        f = self.lib.lkf_drain_run_async
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        self._chk(f(self.h, age, out_ptr, cap, arena_ptr, arena_cap, C.byref(n), C.byref(alen)), "drain_run_async")
        return n.value, alen.value

    def drain_wait(self):
        self.lib.lkf_drain_wait.restype = C.c_int
        self.lib.lkf_drain_wait.argtypes = [C.c_void_p]
        self._chk(self.lib.lkf_drain_wait(self.h), "drain_wait")

    def output_device(self):
        d_out = C.c_void_p()
        d_ar = C.c_void_p()
        n = C.c_uint64()
        alen = C.c_uint64()
        self._chk(self.lib.lkf_output_device(self.h, C.byref(d_out), C.byref(n), C.byref(d_ar), C.byref(alen)),
                  "output_device")
        return d_out.value, n.value, d_ar.value, alen.value

    def timings(self):
        a, b, c = C.c_float(), C.c_float(), C.c_float()
        self._chk(self.lib.lkf_last_timings(self.h, C.byref(a), C.byref(b), C.byref(c)), "timings")
        return a.value, b.value, c.value

    def timing_window(self, n):
        a, b, c = C.c_float(), C.c_float(), C.c_float()
        self._chk(self.lib.lkf_timing_window(self.h, n, C.byref(a), C.byref(b), C.byref(c)), "timing_window")
        return a.value, b.value, c.value

    def cumulative(self, reset=False):
        st = abi.lkf_stats()
        self._chk(self.lib.lkf_get_cumulative(self.h, C.byref(st), 1 if reset else 0), "cumulative")
        return st.as_dict()

    def close(self):
        if self.h:
            self.lib.lkf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
