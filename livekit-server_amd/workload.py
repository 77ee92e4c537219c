"""Synthetic workloads (BASELINE.json configs) through the C generator.

`Trace` wraps csrc/synth.cpp: topology, ExtPacket batches and scripted control
events, deterministic for a given (config, seed).  `load_topology` and
`queue_events` push a trace into anything exposing the lkf_* shaped API
(the MI355X engine, or — in tests only — the oracle), so both receive
byte-identical inputs.
"""
import ctypes as C

from . import abi


class Trace:
    def __init__(self, config, duration_s=10.0, batch_s=1.0, rooms=0, participants=0, room_base=0,
                 loss=-1.0, reorder=-1.0, with_events=-1, has_callbacks=-1, seed=0, svc_dd=-1, h264=0, room_ids=None,
                 synth_lib=None, twcc=0):
        self.lib = synth_lib or abi.load_synth()
        cfg = abi.lkfs_cfg(config=config, seed=seed, duration_s=duration_s, batch_s=batch_s, rooms=rooms,
                           participants=participants, room_base=room_base, loss=loss, reorder=reorder,
                           with_events=with_events, has_callbacks=has_callbacks, svc_dd=svc_dd, h264=h264,
                           twcc=twcc)
        if room_ids is not None:  # a bin-packed shard (rooms.plan_room_shards)
            self._room_ids = (C.c_uint32 * max(1, len(room_ids)))(*room_ids)
            cfg.room_ids = self._room_ids
            cfg.rooms = len(room_ids)
        self.config = config
        self.h = self.lib.lkfs_generate(C.byref(cfg))
        if not self.h:
            raise ValueError("lkfs_generate failed for config %r" % config)
        self.ntracks = self.lib.lkfs_num_tracks(self.h)
        self.ndts = self.lib.lkfs_num_downtracks(self.h)
        self.tracks = self.lib.lkfs_tracks(self.h)
        self.downtracks = self.lib.lkfs_downtracks(self.h)
        self.nbatches = self.lib.lkfs_num_batches(self.h)
        self.total_pkts = self.lib.lkfs_total_pkts(self.h)
        self.total_arena = self.lib.lkfs_total_arena(self.h)
        self.max_batch_pkts = self.lib.lkfs_max_batch_pkts(self.h)
        self.max_batch_arena = self.lib.lkfs_max_batch_arena(self.h)
        self.max_batch_tuples = self.lib.lkfs_max_batch_tuples(self.h)
        self.max_batch_out_bytes = self.lib.lkfs_max_batch_out_bytes(self.h)
        self.nstreams = self.lib.lkfs_num_streams(self.h)
        self.streams = self.lib.lkfs_streams(self.h)

    def batch(self, b):
        pk = C.POINTER(abi.lkf_pkt)()
        n = C.c_uint32()
        ar = C.POINTER(C.c_uint8)()
        alen = C.c_uint64()
        rc = self.lib.lkfs_batch(self.h, b, C.byref(pk), C.byref(n), C.byref(ar), C.byref(alen))
        if rc != 0:
            raise IndexError(b)
        return pk, n.value, ar, alen.value

    def batch_dd(self, b):
        """Batch b's lkf_pkt_dd side array (pointer, n) — parallel to batch(b)."""
        dd = C.POINTER(abi.lkf_pkt_dd)()
        n = C.c_uint32()
        if self.lib.lkfs_batch_dd(self.h, b, C.byref(dd), C.byref(n)) != 0:
            raise IndexError(b)
        return dd, n.value

    def has_dd(self):
        return any(self.tracks[t].has_dd for t in range(self.ntracks))

    def batch_raw(self, b):
        """Batch b as raw datagrams (ingress input): (raw_pkts, n, arena, arena_len)."""
        rp = C.POINTER(abi.lkf_raw_pkt)()
        n = C.c_uint32()
        if self.lib.lkfs_batch_raw(self.h, b, C.byref(rp), C.byref(n)) != 0:
            raise IndexError(b)
        _, _, ar, alen = self.batch(b)
        return rp, n.value, ar, alen

    def events(self, b):
        ev = C.POINTER(abi.lkfs_event)()
        n = C.c_uint32()
        rc = self.lib.lkfs_batch_events(self.h, b, C.byref(ev), C.byref(n))
        if rc != 0:
            raise IndexError(b)
        return [ev[i] for i in range(n.value)]

    def close(self):
        if self.h:
            self.lib.lkfs_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_topology(api, eng, trace):
    for t in range(trace.ntracks):
        h = api["add_track"](eng, C.byref(trace.tracks[t]))
        if h != t:
            raise RuntimeError("add_track returned %d for track %d" % (h, t))
    for d in range(trace.ndts):
        h = api["add_downtrack"](eng, C.byref(trace.downtracks[d]))
        if h != d:
            raise RuntimeError("add_downtrack returned %d for dt %d" % (h, d))


def load_streams(api, eng, trace):
    """Adds the trace's ingress streams (one per received SSRC) in handle order."""
    for i in range(trace.nstreams):
        h = api["add_stream"](eng, C.byref(trace.streams[i]))
        if h != i:
            raise RuntimeError("add_stream returned %d for stream %d" % (h, i))


def events_ptr(trace, b):
    ev = C.POINTER(abi.lkfs_event)()
    n = C.c_uint32()
    if trace.lib.lkfs_batch_events(trace.h, b, C.byref(ev), C.byref(n)) != 0:
        raise IndexError(b)
    return ev, n.value


def events_at_batch_start(trace):
    """The ingress steps: every scripted control op applies at the start of
    its batch (at_pkt 0).  The workload computes at_pkt as an index into its
    own ExtPacket batch, which in an ingress step exists only after
    Buffer.calc, with other per-track counts (late datagrams, padding):
    there the index would land on another track's packet, and where it lands
    would depend on which rooms share the engine, so engines holding
    different room sets (bench.py's sharded parity gate and CPU baseline)
    would not apply the op at the same point."""
    for b in range(trace.nbatches):
        ev, n = events_ptr(trace, b)
        if n:
            for e in (abi.lkfs_event * n).from_address(C.cast(ev, C.c_void_p).value):
                e.at_pkt = 0


def queue_events(api, eng, trace, b):
    """Queues batch b's scripted control ops (lkfs_event == lkf_ctl_event layout)."""
    ev, n = events_ptr(trace, b)
    if n:
        rc = api["ctl_batch"](eng, C.cast(ev, C.c_void_p), n)
        if rc != 0:
            raise RuntimeError("ctl_batch failed rc=%d" % rc)
