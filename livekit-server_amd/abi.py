"""ctypes mirror of include/lkfwd.h and csrc/synth.h (plain C structs).

The Python layer is host plumbing only: it loads ``liblkfwd.so`` (the HIP
engine) and ``liblkfsynth.so`` (the synthetic workload generator) and gives the
tests / bench a typed view of the C-ABI.  There is no compute here and no
fallback: a missing library raises.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(HERE, "lib")


class lkf_cfg(C.Structure):
    _fields_ = [
        ("max_tracks", C.c_uint32),
        ("max_downtracks", C.c_uint32),
        ("max_batch_pkts", C.c_uint32),
        ("seq_size", C.c_uint32),
        ("max_batch_arena", C.c_uint64),
        ("max_out_bytes", C.c_uint64),
        ("max_out_pkts", C.c_uint64),
        ("max_batch_tuples", C.c_uint64),
        ("max_streams", C.c_uint32),
        ("reserved_cfg", C.c_uint32),
    ]


class lkf_stream_params(C.Structure):
    _fields_ = [
        ("track", C.c_int32),
        ("layer", C.c_int32),
        ("ssrc", C.c_uint32),
        ("audio_level_ext", C.c_uint8),
        ("active_level", C.c_uint8),
        ("min_percentile", C.c_uint8),
        ("dd_ext", C.c_uint8),
        ("observe_duration_ms", C.c_uint32),
        ("smooth_intervals", C.c_uint32),
        ("nack", C.c_uint8),
        ("twcc_ext", C.c_uint8),
        ("reserved", C.c_uint8 * 2),
        ("rtt_ms", C.c_uint32),
    ]


class lkf_raw_pkt(C.Structure):
    _fields_ = [
        ("arrival_ns", C.c_int64),
        ("stream", C.c_uint32),
        ("off", C.c_uint32),
        ("len", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class lkf_flow(C.Structure):
    _fields_ = [
        ("ext_sn", C.c_uint64),
        ("ext_ts", C.c_uint64),
        ("loss_start", C.c_uint64),
        ("loss_end", C.c_uint64),
        ("pkt", C.c_uint32),
        ("flags", C.c_uint8),
        ("reserved", C.c_uint8 * 3),
    ]


class lkf_stream_stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "ext_start_sn", "ext_highest_sn", "ext_start_ts", "ext_highest_ts", "packets_lost",
        "packets_out_of_order", "packets_duplicate", "packets_padding", "bytes", "header_bytes",
        "bytes_duplicate", "bytes_padding", "frames", "nacks")] + [
            ("initialized", C.c_uint8), ("reserved", C.c_uint8 * 7),
            ("first_time_ns", C.c_int64), ("highest_time_ns", C.c_int64),
            ("last_transit", C.c_uint64), ("last_jitter_ext_ts", C.c_uint64),
            ("jitter", C.c_double), ("max_jitter", C.c_double),
            ("gap_histogram", C.c_uint32 * 101), ("reserved2", C.c_uint32)]

    def as_tuple(self):
        """Every field but the reserved ones (jitter as float64 bits: compared exactly)."""
        import struct
        out = []
        for n, _ in self._fields_:
            if n.startswith("reserved"):
                continue
            v = getattr(self, n)
            if n in ("jitter", "max_jitter"):
                v = struct.unpack("<Q", struct.pack("<d", v))[0]
            elif n == "gap_histogram":
                v = tuple(v)
            out.append(v)
        return tuple(out)


class lkf_speaker(C.Structure):
    _fields_ = [
        ("room", C.c_uint32),
        ("participant", C.c_uint32),
        ("level", C.c_float),
        ("active", C.c_uint32),
    ]


RTCP_NACK_DTYPE = np.dtype([("datagram", "<u4"), ("stream", "<u4"), ("media_ssrc", "<u4"), ("pair_off", "<u4"),
                            ("n_pairs", "<u2"), ("num_nacked", "<u2"), ("reserved", "<u4")])
assert RTCP_NACK_DTYPE.itemsize == 24
NACK_PAIR_DTYPE = np.dtype([("packet_id", "<u2"), ("lost_packets", "<u2")])
FLOW_DTYPE = np.dtype([("ext_sn", "<u8"), ("ext_ts", "<u8"), ("loss_start", "<u8"), ("loss_end", "<u8"),
                       ("pkt", "<u4"), ("flags", "u1"), ("reserved", "V3")])
assert FLOW_DTYPE.itemsize == 40
SPEAKER_DTYPE = np.dtype([("room", "<u4"), ("participant", "<u4"), ("level", "<f4"), ("active", "<u4")])
# lkf_dt_summary (per-DownTrack sendingPacket totals + lastAllocation.IsDeficient)
DT_SUMMARY_DTYPE = np.dtype([("dt", "<i4"), ("subscriber", "<u4"), ("room", "<u4"), ("flags", "<u4"),
                             ("packets_sent", "<u8"), ("bytes_sent", "<u8")])
assert DT_SUMMARY_DTYPE.itemsize == 32
# the cooperative allocation pass (lkf_prov_req / lkf_prov_result / lkf_alloc_group)
PROV_REQ_DTYPE = np.dtype([("dt", "<i4"), ("spatial", "<i4"), ("temporal", "<i4"), ("allow_pause", "u1"),
                           ("allow_overshoot", "u1"), ("reserved", "u1", 2), ("capacity", "<i8")])
assert PROV_REQ_DTYPE.itemsize == 24
PROV_RESULT_DTYPE = np.dtype([("dt", "<i4"), ("is_candidate", "u1"), ("reserved", "u1", 3), ("used", "<i8")])
assert PROV_RESULT_DTYPE.itemsize == 16
ALLOC_GROUP_DTYPE = np.dtype([("first", "<u4"), ("count", "<u4"), ("capacity", "<i8"), ("allow_pause", "u1"),
                              ("allow_overshoot", "u1"), ("reserved", "u1", 6)])
assert ALLOC_GROUP_DTYPE.itemsize == 24
# lkf_dd_tracker_status (StreamTrackerDependencyDescriptor)
DD_TRACKER_STATUS_DTYPE = np.dtype([("tracker", "<i4"), ("max_spatial", "<i4"), ("max_temporal", "<i4"),
                                    ("bitrate_changed", "<u4"), ("notifications", "<u4", (3,)),
                                    ("last_notified", "<i4", (3,)), ("status", "u1", (3,)), ("worker", "u1"),
                                    ("reserved", "<u4"), ("bitrate", "<i8", (3, 4))])
assert DD_TRACKER_STATUS_DTYPE.itemsize == 144
# lkf_sender_stats (DownTrack.rtpStats = buffer.RTPStatsSender)
SENDER_STATS_DTYPE = np.dtype(
    [(f, "<u8") for f in ("ext_start_sn", "ext_highest_sn", "ext_start_ts", "ext_highest_ts")]
    + [("first_time_ns", "<i8"), ("highest_time_ns", "<i8"), ("last_transit", "<u8"), ("last_jitter_ext_ts", "<u8")]
    + [(f, "<u8") for f in ("bytes", "header_bytes", "bytes_duplicate", "header_bytes_duplicate", "bytes_padding",
                            "header_bytes_padding", "packets_duplicate", "packets_padding", "packets_out_of_order",
                            "packets_lost")]
    + [("jitter", "<f8"), ("max_jitter", "<f8")]
    + [(f, "<u4") for f in ("frames", "key_frames", "initialized", "clock_rate")]
    + [("gap_histogram", "<u4", (101,)), ("reserved", "<u4")])
assert SENDER_STATS_DTYPE.itemsize == 584
# NACK -> RTX (lkf_nack / lkf_rtx)
NACK_DTYPE = np.dtype([("dt", "<i4"), ("sn", "<u2"), ("reserved", "<u2")])
assert NACK_DTYPE.itemsize == 8
RTX_DTYPE = np.dtype([("ext_sn", "<u8"), ("ext_ts", "<u8"), ("source_sn", "<u2"), ("target_sn", "<u2"),
                      ("timestamp", "<u4"), ("last_nack", "<u4"), ("marker", "u1"), ("nacked", "u1"), ("layer", "i1"),
                      ("codec_len", "u1"), ("codec", "u1", 8), ("dt", "<i4"), ("reserved", "<u4")])
assert RTX_DTYPE.itemsize == 48
DTS_ACTIVE = 0x1
DTS_DEFICIENT = 0x2
# padding / blank frames (lkf_pad_req)
PAD_REQ_DTYPE = np.dtype([("dt", "<i4"), ("bytes_to_send", "<u4"), ("flags", "<u4"), ("start_sn", "<u4"),
                          ("start_ts", "<u4"), ("reserved", "<u4")])
assert PAD_REQ_DTYPE.itemsize == 24
ALLOC_REQ_DTYPE = np.dtype([("dt", "<i4"), ("available_layers", "<u4"), ("bitrates", "<i8", (3, 4)),
                            ("allow_overshoot", "u1"), ("reserved", "u1", 7)])
assert ALLOC_REQ_DTYPE.itemsize == 112
ALLOCATION_DTYPE = np.dtype([("dt", "<i4"), ("pause_reason", "<i4"), ("bandwidth_requested", "<i8"),
                             ("bandwidth_delta", "<i8"), ("bandwidth_needed", "<i8"), ("target_spatial", "<i4"),
                             ("target_temporal", "<i4"), ("request_spatial", "<i4"), ("max_spatial", "<i4"),
                             ("max_temporal", "<i4"), ("is_deficient", "u1"), ("boosted", "u1"),
                             ("reserved", "u1", 2),
                             ("distance_to_desired", "<f8")])
assert ALLOCATION_DTYPE.itemsize == 64
VIDEO_TRANSITION_DTYPE = np.dtype([("dt", "<i4"), ("from_spatial", "<i4"), ("from_temporal", "<i4"),
                                   ("to_spatial", "<i4"), ("to_temporal", "<i4"), ("available", "u1"),
                                   ("reserved", "u1", 3), ("bandwidth_delta", "<i8")])
assert VIDEO_TRANSITION_DTYPE.itemsize == 32
TRACKER_STATUS_DTYPE = np.dtype([("tracker", "<i4"), ("status", "u1"), ("bitrate_changed", "u1"), ("reserved", "u1", 2),
                                 ("notifications", "<u4"), ("reserved2", "<u4"), ("bitrate", "<i8", 4),
                                 ("cumulative", "<i8", 4)])
assert TRACKER_STATUS_DTYPE.itemsize == 80
TRACKER_RESET, TRACKER_PAUSE, TRACKER_STOP = 1, 2, 3
PAD_ON_MUTE = 0x1
PAD_FORCE_MARKER = 0x2
PAD_WRITABLE = 0x4
PAD_RR_SEEN = 0x8


class lkf_track_params(C.Structure):
    _fields_ = [
        ("track_id", C.c_uint64),
        ("room", C.c_uint32),
        ("publisher", C.c_uint32),
        ("kind", C.c_uint8),
        ("codec", C.c_uint8),
        ("has_ref_ts", C.c_uint8),
        ("is_mic", C.c_uint8),
        ("clock_rate", C.c_uint32),
        ("layer_offsets", (C.c_uint32 * 3) * 3),
        ("has_dd", C.c_uint8),
        ("reserved_tp", C.c_uint8 * 3),
    ]


class lkf_downtrack_params(C.Structure):
    _fields_ = [
        ("track", C.c_int32),
        ("subscriber", C.c_uint32),
        ("ssrc", C.c_uint32),
        ("payload_type", C.c_uint8),
        ("ext_dd", C.c_uint8),
        ("ext_playout", C.c_uint8),
        ("ext_abs_send_time", C.c_uint8),
        ("playout_delay", C.c_uint8 * 3),
        ("has_expected_ts", C.c_uint8),
        ("ext_transport_cc", C.c_uint8),
        ("reserved_dp", C.c_uint8 * 3),
        ("bind_time_ns", C.c_int64),
    ]


class lkf_pkt(C.Structure):
    _fields_ = [
        ("ext_sn", C.c_uint64),
        ("ext_ts", C.c_uint64),
        ("arrival_ns", C.c_int64),
        ("arena_off", C.c_uint32),
        ("track", C.c_uint32),
        ("ssrc", C.c_uint32),
        ("payload_off", C.c_uint16),
        ("payload_len", C.c_uint16),
        ("hdr0", C.c_uint8),
        ("hdr1", C.c_uint8),
        ("spatial", C.c_int8),
        ("temporal", C.c_int8),
        ("flags", C.c_uint8),
        ("vp8_first", C.c_uint8),
        ("vp8_bits", C.c_uint8),
        ("vp8_hdr_size", C.c_uint8),
        ("vp8_picture_id", C.c_uint16),
        ("vp8_tl0picidx", C.c_uint8),
        ("vp8_tid", C.c_uint8),
        ("vp8_keyidx", C.c_uint8),
        ("layer", C.c_int8),
        ("audio_level", C.c_uint8),
        ("vp9_bits", C.c_uint8),
        ("reserved", C.c_uint8 * 8),
    ]


class lkf_pkt_dd(C.Structure):
    _fields_ = [
        ("ext_frame_num", C.c_uint64),
        ("ext_key_frame_num", C.c_uint64),
        ("dd_off", C.c_uint16),
        ("dd_len", C.c_uint8),
        ("flags", C.c_uint8),
        ("reserved", C.c_uint32 * 3),
    ]


class lkf_out(C.Structure):
    _fields_ = [
        ("ext_sn", C.c_uint64),
        ("ext_ts", C.c_uint64),
        ("out_off", C.c_uint64),
        ("dt", C.c_uint32),
        ("pkt", C.c_uint32),
        ("out_len", C.c_uint16),
        ("flags", C.c_uint8),
        ("layer", C.c_int8),
        ("reserved", C.c_uint32),
    ]


LKF_DROP_NREASONS = 11
LKF_KIND_AUDIO, LKF_KIND_VIDEO = 0, 1  # enum lkf_kind
LKF_CTL_MUTE, LKF_CTL_PUBMUTE, LKF_CTL_SET_MAX_SPATIAL, LKF_CTL_SET_MAX_TEMPORAL = 1, 2, 3, 4
LKF_CTL_SET_MAX_SEEN_SPATIAL, LKF_CTL_SET_MAX_SEEN_TEMPORAL, LKF_CTL_SET_ALLOCATION = 5, 6, 7
LKF_CTL_RESYNC, LKF_CTL_SET_TARGET, LKF_CTL_PLAYOUT_ACKED = 8, 9, 10


class lkf_stats(C.Structure):
    _fields_ = [
        ("tuples", C.c_uint64),
        ("forwarded", C.c_uint64),
        ("out_bytes", C.c_uint64),
        ("arena_bytes", C.c_uint64),
        ("drops", C.c_uint64 * LKF_DROP_NREASONS),
    ]

    def as_dict(self):
        return {
            "tuples": self.tuples,
            "forwarded": self.forwarded,
            "out_bytes": self.out_bytes,
            "arena_bytes": self.arena_bytes,
            "drops": list(self.drops),
        }


class lkf_fwd_state(C.Structure):
    _fields_ = [
        ("started", C.c_uint8),
        ("last_marker", C.c_uint8),
        ("second_last_marker", C.c_uint8),
        ("has_vp8", C.c_uint8),
        ("reference_layer_spatial", C.c_int32),
        ("pre_start_time_ns", C.c_int64),
        ("ext_first_ts", C.c_uint64),
        ("ref_ts_offset", C.c_uint64),
        ("ext_last_sn", C.c_uint64),
        ("ext_second_last_sn", C.c_uint64),
        ("ext_last_ts", C.c_uint64),
        ("ext_second_last_ts", C.c_uint64),
        ("vp8_ext_last_picture_id", C.c_int32),
        ("vp8_picture_id_used", C.c_uint8),
        ("vp8_last_tl0picidx", C.c_uint8),
        ("vp8_tl0picidx_used", C.c_uint8),
        ("vp8_tid_used", C.c_uint8),
        ("vp8_last_keyidx", C.c_uint8),
        ("vp8_keyidx_used", C.c_uint8),
        ("pad", C.c_uint8 * 2),
    ]

    def as_tuple(self):
        return tuple(getattr(self, f[0]) for f in self._fields_ if f[0] != "pad")


class lkf_transport_params(C.Structure):
    _fields_ = [
        ("master_key", C.c_uint8 * 16),
        ("master_salt", C.c_uint8 * 14),
        ("profile", C.c_uint16),
    ]


LKF_SRTP_AES128_CM_HMAC_SHA1_80 = 1
LKF_SRTP_AEAD_AES_128_GCM = 2
LKF_TWCC_PUSH = 0x80000000
# lkf_flow.flags (LKF_FLOW_*)
LKF_FLOW_NOT_HANDLED, LKF_FLOW_DUPLICATE, LKF_FLOW_OUT_OF_ORDER, LKF_FLOW_HAS_LOSS = 0x01, 0x02, 0x04, 0x08
LKF_FLOW_PADDING, LKF_FLOW_FORWARD, LKF_FLOW_BAD, LKF_FLOW_BUCKET = 0x10, 0x20, 0x40, 0x80
LKF_TWCC_MARKER = 0x00010000
SRTP_TAG_LEN = 10


class lkf_seq_meta(C.Structure):
    _fields_ = [
        ("ext_sn", C.c_uint64),
        ("ext_ts", C.c_uint64),
        ("source_sn", C.c_uint16),
        ("target_sn", C.c_uint16),
        ("timestamp", C.c_uint32),
        ("last_nack", C.c_uint32),
        ("marker", C.c_uint8),
        ("nacked", C.c_uint8),
        ("layer", C.c_int8),
        ("codec_len", C.c_uint8),
        ("codec", C.c_uint8 * 8),
    ]


class lkfs_cfg(C.Structure):
    _fields_ = [
        ("config", C.c_int32),
        ("seed", C.c_uint64),
        ("duration_s", C.c_double),
        ("batch_s", C.c_double),
        ("rooms", C.c_uint32),
        ("participants", C.c_uint32),
        ("room_base", C.c_uint32),
        ("loss", C.c_double),
        ("reorder", C.c_double),
        ("with_events", C.c_int32),
        ("has_callbacks", C.c_int32),
        ("svc_dd", C.c_int32),
        ("h264", C.c_int32),
        ("twcc", C.c_int32),
        ("room_ids", C.POINTER(C.c_uint32)),
    ]


class lkfs_event(C.Structure):
    _fields_ = [
        ("dt", C.c_int32),
        ("op", C.c_int32),
        ("a", C.c_int64 * 4),
        ("at_pkt", C.c_uint32),
        ("pad", C.c_uint32),
    ]


assert C.sizeof(lkf_pkt) == 64, C.sizeof(lkf_pkt)
assert C.sizeof(lkf_pkt_dd) == 32, C.sizeof(lkf_pkt_dd)
assert C.sizeof(lkf_track_params) == 64, C.sizeof(lkf_track_params)
assert C.sizeof(lkf_out) == 40, C.sizeof(lkf_out)

LKF_OUT_SWITCHING, LKF_OUT_RESUMING, LKF_OUT_KEYFRAME, LKF_OUT_MARKER = 0x01, 0x02, 0x04, 0x08  # lkf_out.flags
OUT_DTYPE = np.dtype(
    [("ext_sn", "<u8"), ("ext_ts", "<u8"), ("out_off", "<u8"), ("dt", "<u4"), ("pkt", "<u4"),
     ("out_len", "<u2"), ("flags", "u1"), ("layer", "i1"), ("reserved", "<u4")]
)
assert OUT_DTYPE.itemsize == 40


def _bind(lib, name, restype, argtypes):
    fn = getattr(lib, name)
    fn.restype = restype
    fn.argtypes = argtypes
    return fn


P = C.POINTER


def bind_engine_api(lib, prefix):
    """Binds the lkf_* (engine) or orc_* (oracle) entry points of `lib`."""
    e = C.c_void_p
    api = {}
    api["add_track"] = _bind(lib, prefix + "add_track", C.c_int32, [e, P(lkf_track_params)])
    api["add_downtrack"] = _bind(lib, prefix + "add_downtrack", C.c_int32, [e, P(lkf_downtrack_params)])
    api["remove_downtrack"] = _bind(lib, prefix + "remove_downtrack", C.c_int, [e, C.c_int32])
    api["remove_track"] = _bind(lib, prefix + "remove_track", C.c_int, [e, C.c_int32])
    api["set_layer_offsets"] = _bind(lib, prefix + "set_layer_offsets", C.c_int, [e, C.c_int32, P(C.c_uint32)])
    api["set_layer_offsets_at"] = _bind(lib, prefix + "set_layer_offsets_at", C.c_int,
                                        [e, C.c_int32, P(C.c_uint32), C.c_uint32])
    api["sender_report"] = _bind(lib, prefix + "sender_report", C.c_int,
                                 [e, C.c_int32, C.c_int32, C.c_uint64, C.c_uint32, C.c_uint32])
    api["ctl"] = _bind(lib, prefix + "ctl", C.c_int,
                       [e, C.c_int32, C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_uint32])
    api["ctl_batch"] = _bind(lib, prefix + "ctl_batch", C.c_int, [e, C.c_void_p, C.c_uint32])
    api["get_stats"] = _bind(lib, prefix + "get_stats", C.c_int, [e, P(lkf_stats)])
    if hasattr(lib, prefix + "last_error"):
        api["last_error"] = _bind(lib, prefix + "last_error", C.c_char_p, [e])
    api["drain"] = _bind(lib, prefix + "drain", C.c_int,
                         [e, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, P(C.c_uint64), P(C.c_uint64)])
    api["get_state"] = _bind(lib, prefix + "get_state", C.c_int, [e, C.c_int32, P(lkf_fwd_state)])
    api["seed_state"] = _bind(lib, prefix + "seed_state", C.c_int, [e, C.c_int32, P(lkf_fwd_state)])
    api["seq_lookup"] = _bind(lib, prefix + "seq_lookup", C.c_int,
                              [e, C.c_int32, P(C.c_uint16), C.c_uint32, C.c_int64, P(lkf_seq_meta), P(C.c_uint32)])
    api["add_stream"] = _bind(lib, prefix + "add_stream", C.c_int32, [e, P(lkf_stream_params)])
    api["ingest"] = _bind(lib, prefix + "ingest", C.c_int, [e, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64])
    if hasattr(lib, prefix + "ingest_device"):  # engine only (the oracle is host-side)
        api["ingest_device"] = _bind(lib, prefix + "ingest_device", C.c_int,
                                     [e, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64])
    api["ingest_twcc"] = _bind(lib, prefix + "ingest_twcc", C.c_int, [e, C.c_void_p, C.c_uint32, P(C.c_uint32)])
    api["ingest_flows"] = _bind(lib, prefix + "ingest_flows", C.c_int, [e, C.c_void_p, C.c_uint32, P(C.c_uint32)])
    api["ingested"] = _bind(lib, prefix + "ingested", C.c_int, [e, C.c_void_p, C.c_uint32, P(C.c_uint32)])
    api["ingested_dd"] = _bind(lib, prefix + "ingested_dd", C.c_int, [e, C.c_void_p, C.c_uint32, P(C.c_uint32)])
    api["submit_dd"] = _bind(lib, prefix + "submit_dd", C.c_int, [e, C.c_void_p, C.c_uint32])
    if hasattr(lib, prefix + "submit_dd_device"):  # engine only
        api["submit_dd_device"] = _bind(lib, prefix + "submit_dd_device", C.c_int, [e, C.c_void_p, C.c_uint32])
    if hasattr(lib, prefix + "speakers_enqueue"):
        api["speakers_enqueue"] = _bind(lib, prefix + "speakers_enqueue", C.c_int, [e, C.c_int64])
    if hasattr(lib, prefix + "room_summaries_enqueue"):  # engine only (device records)
        api["room_summaries_enqueue"] = _bind(lib, prefix + "room_summaries_enqueue", C.c_int,
                                              [e, C.c_int64, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                               C.c_void_p, C.c_uint32, C.c_void_p])
    api["stream_stats_get"] = _bind(lib, prefix + "stream_stats_get", C.c_int, [e, C.c_int32, P(lkf_stream_stats)])
    api["ingest_nacks"] = _bind(lib, prefix + "ingest_nacks", C.c_int,
                                [e, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, P(C.c_uint32), P(C.c_uint32)])
    api["stream_set_rtt"] = _bind(lib, prefix + "stream_set_rtt", C.c_int, [e, C.c_int32, C.c_uint32])
    api["speakers"] = _bind(lib, prefix + "speakers", C.c_int, [e, C.c_int64, C.c_void_p, C.c_uint32, P(C.c_uint32)])
    api["downtrack_summaries"] = _bind(lib, prefix + "downtrack_summaries", C.c_int,
                                       [e, C.c_void_p, C.c_uint32, P(C.c_uint32)])
    api["rtx_lookup"] = _bind(lib, prefix + "rtx_lookup", C.c_int,
                              [e, C.c_void_p, C.c_uint32, C.c_int64, C.c_void_p, C.c_uint32, P(C.c_uint32)])
    api["rtx_emit"] = _bind(lib, prefix + "rtx_emit", C.c_int,
                            [e, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                             C.c_uint64, P(C.c_uint32), P(C.c_uint64)])
    api["rtx_emit_bucket"] = _bind(lib, prefix + "rtx_emit_bucket", C.c_int,
                                   [e, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, P(C.c_uint32),
                                    P(C.c_uint64)])
    api["add_transport"] = _bind(lib, prefix + "add_transport", C.c_int32, [e, P(lkf_transport_params)])
    api["set_downtrack_transport"] = _bind(lib, prefix + "set_downtrack_transport", C.c_int, [e, C.c_int32, C.c_int32])
    api["protect"] = _bind(lib, prefix + "protect", C.c_int, [e, C.c_int64])
    api["drain_protected"] = _bind(lib, prefix + "drain_protected", C.c_int, [e, C.c_void_p, C.c_uint64, P(C.c_uint64)])
    if not hasattr(lib, prefix + "padding"):  # (an older build, e.g. an A/B baseline library)
        return api
    api["padding"] = _bind(lib, prefix + "padding", C.c_int,
                           [e, C.c_void_p, C.c_uint32, C.c_int64, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                            P(C.c_uint32), P(C.c_uint64), C.c_void_p])
    if hasattr(lib, prefix + "add_stream_tracker"):
        api["add_stream_tracker"] = _bind(lib, prefix + "add_stream_tracker", C.c_int32,
                                          [e, C.c_int32, C.c_int32, C.c_uint32, C.c_uint32])
        api["stream_tracker_ctl"] = _bind(lib, prefix + "stream_tracker_ctl", C.c_int, [e, C.c_int32, C.c_int32, C.c_int32])
        api["stream_trackers_tick"] = _bind(lib, prefix + "stream_trackers_tick", C.c_int,
                                            [e, C.c_void_p, C.c_uint32, C.c_int, C.c_int64, C.c_void_p])
    if hasattr(lib, prefix + "add_stream_tracker_frame"):
        api["add_stream_tracker_frame"] = _bind(lib, prefix + "add_stream_tracker_frame", C.c_int32,
                                                [e, C.c_int32, C.c_int32, C.c_uint32, C.c_double])
        api["stream_trackers_tick_at"] = _bind(lib, prefix + "stream_trackers_tick_at", C.c_int,
                                               [e, C.c_void_p, C.c_uint32, C.c_int, C.c_int64, C.c_int64, C.c_void_p])
    if hasattr(lib, prefix + "red_encode"):
        for nm in ("red_encode", "red_decode"):
            api[nm] = _bind(lib, prefix + nm, C.c_int,
                            [e, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p,
                             C.c_uint32, C.c_void_p, C.c_uint64, P(C.c_uint32), P(C.c_uint64)])
    if hasattr(lib, prefix + "allocate_optimal"):
        api["allocate_optimal"] = _bind(lib, prefix + "allocate_optimal", C.c_int,
                                        [e, C.c_void_p, C.c_uint32, C.c_void_p])
    if hasattr(lib, prefix + "pause"):
        api["allocate_next_higher"] = _bind(lib, prefix + "allocate_next_higher", C.c_int,
                                            [e, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p])
        api["next_higher_transition"] = _bind(lib, prefix + "next_higher_transition", C.c_int,
                                              [e, C.c_void_p, C.c_uint32, C.c_void_p])
        api["pause"] = _bind(lib, prefix + "pause", C.c_int, [e, C.c_void_p, C.c_uint32, C.c_void_p])
    if hasattr(lib, prefix + "add_stream_tracker_dd"):
        api["add_stream_tracker_dd"] = _bind(lib, prefix + "add_stream_tracker_dd", C.c_int32, [e, C.c_int32])
        api["dd_tracker_ctl"] = _bind(lib, prefix + "dd_tracker_ctl", C.c_int, [e, C.c_int32, C.c_int32, C.c_int32])
        api["dd_trackers_tick"] = _bind(lib, prefix + "dd_trackers_tick", C.c_int,
                                        [e, C.c_void_p, C.c_uint32, C.c_int64, C.c_void_p])
    if hasattr(lib, prefix + "provisional_prepare"):
        api["provisional_prepare"] = _bind(lib, prefix + "provisional_prepare", C.c_int, [e, C.c_void_p, C.c_uint32])
        api["provisional_reset"] = _bind(lib, prefix + "provisional_reset", C.c_int, [e, C.c_void_p, C.c_uint32])
        for nm in ("provisional_allocate", "provisional_cooperative", "provisional_best_weighted",
                   "provisional_commit"):
            api[nm] = _bind(lib, prefix + nm, C.c_int, [e, C.c_void_p, C.c_uint32, C.c_void_p])
        api["allocate_all"] = _bind(lib, prefix + "allocate_all", C.c_int,
                                    [e, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p])
    if hasattr(lib, prefix + "sender_stats_get"):
        api["sender_stats_get"] = _bind(lib, prefix + "sender_stats_get", C.c_int, [e, C.c_int32, C.c_void_p])
        api["sender_sninfo"] = _bind(lib, prefix + "sender_sninfo", C.c_int, [e, C.c_int32, C.c_uint64, P(C.c_uint32)])
        api["sender_stats_seed"] = _bind(lib, prefix + "sender_stats_seed", C.c_int, [e, C.c_int32, C.c_int32])
    api["blank_frames"] = _bind(lib, prefix + "blank_frames", C.c_int,
                                [e, C.c_void_p, C.c_uint32, C.c_int64, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                 P(C.c_uint32), P(C.c_uint64)])
    return api


def load_synth(path=None):
    path = path or os.path.join(LIBDIR, "liblkfsynth.so")
    lib = C.CDLL(path)
    t = C.c_void_p
    _bind(lib, "lkfs_generate", t, [P(lkfs_cfg)])
    _bind(lib, "lkfs_free", None, [t])
    _bind(lib, "lkfs_num_tracks", C.c_uint32, [t])
    _bind(lib, "lkfs_num_downtracks", C.c_uint32, [t])
    _bind(lib, "lkfs_tracks", P(lkf_track_params), [t])
    _bind(lib, "lkfs_downtracks", P(lkf_downtrack_params), [t])
    _bind(lib, "lkfs_num_batches", C.c_uint32, [t])
    _bind(lib, "lkfs_batch", C.c_int,
          [t, C.c_uint32, P(P(lkf_pkt)), P(C.c_uint32), P(P(C.c_uint8)), P(C.c_uint64)])
    _bind(lib, "lkfs_batch_events", C.c_int, [t, C.c_uint32, P(P(lkfs_event)), P(C.c_uint32)])
    _bind(lib, "lkfs_total_pkts", C.c_uint64, [t])
    _bind(lib, "lkfs_total_arena", C.c_uint64, [t])
    _bind(lib, "lkfs_max_batch_pkts", C.c_uint32, [t])
    _bind(lib, "lkfs_max_batch_arena", C.c_uint64, [t])
    _bind(lib, "lkfs_max_batch_tuples", C.c_uint64, [t])
    _bind(lib, "lkfs_max_batch_out_bytes", C.c_uint64, [t])
    _bind(lib, "lkfs_num_streams", C.c_uint32, [t])
    _bind(lib, "lkfs_streams", P(lkf_stream_params), [t])
    _bind(lib, "lkfs_batch_raw", C.c_int, [t, C.c_uint32, P(P(lkf_raw_pkt)), P(C.c_uint32)])
    _bind(lib, "lkfs_batch_dd", C.c_int, [t, C.c_uint32, P(P(lkf_pkt_dd)), P(C.c_uint32)])
    return lib
