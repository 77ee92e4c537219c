/*
 * lkfwd.h — C-ABI of the MI355X batched RTP forwarding engine (liblkfwd.so).
 *
 * This is the drop-in boundary for livekit-server's per-packet SFU path
 * (reference: /root/reference = suryatmodulus/livekit-server v1.5.2, Go).
 * Each entry point names the reference interface it replaces; the cgo
 * binding a maintainer adds on the Go side is in INTEGRATION.md.
 *
 * Plain C types only: pointers, sizes, fixed-width integers.  No torch types.
 * Return codes: 0 = ok, < 0 = errno-like (LKF_E*).  One engine per GPU,
 * driven by one host thread (the reference's per-Forwarder mutex becomes
 * "one lane per DownTrack, packets of a track processed in order").
 */
#ifndef LKFWD_H_
#define LKFWD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------- */
#define LKF_OK 0
#define LKF_EINVAL (-22)
#define LKF_ENOMEM (-12)
#define LKF_ENOSPC (-28)
#define LKF_ENODEV (-19)
#define LKF_EHIP (-5)
#define LKF_EORDER (-34) /* batch not grouped by track */

/* ---- enums ------------------------------------------------------------- */
enum lkf_kind { LKF_KIND_AUDIO = 0, LKF_KIND_VIDEO = 1 };
/* mime of webrtc.RTPCodecCapability (forwarder.go:269-338) */
enum lkf_codec {
  LKF_CODEC_NONE = 0,
  LKF_CODEC_OPUS = 1,
  LKF_CODEC_VP8 = 2,  /* Simulcast selector + VP8 temporal selector + VP8 munger  forwarder.go:287-294 */
  LKF_CODEC_H264 = 3, /* Simulcast selector                                          :295-300 */
  LKF_CODEC_VP9 = 4,  /* SVC: VP9 selector, or the DD selector with has_dd            :301-316 */
  LKF_CODEC_AV1 = 5   /* SVC: DD selector with has_dd, else Simulcast                 :317-334 */
};

/* Control ops, applied to one DownTrack immediately before the first packet
 * of its track whose batch index >= at_pkt (or at batch end).  Each op is the
 * Forwarder/DownTrack method named beside it (pkg/sfu/forwarder.go).
 * at_pkt indexes the ExtPacket batch the next lkf_run forwards.  When that
 * batch comes from lkf_ingest* (Buffer.calc on the GPU), its ExtPackets exist
 * only after the ingest, so a caller cannot in general name a position inside
 * it: such callers queue their ops at 0 (the batch start) or beyond the batch
 * (its end), which is what bench.py's ingress steps do
 * (workload.events_at_batch_start); an ExtPacket batch the caller submits
 * itself (lkf_submit*) takes any index. */
enum lkf_ctl_op {
  LKF_CTL_MUTE = 1,              /* Mute(a0 muted, a1 isSubscribeMutable)  :377  */
  LKF_CTL_PUBMUTE = 2,           /* PubMute(a0)                            :422  */
  LKF_CTL_SET_MAX_SPATIAL = 3,   /* SetMaxSpatialLayer(a0)                 :454  */
  LKF_CTL_SET_MAX_TEMPORAL = 4,  /* SetMaxTemporalLayer(a0)                :472  */
  LKF_CTL_SET_MAX_SEEN_SPATIAL = 5,  /* SetMaxPublishedLayer(a0)           :241  */
  LKF_CTL_SET_MAX_SEEN_TEMPORAL = 6, /* SetMaxTemporalLayerSeen(a0)        :255  */
  LKF_CTL_SET_ALLOCATION = 7,    /* updateAllocation: a0 target spatial, a1 target temporal,
                                    a2 request spatial, a3 isDeficient   :1353 */
  LKF_CTL_RESYNC = 8,            /* Resync()                               :1384 */
  LKF_CTL_SET_TARGET = 9,        /* vls.SetTarget(a0,a1) (test hook, no resync) */
  LKF_CTL_PLAYOUT_ACKED = 10     /* DownTrack.playoudDelayAcked = a0       downtrack.go:719 */
};

/* Drop reasons (TranslationParams.shouldDrop causes), counted per batch. */
enum lkf_drop {
  LKF_DROP_MUTED = 0,        /* muted || pubMuted                       forwarder.go:1440 */
  LKF_DROP_PAUSED = 1,       /* target layer invalid                    :1687 */
  LKF_DROP_NOT_SELECTED = 2, /* vls.Select !IsSelected                  :1694 */
  LKF_DROP_DOWNGRADE = 3,    /* pause-on-downgrade                      :1709 */
  LKF_DROP_SWITCH = 4,       /* processSourceSwitch error               :1652 */
  LKF_DROP_PADDING = 5,      /* ErrPaddingOnlyPacket                    rtpmunger.go:264 */
  LKF_DROP_DUPLICATE = 6,    /* ErrDuplicatePacket                      rtpmunger.go:270 */
  LKF_DROP_OOO_MISS = 7,     /* ErrOutOfOrderSequenceNumberCacheMiss    rtpmunger.go:226 */
  LKF_DROP_TEMPORAL = 8,     /* ErrFilteredVP8TemporalLayer             vp8.go:266 */
  LKF_DROP_PICID_MISS = 9,   /* ErrOutOfOrderVP8PictureIdCacheMiss      vp8.go:173 */
  LKF_DROP_OTHER = 10,
  LKF_DROP_NREASONS = 11
};

/* ---- engine configuration ---------------------------------------------- */
typedef struct lkf_cfg {
  uint32_t max_tracks;      /* capacity of the track table */
  uint32_t max_downtracks;  /* capacity of the DownTrack table */
  uint32_t max_batch_pkts;  /* max ExtPackets per batch */
  uint32_t seq_size;        /* sequencer ring = PacketBufferSize (config.go:326, default 500) */
  uint64_t max_batch_arena; /* max input arena bytes per batch */
  uint64_t max_out_bytes;   /* output arena capacity per batch */
  uint64_t max_out_pkts;    /* output record capacity per batch */
  uint64_t max_batch_tuples; /* (packet x DownTrack) evaluations per batch (decide slots) */
  uint32_t max_streams;     /* ingress streams (one per received SSRC); 0 = 3 x max_tracks */
  uint32_t reserved_cfg;
} lkf_cfg;

/* One published track (a MediaTrack/WebRTCReceiver, receiver.go:195). */
typedef struct lkf_track_params {
  uint64_t track_id;
  uint32_t room;        /* room index (speaker ranking, room sharding) */
  uint32_t publisher;   /* publisher participant index within the room */
  uint8_t kind;         /* lkf_kind */
  uint8_t codec;        /* lkf_codec */
  uint8_t has_ref_ts;   /* 1: getReferenceLayerRTPTimestamp wired to layer_offsets
                           (streamtrackermanager.go:660-679); 0: nil callback */
  uint8_t is_mic;       /* TrackSource_MICROPHONE (uptrackmanager.go:425) */
  uint32_t clock_rate;
  uint32_t layer_offsets[3][3]; /* layerOffsets[ref][layer]; 0 = unavailable */
  uint8_t has_dd;       /* the receiver negotiated the dependency-descriptor extension
                           (Forwarder.DetermineCodec ddAvailable forwarder.go:278-285):
                           VP9 / AV1 then use videolayerselector.DependencyDescriptor */
  uint8_t reserved_tp[3];
} lkf_track_params;

/* One subscriber DownTrack (NewDownTrack downtrack.go:286 + Bind :362). */
typedef struct lkf_downtrack_params {
  int32_t track;        /* handle from lkf_add_track */
  uint32_t subscriber;  /* subscriber participant index within the room */
  uint32_t ssrc;        /* d.ssrc */
  uint8_t payload_type; /* d.payloadType */
  uint8_t ext_dd;       /* dependencyDescriptorExtID (0 = none) */
  uint8_t ext_playout;  /* playoutDelayExtID */
  uint8_t ext_abs_send_time; /* absSendTimeExtID: 3 placeholder bytes, stamped by the sender */
  uint8_t playout_delay[3];  /* PlayOutDelay.Marshal() bytes (rtpextension/playoutdelay.go:40) */
  uint8_t has_expected_ts;   /* 1: getExpectedRTPTimestamp wired (downtrack.go:1765); 0: nil */
  /* transport-cc extension id (0 = none): with send-side BWE (config.go:119-121) a video
   * subscriber negotiates transport-cc instead of abs-send-time, and pion's TWCC
   * HeaderExtensionInterceptor (transport.go:352-355; pion/interceptor v0.1.25
   * pkg/twcc/header_extension_interceptor.go) appends a 2-byte transport-wide sequence number
   * to every RTP packet the subscriber PeerConnection sends, counted per transport in send
   * order (lkf_set_downtrack_transport binds the DownTrack to its PeerConnection's transport;
   * an unbound DownTrack counts on its own) */
  uint8_t ext_transport_cc;
  uint8_t reserved_dp[3];
  int64_t bind_time_ns;      /* sequencer startTime (sequencer.go:100) on the virtual clock */
} lkf_downtrack_params;

/* ExtPacket descriptor (buffer.ExtPacket, buffer.go:54-64), 64 bytes.
 * A batch is an array of these, grouped by track (each track's packets
 * contiguous, in arrival order), plus one input arena of raw RTP packets. */
typedef struct lkf_pkt {
  uint64_t ext_sn;       /* ExtSequenceNumber (after ingress padding-exclusion adjust) */
  uint64_t ext_ts;       /* ExtTimestamp */
  int64_t arrival_ns;    /* Arrival, virtual clock */
  uint32_t arena_off;    /* offset of the raw RTP packet in the batch arena */
  uint32_t track;        /* track handle */
  uint32_t ssrc;         /* Packet.SSRC */
  uint16_t payload_off;  /* offset of the RTP payload within the raw packet */
  uint16_t payload_len;  /* len(Packet.Payload) (padding excluded) */
  uint8_t hdr0;          /* raw RTP byte 0: V(2) P(1) X(1) CC(4) */
  uint8_t hdr1;          /* raw RTP byte 1: M(1) PT(7) */
  int8_t spatial;        /* VideoLayer.Spatial */
  int8_t temporal;       /* VideoLayer.Temporal */
  uint8_t flags;         /* LKF_PKT_* */
  uint8_t vp8_first;     /* VP8.FirstByte */
  uint8_t vp8_bits;      /* LKF_VP8_* */
  uint8_t vp8_hdr_size;  /* VP8.HeaderSize */
  uint16_t vp8_picture_id;
  uint8_t vp8_tl0picidx;
  uint8_t vp8_tid;
  uint8_t vp8_keyidx;
  int8_t layer;          /* the `layer` argument of TrackSender.WriteRTP (downtrack.go:680);
                            for SVC the packet's spatial layer (receiver.go:667-672) */
  uint8_t audio_level;   /* RFC 6464 level (ingress only) */
  uint8_t vp9_bits;      /* LKF_VP9_*: codecs.VP9Packet flags (valid with LKF_PKT_VP9) */
  uint8_t reserved[8];
} lkf_pkt;

#define LKF_PKT_KEYFRAME 0x01
#define LKF_PKT_VP8 0x02        /* Payload is buffer.VP8 */
#define LKF_PKT_HAS_LEVEL 0x04  /* audio_level valid */
#define LKF_PKT_VP9 0x08        /* Payload is codecs.VP9Packet (spatial/temporal = SID/TID) */
#define LKF_PKT_DD 0x10         /* ExtPacket.DependencyDescriptor != nil (spatial/temporal from
                                   the DD; per-packet metadata in the lkf_pkt_dd side array) */

/* buffer.ExtDependencyDescriptor (buffer/dependencydescriptorparser.go:63-73),
 * 32 B, one per packet of a batch (entries of packets without LKF_PKT_DD are
 * ignored).  The parsed descriptor itself is not passed: the engine reads the
 * DD extension payload from the raw packet (dd_off/dd_len) with the track's
 * current FrameDependencyStructure, as the Go parser did at ingress
 * (DependencyDescriptorExtension.Unmarshal, dependencydescriptorreader.go). */
typedef struct lkf_pkt_dd {
  uint64_t ext_frame_num;      /* ExtFrameNum */
  uint64_t ext_key_frame_num;  /* ExtKeyFrameNum */
  uint16_t dd_off;             /* DD extension payload: offset within the raw RTP packet */
  uint8_t dd_len;              /* and length (1..255) */
  uint8_t flags;               /* LKF_DD_* */
  uint32_t reserved[3];
} lkf_pkt_dd;
#define LKF_DD_STRUCTURE_UPDATED 0x01  /* StructureUpdated */
#define LKF_DD_ACTIVE_UPDATED 0x02     /* ActiveDecodeTargetsUpdated */
#define LKF_DD_INTEGRITY 0x04          /* Integrity (FrameIntegrityChecker) */

/* codecs.VP9Packet flags (pion/rtp v1.8.3 codecs/vp9_packet.go); the first
 * seven are the descriptor's first byte I|P|L|F|B|E|V, U is from the layer
 * indices byte (TID|U|SID|D). */
#define LKF_VP9_I 0x80
#define LKF_VP9_P 0x40
#define LKF_VP9_L 0x20
#define LKF_VP9_F 0x10
#define LKF_VP9_B 0x08
#define LKF_VP9_E 0x04
#define LKF_VP9_V 0x02
#define LKF_VP9_U 0x01

#define LKF_VP8_S 0x01
#define LKF_VP8_I 0x02
#define LKF_VP8_M 0x04
#define LKF_VP8_L 0x08
#define LKF_VP8_T 0x10
#define LKF_VP8_Y 0x20
#define LKF_VP8_K 0x40

/* One forwarded (packet x DownTrack) tuple = one wire packet handed to the
 * pacer (pacer.Packet, pacer/pacer.go:25-39), 40 bytes.  Records are ordered
 * by track handle, then DownTrack handle, then packet (a DownTrack's packets
 * contiguous, in send order; the DownTracks of one track adjacent). */
typedef struct lkf_out {
  uint64_t ext_sn;      /* tp.rtp.extSequenceNumber (munged) */
  uint64_t ext_ts;      /* tp.rtp.extTimestamp (munged) */
  uint64_t out_off;     /* offset of the wire packet in the output arena */
  uint32_t dt;          /* DownTrack handle */
  uint32_t pkt;         /* index of the incoming packet in the batch */
  uint16_t out_len;     /* wire packet length (RTP header + payload) */
  uint8_t flags;        /* LKF_OUT_* */
  int8_t layer;
  uint32_t reserved;
} lkf_out;

#define LKF_OUT_SWITCHING 0x01 /* tp.isSwitching */
#define LKF_OUT_RESUMING 0x02  /* tp.isResuming */
#define LKF_OUT_KEYFRAME 0x04  /* extPkt.KeyFrame */
#define LKF_OUT_MARKER 0x08    /* hdr.Marker */

/* Per-batch counters. */
typedef struct lkf_stats {
  uint64_t tuples;        /* (packet x DownTrack) evaluations */
  uint64_t forwarded;     /* tuples that emitted a wire packet */
  uint64_t out_bytes;     /* sum of out_len */
  uint64_t arena_bytes;   /* output arena bytes used (16-B aligned packets) */
  uint64_t drops[LKF_DROP_NREASONS];
} lkf_stats;

/* Exported Forwarder state: ForwarderState forwarder.go:158-166 with
 * RTPMungerState rtpmunger.go:53-60 and VP8State codecmunger/vp8.go:35-43. */
typedef struct lkf_fwd_state {
  uint8_t started;
  uint8_t last_marker, second_last_marker;
  uint8_t has_vp8;
  int32_t reference_layer_spatial;
  int64_t pre_start_time_ns;
  uint64_t ext_first_ts;
  uint64_t ref_ts_offset;
  uint64_t ext_last_sn, ext_second_last_sn, ext_last_ts, ext_second_last_ts;
  int32_t vp8_ext_last_picture_id;
  uint8_t vp8_picture_id_used, vp8_last_tl0picidx, vp8_tl0picidx_used, vp8_tid_used;
  uint8_t vp8_last_keyidx, vp8_keyidx_used, pad[2];
} lkf_fwd_state;

/* ---- ingress ------------------------------------------------------------
 * One received RTP stream = one buffer.Buffer (buffer.go:66-130, bound by
 * WebRTCReceiver.AddUpTrack receiver.go:320-360): RTPStatsReceiver, the
 * padding-exclusion RangeMap(100), and (audio) the AudioLevel observer. */
typedef struct lkf_stream_params {
  int32_t track;            /* forwarding track handle (lkf_add_track) */
  int32_t layer;            /* receiver layer of this SSRC (RidToSpatialLayer); 0 for audio */
  uint32_t ssrc;
  uint8_t audio_level_ext;  /* negotiated ssrc-audio-level header extension id; 0 = none */
  /* AudioLevelParams (receiver.go:342-347); all zero -> config.go:380-385
   * defaults 35 / 40 / 400 ms / 2 */
  uint8_t active_level;
  uint8_t min_percentile;
  uint8_t dd_ext;           /* negotiated dependency-descriptor extension id (buffer.go:191-201):
                               the stream's DependencyDescriptorParser; 0 = none */
  uint32_t observe_duration_ms;
  uint32_t smooth_intervals;
  /* NACK feedback negotiated for the codec (buffer.go:248-256): the Buffer
   * gets mediatransportutil's NackQueue (NackQueueParamsDefault); 0 = none
   * (audio/red, or no "nack" RTCP feedback) */
  uint8_t nack;
  uint8_t twcc_ext;         /* negotiated transport-cc extension id (buffer.go:238-245, SetTWCC): the
                               datagrams' TWCC responder pushes (lkf_ingest_twcc); 0 = none */
  uint8_t reserved[2];
  uint32_t rtt_ms;          /* initial NackQueue RTT (Buffer.SetRTT); 0 = the queue's default 70 ms */
} lkf_stream_params;

/* One received datagram of a raw batch (24 B).  A raw batch is grouped by
 * track (every packet of a track's streams contiguous, in arrival order),
 * like an ExtPacket batch. */
typedef struct lkf_raw_pkt {
  int64_t arrival_ns;  /* arrival time, virtual clock */
  uint32_t stream;     /* lkf_add_stream handle */
  uint32_t off;        /* offset of the datagram in the raw arena */
  uint32_t len;        /* datagram length */
  uint32_t reserved;
} lkf_raw_pkt;

/* Per-datagram ingress outcome: RTPFlowState (rtpstats_receiver.go:33-45)
 * plus the Buffer.calc disposition (buffer.go:417-491), 40 B. */
typedef struct lkf_flow {
  uint64_t ext_sn;      /* ExtSequenceNumber, after the padding adjustment (buffer.go:464-471) */
  uint64_t ext_ts;      /* ExtTimestamp */
  uint64_t loss_start;  /* NACK range [loss_start, loss_end) when LKF_FLOW_HAS_LOSS */
  uint64_t loss_end;
  uint32_t pkt;         /* index of the ExtPacket produced in the forwarding batch, or 0xffffffff */
  uint8_t flags;        /* LKF_FLOW_* */
  uint8_t reserved[3];
} lkf_flow;
#define LKF_FLOW_NOT_HANDLED 0x01  /* flowState.IsNotHandled */
#define LKF_FLOW_DUPLICATE 0x02    /* flowState.IsDuplicate */
#define LKF_FLOW_OUT_OF_ORDER 0x04 /* flowState.IsOutOfOrder */
#define LKF_FLOW_HAS_LOSS 0x08     /* flowState.HasLoss */
#define LKF_FLOW_PADDING 0x10      /* padding-only packet dropped (buffer.go:439-460) */
#define LKF_FLOW_FORWARD 0x20      /* an ExtPacket was produced (buffer.go:489) */
#define LKF_FLOW_BAD 0x40          /* RTP unmarshal / codec parse / DD parse failed (buffer.go:424,
                                      :613-616, :632): getExtPacket returned nil */
#define LKF_FLOW_BUCKET 0x80       /* stored in the stream's RTX bucket (buffer.go:471): every packet
                                      the bucket takes, an ExtPacket or not */

/* RTPStatsReceiver counters of one stream (rtpstats_receiver.go:76-241). */
typedef struct lkf_stream_stats {
  uint64_t ext_start_sn, ext_highest_sn, ext_start_ts, ext_highest_ts;
  uint64_t packets_lost, packets_out_of_order, packets_duplicate, packets_padding;
  uint64_t bytes, header_bytes, bytes_duplicate, bytes_padding, frames;
  uint64_t nacks;  /* sequence numbers NACKed (rtpStats.UpdateNack(numSeqNumsNacked), buffer.go:682-684) */
  uint8_t initialized;
  uint8_t reserved[7];
  /* rtpStatsBase timing (rtpstats_receiver.go:106-107, :209-213): the first packet's arrival and the
   * arrival of the latest in-order packet that started a new timestamp */
  int64_t first_time_ns, highest_time_ns;
  /* updateJitter (rtpstats_base.go:775-810, receive jitter in RTP clock units, float64) over the
   * in-order and out-of-order non-duplicate packets with a payload, first packet of each timestamp */
  uint64_t last_transit, last_jitter_ext_ts;
  double jitter, max_jitter;
  uint32_t gap_histogram[101]; /* updateGapHistogram (:201): [missing - 1] of in-order gaps, last bin also larger */
  uint32_t reserved2;
} lkf_stream_stats;

/* One RTCP TransportLayerNack a Buffer sent from its deferred doNACKs
 * (buffer.go:417-421, :673-710): NackQueue.Pairs() at the arrival time of
 * the datagram whose calc emitted it (24 B).  Its pairs are n_pairs
 * consecutive lkf_nack_pair entries from pair_off. */
typedef struct lkf_rtcp_nack {
  uint32_t datagram;    /* index in the ingested raw batch */
  uint32_t stream;      /* lkf_add_stream handle */
  uint32_t media_ssrc;  /* SenderSSRC = MediaSSRC = the Buffer's mediaSSRC */
  uint32_t pair_off;
  uint16_t n_pairs;
  uint16_t num_nacked;  /* numSeqNumsNacked */
  uint32_t reserved;
} lkf_rtcp_nack;
typedef struct lkf_nack_pair { /* rtcp.NackPair */
  uint16_t packet_id;
  uint16_t lost_packets; /* bit i: packet_id + i + 1 is lost too */
} lkf_nack_pair;

/* One active speaker (livekit.SpeakerInfo, room.go:254-279), 16 B. */
typedef struct lkf_speaker {
  uint32_t room;
  uint32_t participant;  /* publisher index */
  float level;           /* quantised: ceil(level * 8) / 8 (room.go:274-276) */
  uint32_t active;
} lkf_speaker;

typedef struct lkf_engine lkf_engine;

/* ---- lifecycle ---------------------------------------------------------- */
/* Creates an engine bound to HIP device `hip_device`.  NULL on failure. */
lkf_engine *lkf_create(int hip_device, const lkf_cfg *cfg);
void lkf_destroy(lkf_engine *e);
const char *lkf_last_error(const lkf_engine *e);

/* ---- topology ----------------------------------------------------------- */
/* sfu.NewWebRTCReceiver (receiver.go:195) + Forwarder.DetermineCodec. >=0 handle. */
int32_t lkf_add_track(lkf_engine *e, const lkf_track_params *p);
/* sfu.NewDownTrack + Bind (downtrack.go:286,362) + receiver.AddDownTrack (:410). */
int32_t lkf_add_downtrack(lkf_engine *e, const lkf_downtrack_params *p);
/* DownTrack.Close / receiver.DeleteDownTrack. */
int lkf_remove_downtrack(lkf_engine *e, int32_t dt);
/* Reference-layer timestamp offsets of a simulcast track
 * (StreamTrackerManager.layerOffsets, read by GetReferenceLayerRTPTimestamp
 * streamtrackermanager.go:660-679 on every source switch, forwarder.go:1512-1520).
 * They change as RTCP sender reports arrive; each change is a control op of
 * the track applied at a packet index of the next lkf_run's batch (every
 * DownTrack of the track sees it from packet at_pkt on), with no pipeline
 * drain.
 *   lkf_sender_report: SetRTCPSenderReportData(layer, _, newest) (:603-627):
 *     the newest sender report of `layer` (64-bit NTP timestamp, RTP
 *     timestamp); the offsets it implies for (layer, i) and (i, layer)
 *     (updateLayerOffsetLocked :561-601: reports at most 60 s apart, the other
 *     layer's RTP timestamp carried to the reference's NTP time; 0 -> 1) apply
 *     from packet at_pkt.  NTP times convert as mediatransportutil NtpTime.Time.
 *   lkf_set_layer_offsets_at: the whole [ref][layer] table from packet at_pkt.
 *   lkf_set_layer_offsets: the same from the next batch's first packet. */
int lkf_sender_report(lkf_engine *e, int32_t track, int32_t layer, uint64_t ntp_timestamp, uint32_t rtp_timestamp,
                      uint32_t at_pkt);
int lkf_set_layer_offsets_at(lkf_engine *e, int32_t track, const uint32_t offsets[9], uint32_t at_pkt);
int lkf_set_layer_offsets(lkf_engine *e, int32_t track, const uint32_t offsets[9]);

/* ---- control ------------------------------------------------------------ */
/* Queues a Forwarder control op for the next lkf_run (lkf_ctl_op). */
int lkf_ctl(lkf_engine *e, int32_t dt, int32_t op, int64_t a0, int64_t a1, int64_t a2, int64_t a3,
            uint32_t at_pkt);

/* Bulk form of lkf_ctl (one call per batch of ops; same semantics, in order). */
typedef struct lkf_ctl_event {
  int32_t dt;
  int32_t op;
  int64_t a[4];
  uint32_t at_pkt;
  uint32_t pad;
} lkf_ctl_event;
int lkf_ctl_batch(lkf_engine *e, const lkf_ctl_event *evs, uint32_t n);

/* ---- data --------------------------------------------------------------- */
/* Host batch: copies descriptors + arena to HBM (WebRTCReceiver.forwardRTP
 * receiver.go:635 -> DownTrackSpreader.Broadcast downtrackspreader.go:89).
 * The host buffers are reusable when lkf_submit returns. */
int lkf_submit(lkf_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len);
/* Device-resident batch (pointers into HBM).  The engine reads them
 * asynchronously on its own streams after lkf_run returns: they must stay
 * valid and unmodified until lkf_sync returns (or until the enqueue of the
 * third lkf_run after this one, which waits for this batch's emit stage).
 * The emit kernel reads payloads as aligned 16-B words: the 32 bytes after
 * arena_len must be readable device memory (their content is ignored). */
int lkf_submit_device(lkf_engine *e, const lkf_pkt *d_pkts, uint32_t n, const uint8_t *d_arena,
                      uint64_t arena_len);
/* The lkf_pkt_dd side array of the batch just submitted (n == its packet
 * count); required when the batch has LKF_PKT_DD packets.  Host form copies;
 * device form has the lifetime of lkf_submit_device's buffers. */
int lkf_submit_dd(lkf_engine *e, const lkf_pkt_dd *dd, uint32_t n);
int lkf_submit_dd_device(lkf_engine *e, const lkf_pkt_dd *d_dd, uint32_t n);
/* Runs the batch on `stream` (a hipStream_t, may be NULL): every DownTrack's
 * TrackSender.WriteRTP (downtrack.go:680-760) for every packet of its track.
 * Asynchronous; lkf_sync waits. */
int lkf_run(lkf_engine *e, void *stream);
/* Waits for every queued run and ingest.  Errors are sticky: the first
 * lkf_sync after any failing batch or ingest (however many runs were queued
 * in between) returns its code (LKF_EORDER / LKF_ENOSPC) and clears it.  A
 * DownTrack whose tuple slots overflowed skips that batch (its state does not
 * advance): a batch reported LKF_ENOSPC is not bit-exact. */
int lkf_sync(lkf_engine *e);
/* Batch results (valid after lkf_sync, until the next lkf_run). */
int lkf_get_stats(lkf_engine *e, lkf_stats *out);
/* Copies up to `cap` records and the wire bytes to host memory. */
int lkf_drain(lkf_engine *e, lkf_out *out, uint64_t cap, uint8_t *arena, uint64_t arena_cap, uint64_t *n_out,
              uint64_t *arena_len);
/* Pipelined host output: copies the records and wire bytes of the run `age`
 * runs before the last one (0 = the last, at most 2: the engine keeps three
 * batch contexts) once its emit stage has finished, without waiting for the
 * runs queued after it — a host loop submit(b); run(b); drain_run(1) moves
 * batch b-1's output over PCIe while batch b computes.  Does not report the
 * sticky error word (lkf_sync does).  LKF_EINVAL if that run does not exist. */
int lkf_drain_run(lkf_engine *e, uint32_t age, lkf_out *out, uint64_t cap, uint8_t *arena, uint64_t arena_cap,
                  uint64_t *n_out, uint64_t *arena_len);
/* The same without waiting for the copies: the record count and byte length
 * are read (after that run's emit stage), then the two device -> host copies
 * are enqueued on the engine's copy stream and the call returns, so a caller's
 * next lkf_submit (host -> device) crosses PCIe while they run — both
 * directions at once.  `out` and `arena` must be page-locked and must not be
 * read or reused before lkf_drain_wait returns. */
int lkf_drain_run_async(lkf_engine *e, uint32_t age, lkf_out *out, uint64_t cap, uint8_t *arena, uint64_t arena_cap,
                        uint64_t *n_out, uint64_t *arena_len);
/* Waits for every copy lkf_drain_run_async enqueued. */
int lkf_drain_wait(lkf_engine *e);
/* Device pointers of the output (zero-copy consumer, e.g. an SRTP stage). */
int lkf_output_device(lkf_engine *e, const lkf_out **d_out, uint64_t *n_out, const uint8_t **d_arena,
                      uint64_t *arena_len);

/* ---- state (Forwarder.GetState / SeedState forwarder.go:340-375) -------- */
int lkf_get_state(lkf_engine *e, int32_t dt, lkf_fwd_state *out);
int lkf_seed_state(lkf_engine *e, int32_t dt, const lkf_fwd_state *in);

/* ---- per-subscriber summaries ------------------------ */
/* Per DownTrack since it was added: DownTrack.sendingPacket's counters
 * (downtrack.go:1930-1941: bytesSent += header + payload of every forwarded
 * packet; one RTPStatsSender packet each) and lastAllocation.IsDeficient as
 * of the last lkf_run (LKF_CTL_SET_ALLOCATION a3) — the per-subscriber
 * bandwidth records a node gathers per room.  One entry per DownTrack handle,
 * removed ones included (without LKF_DTS_ACTIVE).  Drains the engine. */
typedef struct lkf_dt_summary {
  int32_t dt;           /* DownTrack handle */
  uint32_t subscriber;  /* lkf_downtrack_params.subscriber */
  uint32_t room;        /* the track's room */
  uint32_t flags;       /* LKF_DTS_* */
  uint64_t packets_sent;
  uint64_t bytes_sent;
} lkf_dt_summary;
#define LKF_DTS_ACTIVE 0x1
#define LKF_DTS_DEFICIENT 0x2
int lkf_downtrack_summaries(lkf_engine *e, lkf_dt_summary *out, uint32_t cap, uint32_t *n_out);

/* ---- sender statistics (DownTrack.rtpStats = buffer.RTPStatsSender) ----- *
 * RTPStatsSender.Update (rtpstats_sender.go:229-432) for every packet
 * DownTrack.sendingPacket accounts (downtrack.go:1930-1959): forwarded
 * packets (packet time = ExtPacket.Arrival; header = the incoming header as
 * getTranslatedRTPHeader keeps it, payload = the forwarded payload), padding
 * (lkf_padding: 12-B header, padding-only), blank frames (lkf_blank_frames:
 * counted as padding) and RTX (lkf_rtx_emit: the bucket packet's header and
 * payload); packet time for the last three = the call's now_ns (lkf_rtx_emit:
 * that of the last lkf_rtx_lookup), the reference's time.Now().  Key frames
 * forwarded: UpdateKeyFrame.  Not kept: startTime / endTime / lastKeyFrame
 * (wall clock) and the RTCP report snapshots.  Waits for queued runs. */
typedef struct lkf_sender_stats {
  uint64_t ext_start_sn, ext_highest_sn, ext_start_ts, ext_highest_ts;
  int64_t first_time_ns, highest_time_ns;
  uint64_t last_transit, last_jitter_ext_ts;
  uint64_t bytes, header_bytes, bytes_duplicate, header_bytes_duplicate, bytes_padding, header_bytes_padding;
  uint64_t packets_duplicate, packets_padding, packets_out_of_order, packets_lost;
  double jitter, max_jitter;
  uint32_t frames, key_frames, initialized, clock_rate;
  uint32_t gap_histogram[101]; /* gapHistogram: [missing - 1], the last bin also counts larger gaps */
  uint32_t reserved;
} lkf_sender_stats;
int lkf_sender_stats_get(lkf_engine *e, int32_t dt, lkf_sender_stats *out);
/* The snInfo ring entry of extended sequence number esn (pktSize | hdrSize << 16
 * | flags << 24, rtpstats_sender.go:42-46), as getIntervalStats reads it. */
int lkf_sender_sninfo(lkf_engine *e, int32_t dt, uint64_t esn, uint32_t *out);
/* RTPStatsSender.Seed (rtpstats_sender.go:173-201; DownTrack.SeedState
 * downtrack.go:1051-1055 on transceiver reuse): dt takes from_dt's statistics,
 * gap histogram and snInfo ring if from_dt's are initialized (clock rate kept). */
int lkf_sender_stats_seed(lkf_engine *e, int32_t dt, int32_t from_dt);

/* ---- sequencer (sequencer.getExtPacketMetas sequencer.go:263, for RTX) --- */
typedef struct lkf_seq_meta {
  uint64_t ext_sn, ext_ts;
  uint16_t source_sn, target_sn;
  uint32_t timestamp;
  uint32_t last_nack;
  uint8_t marker, nacked;
  int8_t layer;
  uint8_t codec_len;
  uint8_t codec[8];
} lkf_seq_meta;
int lkf_seq_lookup(lkf_engine *e, int32_t dt, const uint16_t *sns, uint32_t n, int64_t now_ns,
                   lkf_seq_meta *out, uint32_t *n_out);

/* ---- NACK -> RTX (DownTrack.retransmitPackets downtrack.go:1596-1712) --- */
typedef struct lkf_nack {
  int32_t dt;       /* DownTrack handle */
  uint16_t sn;      /* NACKed (munged, outgoing) sequence number */
  uint16_t reserved;
} lkf_nack;
typedef struct lkf_rtx {
  lkf_seq_meta meta; /* the sequencer record to retransmit (getExtPacketMetas) */
  int32_t dt;
  uint32_t reserved;
} lkf_rtx;
/* Every DownTrack's NACK list in one call (nacks grouped by DownTrack, each
 * list in NACK order; LKF_EORDER otherwise): Forwarder.FilterRTX
 * (forwarder.go:1406-1434, FlagFilterRTX off / FlagFilterRTXLayers on: a
 * deficient DownTrack retransmits nothing while its target is below its
 * current layer, and nothing above its current layer),
 * sequencer.getExtPacketMetas (sequencer.go:263-332; bumps each record's NACK
 * count and time), then the disallowed layers are skipped.  The records are
 * what the host reads from the receiver's bucket (Receiver.ReadRTP(layer,
 * source_sn)).  Waits for queued runs. */
int lkf_rtx_lookup(lkf_engine *e, const lkf_nack *nacks, uint32_t n, int64_t now_ns, lkf_rtx *out, uint32_t cap,
                   uint32_t *n_out);
/* The retransmissions (downtrack.go:1640-1698): src[i] locates record i's
 * source packet (the bucket's raw RTP bytes) in src_arena (len 0: the read
 * failed, no packet); the header gets the sequencer's marker/SN/TS and the
 * DownTrack's SSRC and payload type, a VP8 payload its stored munged
 * descriptor (translateVP8PacketTo), and the pacer's extension block: the
 * sequencer slot's ddBytes under the DownTrack's DD extension id
 * (sequencer.go:198-199, :326; downtrack.go:1684 — lkf_rtx.reserved carries
 * the slot from lkf_rtx_lookup, read while the slot still holds the record, so
 * emit before the next lkf_run), then the abs-send-time placeholder.  Output as
 * lkf_out records (pkt = index of the lkf_rtx) + 16-B aligned wire packets. */
int lkf_rtx_emit(lkf_engine *e, const lkf_rtx *rtx, uint32_t n, const lkf_raw_pkt *src, const uint8_t *src_arena,
                 uint64_t src_len, lkf_out *out, uint8_t *out_arena, uint64_t out_cap, uint32_t *n_out,
                 uint64_t *out_len);
/* The same with the source packets read from the receivers' buckets on the GPU
 * (Receiver.ReadRTP(layer, sourceSeqNo) -> Buffer.GetPacket -> Bucket.GetPacket,
 * receiver.go:559-566, buffer.go:772-784): lkf_ingest stores every packet the
 * Buffer's bucket takes (buffer.go:471, mediatransportutil bucket: video
 * PacketBufferSize = seq_size slots, audio 200, of 1500 bytes) in HBM under
 * its adjusted SN; the record's track buffer of its layer (an SVC track's
 * single buffer) is read, a miss (closed buffer, too new, too old, slot
 * invalid or holding another SN) skips the record.  No host copy of the
 * packets is needed. */
int lkf_rtx_emit_bucket(lkf_engine *e, const lkf_rtx *rtx, uint32_t n, lkf_out *out, uint8_t *out_arena,
                        uint64_t out_cap, uint32_t *n_out, uint64_t *out_len);

/* ---- padding and blank frames ---------------------- *
 * One request per DownTrack per call (distinct DownTracks; LKF_EINVAL
 * otherwise).  Both wait for queued runs and change the DownTrack's
 * Forwarder/sequencer state, so the next lkf_run continues from it.  The
 * facts the engine does not track come with the request (LKF_PAD_*), and so
 * does Forwarder.maybeStart's random start (forwarder.go:1774-1775: SN in
 * [2^15, 2^15 + 2^14), TS in [2^31, 2^31 + 2^30)), used only by a Forwarder
 * that has not started.  Output as lkf_out records (pkt = request index,
 * layer -1) + 16-B aligned wire packets, request order; the pacer's
 * abs-send-time element is a placeholder (TWCC is the sender's). */
typedef struct lkf_pad_req {
  int32_t dt;
  uint32_t bytes_to_send; /* WritePaddingRTP bytesToSend (ignored by lkf_blank_frames) */
  uint32_t flags;         /* LKF_PAD_* */
  uint32_t start_sn;      /* maybeStart's random sequence number (16 bits) */
  uint32_t start_ts;      /* maybeStart's random timestamp */
  uint32_t reserved;
} lkf_pad_req;
#define LKF_PAD_ON_MUTE 0x1      /* WritePaddingRTP paddingOnMute */
#define LKF_PAD_FORCE_MARKER 0x2 /* WritePaddingRTP forceMarker */
#define LKF_PAD_WRITABLE 0x4     /* d.writable (bound and not closed) */
#define LKF_PAD_RR_SEEN 0x8      /* rtpStats.LastReceiverReportTime() is set (an RTCP RR arrived) */
/* DownTrack.WritePaddingRTP (downtrack.go:764-859): video only, the
 * mute/RR/active gates, ceil(bytes / 275) padding-only packets of 255 bytes
 * (Forwarder.GetSnTsForPadding forwarder.go:1798-1813 ->
 * RTPMunger.UpdateAndGetPaddingSnTs rtpmunger.go:288-346), registered with
 * sequencer.pushPadding (sequencer.go:211-261) so NACKs for them are
 * dropped.  bytes_sent[i] = request i's return value (0: nothing sent). */
int lkf_padding(lkf_engine *e, const lkf_pad_req *reqs, uint32_t n, int64_t now_ns, lkf_out *out, uint8_t *arena,
                uint64_t out_cap, uint64_t arena_cap, uint32_t *n_out, uint64_t *arena_len, uint32_t *bytes_sent);
/* One tick of DownTrack.writeBlankFrameRTP (downtrack.go:1307-1401) per
 * request: Forwarder.GetSnTsForBlankFrames(frameRate, 1) (forwarder.go:
 * 1815-1839; 30 fps video, 50 audio; one more packet to end an open frame)
 * and the codec's blank frame — Opus silence, VP8 padding descriptor
 * (GetPadding :1841, VP8.UpdateAndGetPadding vp8.go:304-363) + 8x8 key frame,
 * H.264 STAP-A 2x2 key frame; other codecs send nothing.  Counted by
 * sendingPacket (lkf_downtrack_summaries).  No E2EE trailer. */
int lkf_blank_frames(lkf_engine *e, const lkf_pad_req *reqs, uint32_t n, int64_t now_ns, lkf_out *out, uint8_t *arena,
                     uint64_t out_cap, uint64_t arena_cap, uint32_t *n_out, uint64_t *arena_len);

/* ---- RED for Opus ---------------------------------- *
 * Both take an ExtPacket batch (grouped by track, as lkf_submit) and a map
 * from track handle to the handle of the track the output belongs to (-1:
 * the track's packets are not converted), and return a new ExtPacket batch
 * (in input order, hence grouped by destination track) whose raw packets are
 * the source RTP header followed by the new payload, 16-B aligned in
 * out_arena — ready for lkf_submit on the destination tracks' DownTracks.
 * Per-track state persists across calls.  Waits for queued runs.
 *   lkf_red_encode  RedReceiver (redreceiver.go:58-207): each Opus primary
 *                   becomes a RED packet carrying up to two earlier payloads
 *                   of its track (RFC 2198, block PT 111);
 *   lkf_red_decode  RedPrimaryReceiver (redprimaryreceiver.go:60-269): each
 *                   RED packet yields the packets its blocks recover (lost
 *                   per the 8-packet receive history; SN/TS/PT patched) and
 *                   then its primary (which keeps the RED packet's header, as
 *                   the reference does).  Malformed RED yields nothing. */
int lkf_red_encode(lkf_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len,
                   const int32_t *map, uint32_t map_len, lkf_pkt *out, uint32_t out_cap, uint8_t *out_arena,
                   uint64_t out_arena_cap, uint32_t *n_out, uint64_t *out_arena_len);
int lkf_red_decode(lkf_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len,
                   const int32_t *map, uint32_t map_len, lkf_pkt *out, uint32_t out_cap, uint8_t *out_arena,
                   uint64_t out_arena_cap, uint32_t *n_out, uint64_t *out_arena_len);

/* ---- stream trackers -------------------------------- *
 * StreamTrackerManager's per-spatial-layer packet trackers (streamtracker.go,
 * streamtracker_packet.go), fed by every lkf_run batch as forwardRTP does
 * (receiver.go:686-695: packets of the tracker's layer with a payload; the
 * packet size is header + payload, a padded packet's padding not counted).
 * The worker goroutine's tickers are host-driven: lkf_stream_trackers_tick
 * with check = 1 at each CycleDuration (CheckStatus) and bitrate_elapsed_ns >
 * 0 at each BitrateReportInterval (the bitrate report over that interval).
 * A tracker's worker runs from its first observed packet after a reset until
 * LKF_TRACKER_RESET / PAUSE / STOP; ticks without a live worker change
 * nothing.  The statuses and bitrates feed lkf_allocate_optimal's
 * available_layers and bitrates. */
typedef struct lkf_tracker_status {
  int32_t tracker;
  uint8_t status;          /* StreamStatus: 0 stopped, 1 active */
  uint8_t bitrate_changed; /* onBitrateAvailable fired by this tick's report */
  uint8_t reserved[2];
  uint32_t notifications;  /* onStatusChanged calls since the tracker was added */
  uint32_t reserved2;
  int64_t bitrate[4];      /* per temporal layer, bps (the last report) */
  int64_t cumulative[4];   /* BitrateTemporalCumulative */
} lkf_tracker_status;
#define LKF_TRACKER_RESET 1 /* StreamTracker.Reset */
#define LKF_TRACKER_PAUSE 2 /* StreamTracker.SetPaused(arg) */
#define LKF_TRACKER_STOP 3  /* StreamTracker.Stop */
/* A StreamTrackerPacket(samples_required, cycles_required) for (track, spatial layer). >= 0 handle. */
int32_t lkf_add_stream_tracker(lkf_engine *e, int32_t track, int32_t layer, uint32_t samples_required,
                               uint32_t cycles_required);
int lkf_stream_tracker_ctl(lkf_engine *e, int32_t tracker, int32_t op, int32_t arg);
int lkf_stream_trackers_tick(lkf_engine *e, const int32_t *trackers, uint32_t n, int check, int64_t bitrate_elapsed_ns,
                             lkf_tracker_status *out);
/* A StreamTrackerFrame (streamtracker_frame.go:39-211) for (track, spatial
 * layer): its layer's marker packets give the frame rate, estimated at each
 * CheckStatus over an interval of max(500 ms, 1 / estimated fps, 1 / min_fps)
 * (StreamTrackerFrameConfig.MinFPS, config.go:413-458: 5 for camera, 0.5 for
 * screen share); status stopped when no two frames arrived in it.  Its
 * time.Now() is the virtual clock: the activating packet's arrival, and the
 * now_ns of lkf_stream_trackers_tick_at (the plain tick passes 0).  Same
 * _ctl and tick calls as the packet trackers.  >= 0 handle. */
int32_t lkf_add_stream_tracker_frame(lkf_engine *e, int32_t track, int32_t layer, uint32_t clock_rate, double min_fps);
int lkf_stream_trackers_tick_at(lkf_engine *e, const int32_t *trackers, uint32_t n, int check,
                                int64_t bitrate_elapsed_ns, int64_t now_ns, lkf_tracker_status *out);

/* The dependency-descriptor stream tracker (streamtracker_dd.go:27-289) of an
 * SVC track with the DD extension (StreamTrackerManager.AddDependencyDescriptorTrackers,
 * streamtrackermanager.go:166-186): observed on the GPU with every lkf_run
 * batch's descriptors (k_dd_decode: an updated active-decode-target mask sets
 * the max spatial / temporal layer and notifies the spatial layers that start
 * or stop; each packet's size is added to the bitrate bytes of every decode
 * target its frame is present in).  Its worker (started by the first mask or
 * SetPaused(true)) reports bitrates at host ticks (Duration.Seconds of the
 * elapsed interval).  Status(layer) = active up to the max spatial layer;
 * BitrateTemporalCumulative(layer) = that layer's per-temporal bitrates. */
typedef struct lkf_dd_tracker_status {
  int32_t tracker;
  int32_t max_spatial, max_temporal;
  uint32_t bitrate_changed;   /* bit s: onBitrateAvailable(s) fired by this tick's report */
  uint32_t notifications[3];  /* onStatusChanged calls per spatial layer */
  int32_t last_notified[3];   /* the status passed by the last call per layer (-1: none) */
  uint8_t status[3];          /* Status(layer): 0 stopped, 1 active */
  uint8_t worker;             /* the bitrate worker runs */
  uint32_t reserved;
  int64_t bitrate[3][4];      /* BitrateTemporalCumulative(layer) */
} lkf_dd_tracker_status;
/* >= 0 handle; LKF_EINVAL for a track without the DD selector or a second tracker. */
int32_t lkf_add_stream_tracker_dd(lkf_engine *e, int32_t track);
int lkf_dd_tracker_ctl(lkf_engine *e, int32_t tracker, int32_t op, int32_t arg); /* LKF_TRACKER_PAUSE / _STOP */
int lkf_dd_trackers_tick(lkf_engine *e, const int32_t *trackers, uint32_t n, int64_t bitrate_elapsed_ns,
                         lkf_dd_tracker_status *out);

/* ---- stream allocation ------------------------------ */
typedef struct lkf_alloc_req {
  int32_t dt;
  uint32_t available_layers;  /* bit s = spatial layer s is available (StreamTrackerManager availableLayers) */
  int64_t bitrates[3][4];     /* Bitrates[spatial][temporal], bps (0: not measured / not available) */
  uint8_t allow_overshoot;
  uint8_t reserved[7];
} lkf_alloc_req;
/* VideoAllocation (forwarder.go:82-93) without its Bitrates (the request's). */
typedef struct lkf_allocation {
  int32_t dt;
  int32_t pause_reason; /* VideoPauseReason: 0 none, 1 muted, 2 pub muted, 3 feed dry, 4 bandwidth */
  int64_t bandwidth_requested, bandwidth_delta, bandwidth_needed;
  int32_t target_spatial, target_temporal, request_spatial, max_spatial, max_temporal;
  uint8_t is_deficient;
  uint8_t boosted; /* lkf_allocate_next_higher: a higher layer was allocated */
  uint8_t reserved[2];
  double distance_to_desired;
} lkf_allocation;
/* Forwarder.AllocateOptimal (forwarder.go:591-725) for many DownTracks (one
 * request each, distinct; LKF_EINVAL otherwise), each applied as
 * updateAllocation (:1353-1373: target layer, request spatial, resync when
 * paused, lastAllocation for the next BandwidthDelta) to the state the next
 * lkf_run continues from.  Waits for queued runs.  An audio DownTrack answers
 * VideoAllocationDefault (:111-116).  (LKF_CTL_SET_ALLOCATION, the host-side
 * allocator's result, does not carry bandwidth: it leaves
 * lastAllocation.BandwidthRequested as this call last set it.) */
int lkf_allocate_optimal(lkf_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_allocation *out);
/* Forwarder.AllocateNextHigher (forwarder.go:1107-1217): for each deficient
 * DownTrack whose target layer has been reached, the next higher layer with a
 * bitrate (temporal up, then spatial up, then above the max layer with
 * allow_overshoot on a simulcast selector) if it fits capacity[i] (the
 * availableChannelCapacity) or overshoot is allowed; applied as
 * updateAllocation with boosted = 1.  Otherwise the DownTrack's
 * lastAllocation with boosted = 0.  The lastAllocation returned and kept is
 * the last lkf_allocate_* result, with is_deficient as the last allocation or
 * LKF_CTL_SET_ALLOCATION left it. */
int lkf_allocate_next_higher(lkf_engine *e, const lkf_alloc_req *reqs, const int64_t *capacity, uint32_t n,
                             lkf_allocation *out);
/* VideoTransition (forwarder.go:134-138) */
typedef struct lkf_video_transition {
  int32_t dt;
  int32_t from_spatial, from_temporal, to_spatial, to_temporal;
  uint8_t available; /* GetNextHigherTransition's second result */
  uint8_t reserved[3];
  int64_t bandwidth_delta;
} lkf_video_transition;
/* Forwarder.GetNextHigherTransition (forwarder.go:1219-1306): the probe
 * goal's next layer (streamallocator.go:1350) for each DownTrack; changes no
 * state.  Waits for queued runs. */
int lkf_next_higher_transition(lkf_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_video_transition *out);
/* Forwarder.Pause (forwarder.go:1308-1351): invalid target, pause reason
 * muted / pub muted / feed dry / bandwidth (deficient), applied as
 * updateAllocation. */
int lkf_pause(lkf_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_allocation *out);

/* ---- the stream allocator's cooperative pass (forwarder.go:727-1105) ---- *
 * The Forwarder halves the stream allocator drives (streamallocator.go
 * allocateTrack :880-1010, allocateAllTracks :1092-1178), each for many video
 * DownTracks per call (distinct DownTracks; an audio or removed DownTrack is
 * LKF_EINVAL: the reference's selector is nil for audio).  The provisional
 * state (VideoAllocationProvisional :96-106) lives per DownTrack in HBM
 * between the calls; Commit applies the result as updateAllocation.  Every
 * call waits for queued runs. */
typedef struct lkf_prov_req {
  int32_t dt;
  int32_t spatial, temporal; /* ProvisionalAllocate: the layer tried */
  uint8_t allow_pause, allow_overshoot;
  uint8_t reserved[2];
  int64_t capacity;          /* ProvisionalAllocate: availableChannelCapacity */
} lkf_prov_req;
typedef struct lkf_prov_result {
  int32_t dt;
  uint8_t is_candidate;
  uint8_t reserved[3];
  int64_t used;              /* the bitrate the allocation adds (may be negative) */
} lkf_prov_result;
/* ProvisionalAllocatePrepare(availableLayers, bitrates) :727-743 */
int lkf_provisional_prepare(lkf_engine *e, const lkf_alloc_req *reqs, uint32_t n);
/* ProvisionalAllocateReset :745-750 */
int lkf_provisional_reset(lkf_engine *e, const int32_t *dts, uint32_t n);
/* ProvisionalAllocate(capacity, layer, allowPause, allowOvershoot) :752-794 */
int lkf_provisional_allocate(lkf_engine *e, const lkf_prov_req *reqs, uint32_t n, lkf_prov_result *out);
/* ProvisionalAllocateGetCooperativeTransition(allow_overshoot) :796-929 */
int lkf_provisional_cooperative(lkf_engine *e, const lkf_prov_req *reqs, uint32_t n, lkf_video_transition *out);
/* ProvisionalAllocateGetBestWeightedTransition :931-1025 */
int lkf_provisional_best_weighted(lkf_engine *e, const int32_t *dts, uint32_t n, lkf_video_transition *out);
/* ProvisionalAllocateCommit :1027-1105 (+ updateAllocation) */
int lkf_provisional_commit(lkf_engine *e, const int32_t *dts, uint32_t n, lkf_allocation *out);
/* allocateAllTracks' managed-track pass (streamallocator.go:1147-1172) for
 * many subscribers at once: per group (one subscriber's stream allocator, its
 * DownTracks reqs[first .. first + count) in priority order), Prepare each,
 * then for every layer (0,0) .. (2,3) and every DownTrack in order
 * ProvisionalAllocate(capacity, layer, allow_pause, allow_overshoot) with
 * capacity -= used (floored at 0), then Commit each -> out[first + k].  One
 * thread per subscriber on the GPU (the pass is serial within one). */
typedef struct lkf_alloc_group {
  uint32_t first, count;
  int64_t capacity;          /* availableChannelCapacity after the exempt tracks */
  uint8_t allow_pause, allow_overshoot;
  uint8_t reserved[6];
} lkf_alloc_group;
int lkf_allocate_all(lkf_engine *e, const lkf_alloc_group *groups, uint32_t ngroups, const lkf_alloc_req *reqs,
                     uint32_t n, lkf_allocation *out);

/* ---- SRTP protect ----------------------------------- *
 * The step after the pacer: writeRTPHeaderExtensions sets abs-send-time
 * (pacer/base.go:71-100), then WriteStream.WriteRTP (base.go:59) protects the
 * packet with the subscriber transport's SRTP context: pion/srtp/v2 v2.0.18
 * (go.mod:87) Context.EncryptRTP, profile SRTP_AES128_CM_HMAC_SHA1_80
 * (RFC 3711: AES-CM keystream, HMAC-SHA1 80-bit tag over header || payload ||
 * ROC, sender rollover counter per SSRC).  A transport is one subscriber
 * PeerConnection's DTLS-SRTP context (its exported master key and salt); its
 * DownTracks are its SSRCs. */
#define LKF_SRTP_AES128_CM_HMAC_SHA1_80 1
/* AEAD_AES_128_GCM (RFC 7714; pion srtp_cipher_aead_aes_gcm.go): 12-byte
 * master salt (master_salt[0..11]), IV = (0^16 || SSRC || ROC || SEQ) XOR the
 * session salt, AAD = the RTP header, a 16-byte tag after the ciphertext */
#define LKF_SRTP_AEAD_AES_128_GCM 2
typedef struct lkf_transport_params {
  uint8_t master_key[16];
  uint8_t master_salt[14];
  uint16_t profile; /* LKF_SRTP_* */
} lkf_transport_params;
/* Adds a transport (session keys derived on the GPU: RFC 3711 §4.3.1). */
int32_t lkf_add_transport(lkf_engine *e, const lkf_transport_params *p);
/* Binds a DownTrack's packets to a transport (-1: none, its packets are
 * copied unprotected).  Binding starts a fresh rollover state for its SSRC.
 * The transport is also the DownTrack's PeerConnection for send-side TWCC:
 * the DownTracks bound to one transport share its transport-wide sequence
 * counter (pkg/rtc/transport.go:352-355). */
int lkf_set_downtrack_transport(lkf_engine *e, int32_t dt, int32_t transport);
/* Protects the last lkf_run's output (asynchronously, after its emit stage):
 * every packet gets the abs-send-time of `send_time_ns` (unix ns, pion/rtp
 * NewAbsSendTimeExtension) in its abs-send-time element, and the packets of a
 * bound DownTrack are SRTP-protected.  Record i's packet is at
 * out_off + 16 * i of the protected arena, out_len (+ 10 with an AES-CM
 * transport, + 16 with GCM) bytes long.  Valid until the run after next is enqueued, like the output. */
int lkf_protect(lkf_engine *e, int64_t send_time_ns);
int lkf_output_protected_device(lkf_engine *e, const uint8_t **d_arena, uint64_t *arena_len);
int lkf_drain_protected(lkf_engine *e, uint8_t *arena, uint64_t cap, uint64_t *arena_len);

/* ---- ingress ------------------------------------------------------------ */
/* Adds one received stream (NewBuffer + Bind, buffer.go:124-215). */
int32_t lkf_add_stream(lkf_engine *e, const lkf_stream_params *p);
/* Buffer.calc (buffer.go:417-491) for a raw batch: RTP unmarshal, header
 * extensions (audio level -> AudioLevel.Observe, buffer.go:573-596),
 * RTPStatsReceiver.Update, NACK loss ranges, padding exclusion, and
 * getExtPacket (buffer.go:599-671).  The ExtPackets produced become the batch
 * of the next lkf_run (the raw arena is the forwarding arena; it must stay
 * valid until that batch's outputs are drained).  Host buffers are copied. */
int lkf_ingest(lkf_engine *e, const lkf_raw_pkt *pkts, uint32_t n, const uint8_t *raw, uint64_t raw_len);
/* Same with device-resident inputs: they must stay valid and unmodified until
 * lkf_sync returns after the lkf_run that forwards them, and the 32 bytes
 * after raw_len must be readable (see lkf_submit_device).  Ingest is enqueued
 * on the engine's prep stream without a host sync: the inputs must be
 * complete when it is called (produced on a synchronized stream).  The
 * ExtPacket count stays on the device and feeds the next lkf_run directly;
 * lkf_ingest_flows / lkf_ingested synchronize. */
int lkf_ingest_device(lkf_engine *e, const lkf_raw_pkt *d_pkts, uint32_t n, const uint8_t *d_raw,
                      uint64_t raw_len);
/* Per-datagram outcomes of the last ingest (input order). */
int lkf_ingest_flows(lkf_engine *e, lkf_flow *out, uint32_t cap, uint32_t *n_out);
/* The ExtPacket batch produced by the last ingest (host copy; the RTX bucket
 * and the host-side stream trackers read it). */
int lkf_ingested(lkf_engine *e, lkf_pkt *out, uint32_t cap, uint32_t *n_out);
/* The TWCC responder's input of the last ingest (processHeaderExtensions,
 * buffer.go:569-576): every datagram that unmarshals, on a stream with a
 * twcc_ext, whose header carries that element (GetExtension: the first
 * element with the id) is pushed as twcc.Responder.Push(BigEndian SN of the
 * element's first two bytes, arrival, marker) — padding-only, duplicate and
 * out-of-order datagrams included, before any stream-state decision.  out[i]
 * is datagram i's word: LKF_TWCC_PUSH | (marker ? LKF_TWCC_MARKER : 0) | SN,
 * or 0 (no push; an element shorter than two bytes, which the reference's
 * ext[0:2] would not survive, is not pushed).  The caller feeds the pushes to
 * its Responder in datagram order with its own arrival times (the Responder
 * builds the RTCP TransportLayerCC at control rate: mediatransportutil, out of
 * the path).  Replaces the per-packet b.twcc.Push call. */
#define LKF_TWCC_PUSH 0x80000000u
#define LKF_TWCC_MARKER 0x00010000u
int lkf_ingest_twcc(lkf_engine *e, uint32_t *out, uint32_t cap, uint32_t *n_out);
/* Its lkf_pkt_dd side array (same order and count as lkf_ingested). */
int lkf_ingested_dd(lkf_engine *e, lkf_pkt_dd *out, uint32_t cap, uint32_t *n_out);
int lkf_stream_stats_get(lkf_engine *e, int32_t stream, lkf_stream_stats *out);
/* The RTCP NACKs the last ingest's Buffer.calc calls emitted, in datagram
 * order (at most one per datagram), and their pairs in the same order.
 * n_out / n_pairs_out are set even when a capacity is too small (LKF_ENOSPC).
 * Replaces the onRtcpFeedback(TransportLayerNack) calls of Buffer.doNACKs
 * (buffer.go:673-686). */
int lkf_ingest_nacks(lkf_engine *e, lkf_rtcp_nack *out, uint32_t cap, lkf_nack_pair *pairs, uint32_t pair_cap,
                     uint32_t *n_out, uint32_t *n_pairs_out);
/* Buffer.SetRTT (buffer.go:400-414): the NackQueue RTT of a stream from the
 * next ingest on (0 is ignored, as in the reference). */
int lkf_stream_set_rtt(lkf_engine *e, int32_t stream, uint32_t rtt_ms);
/* Removes a published track: WebRTCReceiver.closeTracks (receiver.go:700-716)
 * closes its DownTracks (as lkf_remove_downtrack each) and the Buffers of its
 * streams (Buffer.Close buffer.go:337-352: Write then returns io.EOF, so a
 * datagram of a closed stream is not processed — its flow is
 * LKF_FLOW_NOT_HANDLED and no state changes), and it leaves the speaker
 * ranking (UpTrackManager.RemovePublishedTrack uptrackmanager.go:272).
 * Handles are not reused; the track's packets in later ExtPacket batches
 * reach no DownTrack. */
int lkf_remove_track(lkf_engine *e, int32_t track);
/* Room.GetActiveSpeakers (room.go:254-279) for every room at virtual time
 * now_ns: per participant the loudest active microphone track
 * (UpTrackManager.GetAudioLevel uptrackmanager.go:422-436, AudioLevel.GetLevel
 * audiolevel.go:105-112), sorted by level (ties: participant index), grouped
 * by room in ascending room order. */
int lkf_speakers(lkf_engine *e, int64_t now_ns, lkf_speaker *out, uint32_t cap, uint32_t *n_out);
/* The same ranking enqueued without a host wait (Room.audioUpdateWorker's
 * tick inside a pipelined loop): it runs after the last enqueued ingest and
 * stays in HBM for the summary all-gather. */
int lkf_speakers_enqueue(lkf_engine *e, int64_t now_ns);
/* The room manager's periodic summary (Room.audioUpdateWorker's tick every
 * UpdateInterval, room.go:1278-1316) without a host wait:
 * the ranking at now_ns and every active DownTrack's sendingPacket totals
 * (bytesSent / packets, downtrack.go:1930-1959) with lastAllocation.IsDeficient,
 * packed into the fixed-shape records a cross-GPU all-gather moves, in
 * caller device memory:
 *   spk int32 [rows][k][3]: (participant, float32 bits of the quantised level,
 *       active) ranked as lkf_speakers; participant -1 pads (k <= 64);
 *   bwe int64 [rows][s][5]: (subscriber, packets, bytes, deficient DownTracks,
 *       DownTracks) per subscriber of the room, subscribers ascending (the
 *       first s); subscriber -1 pads;
 * row r is room room_ids[r] (ascending; every room of the engine's tracks
 * must be listed).  Enqueued after the last enqueued ingest and decide; the
 * writes run on `stream` (a hipStream_t), which then orders the caller's
 * collective; the engine's next ranking and decide wait for them. */
int lkf_room_summaries_enqueue(lkf_engine *e, int64_t now_ns, const uint32_t *room_ids, uint32_t rows, int32_t *spk,
                               uint32_t k, int64_t *bwe, uint32_t s, void *stream);

/* ---- introspection ------------------------------------------------------ */
/* Duration of the last batch's decide kernel, emit kernel and whole batch, ms. */
int lkf_last_timings(lkf_engine *e, float *decide_ms, float *emit_ms, float *total_ms);
/* Over the last n runs (n <= 256): sums of the decide-kernel and emit-kernel
 * durations, and the GPU span from the first run's start to the last run's
 * emit end (stages overlap across runs).  HIP events recorded on the engine's
 * decide and emit streams; synchronises on the newest. */
int lkf_timing_window(lkf_engine *e, uint32_t n, float *decide_ms, float *emit_ms, float *total_ms);
/* Over the last n runs, all protected (n <= 256): the sum of the SRTP
 * protect stage spans (k_srtp_roc + k_srtp_protect), ms. */
int lkf_protect_timing_window(lkf_engine *e, uint32_t n, float *protect_ms);
/* Counters accumulated on the GPU over all runs since the last reset. */
int lkf_get_cumulative(lkf_engine *e, lkf_stats *out, int reset);
const char *lkf_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LKFWD_H_ */
