// =============================================================================
//  oracle_engine.cpp — TEST INFRASTRUCTURE ONLY (checker + CPU baseline).
//
//  Drives the lkf_oracle.h restatement with the same topology / batch /
//  control inputs as the MI355X engine (include/lkfwd.h), so that parity
//  tests call both through identically shaped C entry points (orc_* mirrors
//  lkf_*).  Per batch it reproduces, for every packet in order and every
//  DownTrack of its track:
//      DownTrack.WriteRTP            pkg/sfu/downtrack.go:680-760
//        Forwarder.GetTranslationParams   forwarder.go:1436
//        translateVP8PacketTo             downtrack.go:1728-1736
//        getTranslatedRTPHeader           downtrack.go:1714-1726
//        pacer writeRTPHeaderExtensions   pacer/base.go:71-100
//        sequencer.push                   sequencer.go:123-209
//        sendingPacket -> RTPStatsSender  downtrack.go:1930, rtpstats_sender.go:229
//  Output: lkf_out records ordered by track, DownTrack, packet + wire bytes
//  (16-B aligned).
// =============================================================================
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <thread>

#include "bucket_oracle.h"
#include "../include/lkfwd.h"
#include "lkf_oracle.h"
#include "srtp_oracle.h"
#include "red_oracle.h"
#include "tracker_oracle.h"
#include "nack_oracle.h"
#include "sender_oracle.h"
#include <map>

using namespace orc;

namespace {

// StreamTrackerManager.senderReports[layer].newest (streamtrackermanager.go:98-104)
struct OSenderReport {
  bool valid = false;
  u64 ntp = 0;  // mediatransportutil.NtpTime
  u32 rtp = 0;
};
struct OTrack {
  lkf_track_params p;  // p.layer_offsets: StreamTrackerManager.layerOffsets as the batch reaches it
  bool removed = false;  // orc_remove_track
  OSenderReport sr[3];
  u32 queued[3][3] = {};  // layerOffsets after every change queued so far (lkf_sender_report)
  // the structure the DD extension bytes of this track's ExtPackets are read
  // with (the Go parser's r.structure at ingress; replaced by every packet
  // that attaches one) and its decode targets (ProcessFrameDependencyStructure)
  std::shared_ptr<orc_dd::Structure> ddStructure;
  std::vector<DDDecodeTarget> ddTargets;
};

struct OOut {
  lkf_out rec;
  std::vector<u8> bytes;
  u64 sent = 0;  // sendingPacket: hdr.MarshalSize() + len(payload) (downtrack.go:1931-1939)
};

struct ODT {
  lkf_downtrack_params p;
  bool active = true;
  std::unique_ptr<Forwarder> f;
  std::unique_ptr<Sequencer> seq;
  // RTPStatsSender fields read by GetExpectedRTPTimestamp (rtpstats_sender.go:581)
  bool statsInit = false;
  i64 firstTime = 0;
  u64 extStartTS = 0;
  bool playoutAcked = false;
  std::vector<OOut> outs;
  // DownTrack.sendingPacket counters (downtrack.go:1930-1941)
  u64 packetsSent = 0, bytesSent = 0;
  // DownTrack.rtpStats (buffer.NewRTPStatsSender downtrack.go:315)
  orc_ss::RTPStatsSender ss;
  // SRTP: the subscriber transport and this SSRC's rollover state
  int32_t transport = -1;
  u32 ownTwcc = 0;  // transport-wide sequence counter while no transport is bound
  orc_srtp::SSRCState srtp;
};

struct OEv {
  int32_t dt, op;
  int64_t a[4];
  uint32_t at;
};

// One received stream = one buffer.Buffer (buffer.go:66-130).
struct OStream {
  lkf_stream_params p;
  u32 clockRate = 0;
  u8 codec = 0;
  RTPStatsReceiver stats;
  RangeMap<u64, u64> snRangeMap{100};  // buffer.go:134
  std::unique_ptr<AudioLevel> level;   // when the audio-level extension is negotiated (buffer.go:203-205)
  std::unique_ptr<DependencyDescriptorParser> ddParser;  // when the DD extension is negotiated (buffer.go:193-201)
  bool latestTSForAudioLevelInitialized = false;
  u32 latestTSForAudioLevel = 0;
  std::unique_ptr<NackQueue> nacker;  // codecs with NACK feedback (buffer.go:248-256)
  bool closed = false;                // Buffer.Close (buffer.go:337-352)
  std::unique_ptr<orc_bucket::Bucket> bucket;  // the RTX bucket (video PacketBufferSize slots, audio 200)
  u64 nacks = 0;                      // rtpStats.nacks (UpdateNack, rtpstats_base.go:315-324)
};

}  // namespace

struct OTrackOp {  // a track's layerOffsets from packet `at` of the next batch on
  u32 track, at;
  u32 offs[3][3];
};
struct orc_engine {
  u32 seqSize = 500;
  std::vector<OTrack> tracks;
  std::vector<OTrackOp> trackOps;
  std::vector<std::unique_ptr<ODT>> dts;
  std::vector<OEv> pending;
  lkf_stats stats{};
  std::vector<lkf_out> outRecs;
  std::vector<u8> outArena;
  // ingress
  std::vector<std::unique_ptr<OStream>> streams;
  std::vector<lkf_flow> flows;
  std::vector<u32> twcc;  // per datagram TWCC responder push word (LKF_TWCC_*)
  std::vector<lkf_rtcp_nack> nackRecs;  // the last ingest's RTCP NACKs
  std::vector<lkf_nack_pair> nackPairs;
  std::vector<lkf_pkt> ingested;
  std::vector<lkf_pkt_dd> ingestedDD;
  // lkf_pkt_dd side array of the next orc_run (orc_submit_dd)
  std::vector<lkf_pkt_dd> pendingDD;
  // SRTP sessions (one per transport) and the last protected output
  std::vector<orc_srtp::Session> transports;
  std::vector<std::unique_ptr<orc_srtp::SessionGcm>> transportsGcm;
  std::vector<u32> transportTwcc;  // pion TWCC HeaderExtensionInterceptor.nextSequenceNr per PeerConnection  // (null: AES-CM transport)
  std::vector<u8> protArena;
  // RED: per source track (lkf_red_encode / lkf_red_decode)
  std::map<u32, orc_red::RedEncoder> redEnc;
  std::map<u32, orc_red::RedDecoder> redDec;
  // stream trackers: (track, spatial layer) and the tracker
  std::vector<std::pair<u32, i32>> trkKey;
  std::vector<orc_st::Tracker> trk;
  i64 rtxNow = 0;  // now_ns of the last orc_rtx_lookup
  // dependency-descriptor stream trackers: the track and the tracker
  std::vector<u32> ddTrkTrack;
  std::vector<orc_st::DDTracker> ddTrk;
  std::vector<int32_t> trackDDTrk;  // track -> DD tracker (-1 none)
};

static void applyCtl(orc_engine *e, ODT &d, const OEv &ev) {
  Forwarder &f = *d.f;
  switch (ev.op) {
    case LKF_CTL_MUTE:
      f.Mute(ev.a[0] != 0, ev.a[1] != 0);
      break;
    case LKF_CTL_PUBMUTE:
      f.PubMute(ev.a[0] != 0);
      break;
    case LKF_CTL_SET_MAX_SPATIAL:
      f.SetMaxSpatialLayer(i32(ev.a[0]));
      break;
    case LKF_CTL_SET_MAX_TEMPORAL:
      f.SetMaxTemporalLayer(i32(ev.a[0]));
      break;
    case LKF_CTL_SET_MAX_SEEN_SPATIAL:
      f.SetMaxPublishedLayer(i32(ev.a[0]));
      break;
    case LKF_CTL_SET_MAX_SEEN_TEMPORAL:
      f.SetMaxTemporalLayerSeen(i32(ev.a[0]));
      break;
    case LKF_CTL_SET_ALLOCATION:
      if (f.kind == KindVideo) f.SetAllocation(VideoLayer{i32(ev.a[0]), i32(ev.a[1])}, i32(ev.a[2]), ev.a[3] != 0);
      break;
    case LKF_CTL_RESYNC:
      f.Resync();
      break;
    case LKF_CTL_SET_TARGET:
      f.vls.SetTarget(VideoLayer{i32(ev.a[0]), i32(ev.a[1])});
      break;
    case LKF_CTL_PLAYOUT_ACKED:
      d.playoutAcked = ev.a[0] != 0;
      break;
    default:
      break;
  }
  (void)e;
}

static ExtPacket toExt(const lkf_pkt &d, const u8 *arena, const lkf_pkt_dd *dd, OTrack &tr, bool &ok) {
  ok = true;
  ExtPacket p;
  const u8 *raw = arena + d.arena_off;
  p.layer.Spatial = d.spatial;
  p.layer.Temporal = d.temporal;
  p.Arrival = d.arrival_ns;
  p.ExtSequenceNumber = d.ext_sn;
  p.ExtTimestamp = d.ext_ts;
  p.Header.Version = d.hdr0 >> 6;
  p.Header.Padding = (d.hdr0 & 0x20) != 0;
  p.Header.Extension = (d.hdr0 & 0x10) != 0;
  p.Header.Marker = (d.hdr1 & 0x80) != 0;
  p.Header.PayloadType = d.hdr1 & 0x7f;
  p.Header.SequenceNumber = u16(d.ext_sn);  // buffer.go:470
  p.Header.Timestamp = u32(d.ext_ts);
  p.Header.SSRC = d.ssrc;
  int cc = d.hdr0 & 0xf;
  for (int i = 0; i < cc; i++) {
    const u8 *c = raw + 12 + 4 * i;
    p.Header.CSRC.push_back((u32(c[0]) << 24) | (u32(c[1]) << 16) | (u32(c[2]) << 8) | u32(c[3]));
  }
  p.Payload.assign(raw + d.payload_off, raw + d.payload_off + d.payload_len);
  p.KeyFrame = (d.flags & LKF_PKT_KEYFRAME) != 0;
  if (d.flags & LKF_PKT_VP8) {
    p.kind = PayloadVP8;
    VP8 &v = p.vp8;
    v.FirstByte = d.vp8_first;
    v.S = d.vp8_bits & LKF_VP8_S;
    v.I = d.vp8_bits & LKF_VP8_I;
    v.M = d.vp8_bits & LKF_VP8_M;
    v.L = d.vp8_bits & LKF_VP8_L;
    v.T = d.vp8_bits & LKF_VP8_T;
    v.Y = d.vp8_bits & LKF_VP8_Y;
    v.K = d.vp8_bits & LKF_VP8_K;
    v.PictureID = d.vp8_picture_id;
    v.TL0PICIDX = d.vp8_tl0picidx;
    v.TID = d.vp8_tid;
    v.KEYIDX = d.vp8_keyidx;
    v.HeaderSize = d.vp8_hdr_size;
    v.IsKeyFrame = p.KeyFrame;
  } else if (d.flags & LKF_PKT_VP9) {
    p.kind = PayloadVP9;
    VP9Flags &v = p.vp9;
    v.I = d.vp9_bits & LKF_VP9_I;
    v.P = d.vp9_bits & LKF_VP9_P;
    v.L = d.vp9_bits & LKF_VP9_L;
    v.F = d.vp9_bits & LKF_VP9_F;
    v.B = d.vp9_bits & LKF_VP9_B;
    v.E = d.vp9_bits & LKF_VP9_E;
    v.V = d.vp9_bits & LKF_VP9_V;
    v.U = d.vp9_bits & LKF_VP9_U;
  }
  if ((d.flags & LKF_PKT_DD) && dd) {
    // ExtPacket.DependencyDescriptor: the descriptor as the ingress parser read
    // it (DependencyDescriptorExtension.Unmarshal with the track's structure,
    // dependencydescriptorparser.go:86-97), plus the parser's metadata
    auto e = std::make_shared<ExtDD>();
    e->Descriptor = std::make_shared<orc_dd::Descriptor>();
    int nread = 0;
    if (orc_dd::Unmarshal(raw + dd->dd_off, dd->dd_len, tr.ddStructure.get(), *e->Descriptor, nread) != orc_dd::DD_OK) {
      ok = false;
      return p;
    }
    if (e->Descriptor->AttachedStructure) {
      tr.ddStructure = e->Descriptor->AttachedStructure;
      tr.ddTargets = ProcessFrameDependencyStructure(*tr.ddStructure);
    }
    e->DecodeTargets = tr.ddTargets;
    e->StructureUpdated = dd->flags & LKF_DD_STRUCTURE_UPDATED;
    e->ActiveDecodeTargetsUpdated = dd->flags & LKF_DD_ACTIVE_UPDATED;
    e->Integrity = dd->flags & LKF_DD_INTEGRITY;
    e->ExtFrameNum = dd->ext_frame_num;
    e->ExtKeyFrameNum = dd->ext_key_frame_num;
    p.dd = e;
  }
  return p;
}

// pion/interceptor v0.1.25 pkg/twcc HeaderExtensionInterceptor.BindLocalStream
// (added per subscriber PeerConnection with send-side BWE, pkg/rtc/
// transport.go:352-355): every RTP packet written on a stream that negotiated
// transport-cc gets SetExtension(id, TransportCCExtension{uint16(n)}.Marshal())
// with n = atomic.AddUint32(&nextSequenceNr, 1) - 1 of the PeerConnection, in
// send order.  PARITY UNPINNED (no reference test covers it).
static u16 twcc_next(orc_engine *e, ODT &d) {
  u32 &c = d.transport >= 0 ? e->transportTwcc[size_t(d.transport)] : d.ownTwcc;
  return u16(c++);
}
// writes the 2-byte element `id` of a marshalled packet in place (the element
// was set with a placeholder where the pacer path builds the header)
static void twcc_put(u8 *pkt, size_t len, u8 id, u16 v) {
  if (len < 12 || !(pkt[0] & 0x10)) return;
  size_t x = 12 + 4 * size_t(pkt[0] & 0x0f);
  if (x + 4 > len) return;
  const u16 prof = u16((pkt[x] << 8) | pkt[x + 1]);
  const size_t end = x + 4 + 4 * ((size_t(pkt[x + 2]) << 8) | pkt[x + 3]);
  size_t p = x + 4;
  while (p < end && end <= len) {
    if (pkt[p] == 0) {
      p++;
      continue;
    }
    u8 eid;
    size_t l;
    if (prof == 0xBEDE) {
      eid = u8(pkt[p] >> 4);
      l = size_t(pkt[p] & 0x0f) + 1;
      p++;
      if (eid == 15) return;
    } else {
      eid = pkt[p];
      l = pkt[p + 1];
      p += 2;
    }
    if (eid == id && l == 2) {
      pkt[p] = u8(v >> 8);
      pkt[p + 1] = u8(v);
      return;
    }
    p += l;
  }
}

// DownTrack.WriteRTP downtrack.go:680-760 on the virtual clock.
static void writeRTP(orc_engine *e, u32 dtIdx, ODT &d, const ExtPacket &ep, u32 pktIdx, int8_t layer,
                     u32 pd_payload_off) {
  e->stats.tuples++;
  TranslationParams tp;
  Err err = d.f->GetTranslationParams(ep, layer, ep.Arrival, tp);
  (void)err;
  if (tp.shouldDrop) {
    int r = tp.dropReason < 0 ? LKF_DROP_OTHER : tp.dropReason;
    e->stats.drops[r]++;
    return;
  }
  std::vector<u8> payload;
  if (!tp.codecBytes.empty() && ep.kind == PayloadVP8) {
    payload = tp.codecBytes;  // translateVP8PacketTo downtrack.go:1728-1736
    payload.insert(payload.end(), ep.Payload.begin() + ep.vp8.HeaderSize, ep.Payload.end());
  } else {
    payload = ep.Payload;
  }
  RtpHeader hdr = ep.Header;  // getTranslatedRTPHeader downtrack.go:1714-1726
  hdr.PayloadType = d.p.payload_type;
  hdr.Timestamp = u32(tp.rtp.extTimestamp);
  hdr.SequenceNumber = u16(tp.rtp.extSequenceNumber);
  hdr.SSRC = d.p.ssrc;
  if (tp.marker) hdr.Marker = true;
  // pacer Base.writeRTPHeaderExtensions pacer/base.go:71-100: DD bytes
  // (downtrack.go:715-718, skipped when the DownTrack has no DD extension id),
  // playout delay until acked, abs-send-time as a 3-byte placeholder the
  // sender stamps (wall clock excluded from parity)
  hdr.Extension = false;
  hdr.ExtensionProfile = 0;
  hdr.Extensions.clear();
  if (d.p.ext_dd && !tp.ddBytes.empty()) hdr.SetExtension(d.p.ext_dd, tp.ddBytes);
  if (d.p.ext_playout && !d.playoutAcked)
    hdr.SetExtension(d.p.ext_playout, std::vector<u8>(d.p.playout_delay, d.p.playout_delay + 3));
  if (d.p.ext_abs_send_time) hdr.SetExtension(d.p.ext_abs_send_time, std::vector<u8>{0, 0, 0});
  // the TWCC interceptor's element (numbered in send order: orc_run's output pass)
  if (d.p.ext_transport_cc) hdr.SetExtension(d.p.ext_transport_cc, std::vector<u8>{0, 0});
  // sequencer.push downtrack.go:724-735
  i64 arrivalMs = ep.Arrival / 1000000;
  d.seq->push(arrivalMs, ep.ExtSequenceNumber, tp.rtp.extSequenceNumber, tp.rtp.extTimestamp, hdr.Marker, i8(layer),
              tp.codecBytes, tp.ddBytes);
  // sendingPacket -> RTPStatsSender.Update init (rtpstats_sender.go:245-262)
  if (!d.statsInit && !payload.empty()) {
    d.statsInit = true;
    d.firstTime = ep.Arrival;
    d.extStartTS = tp.rtp.extTimestamp;
  }
  // sendingPacket (downtrack.go:737-749, :1930-1959): hdr.MarshalSize() of the
  // translated header (getTranslatedRTPHeader keeps the incoming extensions:
  // the raw header, payload_off bytes), len(payload), packet time = Arrival
  d.ss.Update(ep.Arrival, tp.rtp.extSequenceNumber, tp.rtp.extTimestamp, hdr.Marker, int(pd_payload_off),
              int(payload.size()), 0);
  if (ep.KeyFrame) d.ss.UpdateKeyFrame(1);
  OOut o;
  // getTranslatedRTPHeader keeps the incoming header's extensions: the
  // counted header is the incoming one (the raw header, payload_off bytes)
  o.sent = u64(pd_payload_off) + payload.size();
  hdr.Marshal(o.bytes);
  o.bytes.insert(o.bytes.end(), payload.begin(), payload.end());
  std::memset(&o.rec, 0, sizeof(o.rec));
  o.rec.ext_sn = tp.rtp.extSequenceNumber;
  o.rec.ext_ts = tp.rtp.extTimestamp;
  o.rec.dt = dtIdx;
  o.rec.pkt = pktIdx;
  o.rec.out_len = u16(o.bytes.size());
  o.rec.flags = u8((tp.isSwitching ? LKF_OUT_SWITCHING : 0) | (tp.isResuming ? LKF_OUT_RESUMING : 0) |
                   (ep.KeyFrame ? LKF_OUT_KEYFRAME : 0) | (hdr.Marker ? LKF_OUT_MARKER : 0));
  o.rec.layer = layer;
  e->stats.forwarded++;
  e->stats.out_bytes += o.bytes.size();
  d.outs.push_back(std::move(o));
}

extern "C" {

orc_engine *orc_create(uint32_t seq_size) {
  auto *e = new orc_engine();
  if (seq_size) e->seqSize = seq_size;
  return e;
}
void orc_destroy(orc_engine *e) { delete e; }

int32_t orc_add_track(orc_engine *e, const lkf_track_params *p) {
  OTrack t;
  t.p = *p;
  std::memcpy(t.queued, p->layer_offsets, sizeof(t.queued));
  e->tracks.push_back(t);
  return int32_t(e->tracks.size() - 1);
}

int32_t orc_add_downtrack(orc_engine *e, const lkf_downtrack_params *p) {
  if (p->track < 0 || p->track >= (int)e->tracks.size()) return LKF_EINVAL;
  auto d = std::make_unique<ODT>();
  d->p = *p;
  const lkf_track_params &tp = e->tracks[p->track].p;
  Kind k = tp.kind == LKF_KIND_VIDEO ? KindVideo : KindAudio;
  d->f = std::make_unique<Forwarder>(k);
  Mime m = tp.codec == LKF_CODEC_VP8    ? MimeVP8
           : tp.codec == LKF_CODEC_H264 ? MimeH264
           : tp.codec == LKF_CODEC_VP9  ? MimeVP9
           : tp.codec == LKF_CODEC_AV1  ? MimeAV1
                                        : MimeOpus;
  d->f->DetermineCodec(m, tp.clock_rate, tp.has_dd != 0);
  d->seq = std::make_unique<Sequencer>(int(e->seqSize), k == KindVideo, p->bind_time_ns / 1000000);
  d->ss.clockRate = tp.clock_rate;
  ODT *dp = d.get();
  int32_t track = p->track;
  if (tp.has_ref_ts) {
    // StreamTrackerManager.GetReferenceLayerRTPTimestamp streamtrackermanager.go:660-679
    dp->f->getReferenceLayerRTPTimestamp = [e, track](u32 ts, i32 layer, i32 ref, u32 &out) -> Err {
      if (layer < 0 || layer >= 3 || ref < 0 || ref >= 3) return ErrRefLayerUnavailable;
      if (e->tracks[track].p.codec == LKF_CODEC_VP9 || e->tracks[track].p.codec == LKF_CODEC_AV1) {  // isSVC (:667-671)
        out = ts;
        return OK;
      }
      u32 off = e->tracks[track].p.layer_offsets[ref][layer];
      if (layer != ref && off == 0) return ErrRefLayerUnavailable;
      out = ts + off;
      return OK;
    };
  }
  if (p->has_expected_ts) {
    u32 cr = tp.clock_rate;
    dp->f->getExpectedRTPTimestamp = [dp, cr](i64 at, u64 &out) -> Err {
      if (!dp->statsInit) return ErrExpectedTSUnavailable;
      i64 diff = (at - dp->firstTime) * i64(cr) / 1000000000LL;
      out = dp->extStartTS + u64(diff);
      return OK;
    };
  }
  e->dts.push_back(std::move(d));
  return int32_t(e->dts.size() - 1);
}

int orc_remove_downtrack(orc_engine *e, int32_t dt) {
  if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
  e->dts[dt]->active = false;
  return LKF_OK;
}

// WebRTCReceiver.closeTracks (receiver.go:700-716): the DownTracks close, the
// Buffers close (Write -> io.EOF), the track leaves the speaker ranking
int orc_remove_track(orc_engine *e, int32_t track) {
  if (track < 0 || track >= (int)e->tracks.size()) return LKF_EINVAL;
  e->tracks[track].removed = true;
  for (auto &d : e->dts)
    if (d->p.track == track) d->active = false;
  for (auto &s : e->streams)
    if (s->p.track == track) s->closed = true;
  return LKF_OK;
}

// The offsets change at a packet index of the next batch (the engine's
// control-op semantics; the reference changes them from its RTCP goroutine).
int orc_set_layer_offsets_at(orc_engine *e, int32_t track, const uint32_t *offs, uint32_t at) {
  if (track < 0 || track >= (int)e->tracks.size() || !offs) return LKF_EINVAL;
  OTrackOp op;
  op.track = u32(track);
  op.at = at;
  std::memcpy(op.offs, offs, sizeof(op.offs));
  std::memcpy(e->tracks[track].queued, offs, sizeof(op.offs));
  e->trackOps.push_back(op);
  return LKF_OK;
}
int orc_set_layer_offsets(orc_engine *e, int32_t track, const uint32_t *offs) {
  return orc_set_layer_offsets_at(e, track, offs, 0);
}
// test hook: a track's layerOffsets as the last queued change leaves them (queued = 1)
// or as the last batch left them (queued = 0)
int orc_debug_layer_offsets(orc_engine *e, int32_t track, int queued, uint32_t *out) {
  if (track < 0 || track >= (int)e->tracks.size() || !out) return LKF_EINVAL;
  std::memcpy(out, queued ? &e->tracks[track].queued[0][0] : &e->tracks[track].p.layer_offsets[0][0], 36);
  return LKF_OK;
}

namespace {
// mediatransportutil (v0.0.0-20231213075826-cccbf2b93d3f, ntp.go; not vendored
// in /root/reference) NtpTime.Time() = ntpEpoch.Add(Duration()), Duration():
//   sec := (t >> 32) * 1e9; frac := (t & 0xffffffff) * 1e9; nsec := frac >> 32;
//   if uint32(frac) >= 0x80000000 { nsec++ }; return time.Duration(sec + nsec)
// Two NtpTimes' Time().Sub is the difference of their Durations.
i64 ntpDuration(u64 t) {
  const u64 sec = (t >> 32) * 1000000000ull;
  const u64 frac = (t & 0xFFFFFFFFull) * 1000000000ull;
  u64 nsec = frac >> 32;
  if (u32(frac) >= 0x80000000u) nsec++;
  return i64(sec + nsec);
}
// time.Duration.Seconds
double durSeconds(i64 d) {
  const i64 sec = d / 1000000000LL, nsec = d % 1000000000LL;
  return double(sec) + double(nsec) / 1e9;
}
// updateLayerOffsetLocked streamtrackermanager.go:561-601
void updateLayerOffset(OTrack &t, int ref, int other) {
  const OSenderReport &srRef = t.sr[ref], &srOther = t.sr[other];
  if (!srRef.valid || srRef.ntp == 0 || !srOther.valid || srOther.ntp == 0) return;
  const i64 ntpDiff = ntpDuration(srRef.ntp) - ntpDuration(srOther.ntp);
  if (std::fabs(durSeconds(ntpDiff)) > 60.0) return;  // senderReportThresholdSeconds
  const i64 rtpDiff = ntpDiff * i64(t.p.clock_rate) / 1000000000LL;  // / 1e9 (int64)
  const u32 normalizedOtherTS = srOther.rtp + u32(rtpDiff);
  u32 offset = srRef.rtp - normalizedOtherTS;
  if (offset == 0) offset = 1;
  t.queued[ref][other] = offset;
}
}  // namespace

// SetRTCPSenderReportData streamtrackermanager.go:603-627 (the newest report;
// srFirst only feeds GetCalculatedClockRate, outside the path)
int orc_sender_report(orc_engine *e, int32_t track, int32_t layer, uint64_t ntp, uint32_t rtp, uint32_t at) {
  if (track < 0 || track >= (int)e->tracks.size()) return LKF_EINVAL;
  if (layer < 0 || layer > 2) return LKF_OK;
  OTrack &t = e->tracks[track];
  u32 before[3][3];
  std::memcpy(before, t.queued, sizeof(before));
  t.sr[layer].valid = true;
  t.sr[layer].ntp = ntp;
  t.sr[layer].rtp = rtp;
  for (int i = 0; i < 3; i++) {
    if (i == layer) continue;
    updateLayerOffset(t, layer, i);
    updateLayerOffset(t, i, layer);
  }
  if (std::memcmp(before, t.queued, sizeof(before)) == 0) return LKF_OK;
  return orc_set_layer_offsets_at(e, track, &t.queued[0][0], at);
}

int orc_ctl(orc_engine *e, int32_t dt, int32_t op, int64_t a0, int64_t a1, int64_t a2, int64_t a3, uint32_t at) {
  if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
  e->pending.push_back(OEv{dt, op, {a0, a1, a2, a3}, at});
  return LKF_OK;
}

int orc_ctl_batch(orc_engine *e, const lkf_ctl_event *evs, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    int rc = orc_ctl(e, evs[i].dt, evs[i].op, evs[i].a[0], evs[i].a[1], evs[i].a[2], evs[i].a[3], evs[i].at_pkt);
    if (rc) return rc;
  }
  return LKF_OK;
}

// lkf_submit_dd: the side array of the next batch.
int orc_submit_dd(orc_engine *e, const lkf_pkt_dd *dd, uint32_t n) {
  e->pendingDD.assign(dd, dd + n);
  return LKF_OK;
}

// Runs one batch; pkts grouped by track (lkf_submit contract).
int orc_run(orc_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len) {
  (void)arena_len;
  std::vector<lkf_pkt_dd> dds;
  dds.swap(e->pendingDD);
  std::memset(&e->stats, 0, sizeof(e->stats));
  const u32 ndt = u32(e->dts.size());
  std::vector<std::vector<OEv>> evq(ndt);
  for (auto &ev : e->pending)  // ops for removed DownTracks are dropped (they get no more control calls)
    if (e->dts[ev.dt]->active) evq[ev.dt].push_back(ev);
  e->pending.clear();
  for (auto &q : evq)
    std::stable_sort(q.begin(), q.end(), [](const OEv &a, const OEv &b) { return a.at < b.at; });
  std::vector<size_t> evc(ndt, 0);
  std::vector<std::vector<u32>> trackDts(e->tracks.size());
  for (u32 d = 0; d < ndt; d++) {
    e->dts[d]->outs.clear();
    if (e->dts[d]->active) trackDts[e->dts[d]->p.track].push_back(d);
  }
  // the tracks' layer-offset changes, per track in packet order
  std::vector<std::vector<OTrackOp>> tq(e->tracks.size());
  for (const auto &op : e->trackOps) tq[op.track].push_back(op);
  e->trackOps.clear();
  for (auto &q : tq)
    std::stable_sort(q.begin(), q.end(), [](const OTrackOp &a, const OTrackOp &b) { return a.at < b.at; });
  std::vector<size_t> tqc(e->tracks.size(), 0);
  for (u32 i = 0; i < n; i++) {
    const lkf_pkt &pd = pkts[i];
    if (pd.track >= e->tracks.size()) return LKF_EINVAL;
    bool ok = true;
    ExtPacket ep = toExt(pd, arena, i < dds.size() ? &dds[i] : nullptr, e->tracks[pd.track], ok);
    if (!ok) return LKF_EINVAL;
    // the DD stream tracker's Observe (receiver.go:686-695; streamtracker_dd.go:133-212)
    if (pd.track < e->trackDDTrk.size() && e->trackDDTrk[pd.track] >= 0 && ep.dd && ep.dd->Descriptor) {
      const ExtDD &x = *ep.dd;
      orc_st::DDTracker::DT tg[32];
      int nt = 0;
      for (const auto &t : x.DecodeTargets)
        if (nt < 32) tg[nt++] = {t.Target, t.Layer.Spatial, t.Layer.Temporal};
      uint8_t dtis[32];
      const auto &di = x.Descriptor->FrameDependencies.DTIs;
      const int nd = int(std::min<size_t>(di.size(), 32));
      for (int k = 0; k < nd; k++) dtis[k] = uint8_t(di[k]);
      e->ddTrk[e->trackDDTrk[pd.track]].Observe(int(pd.payload_off) + pd.payload_len, pd.payload_len, true,
                                                x.ActiveDecodeTargetsUpdated, x.Descriptor->hasActiveMask,
                                                x.Descriptor->ActiveDecodeTargetsBitmask, tg, nt, dtis, nd);
    }
    {
      auto &q = tq[pd.track];
      size_t &c = tqc[pd.track];
      for (; c < q.size() && q[c].at <= i; c++) std::memcpy(e->tracks[pd.track].p.layer_offsets, q[c].offs, 36);
    }
    for (u32 d : trackDts[pd.track]) {
      ODT &dt = *e->dts[d];
      while (evc[d] < evq[d].size() && evq[d][evc[d]].at <= i) applyCtl(e, dt, evq[d][evc[d]++]);
      writeRTP(e, d, dt, ep, i, pd.layer, pd.payload_off);
    }
  }
  for (u32 d = 0; d < ndt; d++)
    while (evc[d] < evq[d].size()) applyCtl(e, *e->dts[d], evq[d][evc[d]++]);
  for (size_t t = 0; t < tq.size(); t++)  // changes after the batch's last packet
    for (; tqc[t] < tq[t].size(); tqc[t]++) std::memcpy(e->tracks[t].p.layer_offsets, tq[t][tqc[t]].offs, 36);
  // spatialTracker.Observe after each packet's fan-out (receiver.go:686-695);
  // len(RawPacket) = header + payload (padding not counted, as the engine)
  if (!e->trk.empty())
    for (u32 i = 0; i < n; i++)
      for (size_t k = 0; k < e->trk.size(); k++)
        if (e->trkKey[k].first == pkts[i].track && e->trkKey[k].second == pkts[i].layer)
          e->trk[k].Observe(pkts[i].temporal, int(pkts[i].payload_off) + pkts[i].payload_len, pkts[i].payload_len,
                            (pkts[i].hdr1 & 0x80) != 0, u32(pkts[i].ext_ts), pkts[i].arrival_ns);
  for (u32 d = 0; d < ndt; d++)  // sendingPacket: bytesSent += hdrSize + payloadSize
    for (auto &o : e->dts[d]->outs) {
      e->dts[d]->packetsSent++;
      e->dts[d]->bytesSent += o.sent;
    }
  // Output order: by track, then DownTrack handle, then packet; wire packets
  // 16-B aligned.  (An engine-defined batch layout: the reference hands each
  // packet to its DownTrack's pacer directly.)
  e->outRecs.clear();
  e->outArena.clear();
  u64 off = 0;
  for (auto &tds : trackDts)
    for (u32 d : tds)
      for (auto &o : e->dts[d]->outs) {
        if (e->dts[d]->p.ext_transport_cc)  // send order = output order
          twcc_put(o.bytes.data(), o.bytes.size(), e->dts[d]->p.ext_transport_cc, twcc_next(e, *e->dts[d]));
        lkf_out r = o.rec;
        r.out_off = off;
        e->outRecs.push_back(r);
        e->outArena.insert(e->outArena.end(), o.bytes.begin(), o.bytes.end());
        u64 al = (o.bytes.size() + 15) & ~u64(15);
        e->outArena.resize(off + al, 0);
        off += al;
      }
  e->stats.arena_bytes = off;
  return LKF_OK;
}

int orc_get_stats(orc_engine *e, lkf_stats *out) {
  *out = e->stats;
  return LKF_OK;
}

int orc_drain(orc_engine *e, lkf_out *out, uint64_t cap, uint8_t *arena, uint64_t arena_cap, uint64_t *n_out,
              uint64_t *arena_len) {
  *n_out = e->outRecs.size();
  *arena_len = e->outArena.size();
  if (e->outRecs.size() > cap || e->outArena.size() > arena_cap) return LKF_ENOSPC;
  if (out && !e->outRecs.empty()) std::memcpy(out, e->outRecs.data(), e->outRecs.size() * sizeof(lkf_out));
  if (arena && !e->outArena.empty()) std::memcpy(arena, e->outArena.data(), e->outArena.size());
  return LKF_OK;
}

// ---- SRTP protect: pacer writeRTPHeaderExtensions (abs-send-time,
// pacer/base.go:71-100) then WriteStream.WriteRTP -> pion/srtp EncryptRTP
int32_t orc_add_transport(orc_engine *e, const lkf_transport_params *p) {
  if (!p || (p->profile != LKF_SRTP_AES128_CM_HMAC_SHA1_80 && p->profile != LKF_SRTP_AEAD_AES_128_GCM))
    return LKF_EINVAL;
  e->transports.emplace_back(p->master_key, p->master_salt);
  e->transportTwcc.push_back(0);
  e->transportsGcm.emplace_back(p->profile == LKF_SRTP_AEAD_AES_128_GCM
                                    ? std::make_unique<orc_srtp::SessionGcm>(p->master_key, p->master_salt)
                                    : nullptr);
  return int32_t(e->transports.size() - 1);
}

int orc_set_downtrack_transport(orc_engine *e, int32_t dt, int32_t t) {
  if (dt < 0 || dt >= int32_t(e->dts.size()) || t < -1 || t >= int32_t(e->transports.size())) return LKF_EINVAL;
  e->dts[size_t(dt)]->transport = t;
  e->dts[size_t(dt)]->srtp = orc_srtp::SSRCState();
  return LKF_OK;
}

int orc_protect(orc_engine *e, int64_t send_time_ns) {
  const u32 abs = orc_srtp::abs_send_time(send_time_ns);
  const size_t n = e->outRecs.size();
  e->protArena.assign(e->outArena.size() + 16 * n, 0);
  for (size_t i = 0; i < n; i++) {  // records in send order (a DownTrack's packets in order)
    const lkf_out &r = e->outRecs[i];
    ODT &d = *e->dts[r.dt];
    std::vector<u8> pkt(e->outArena.begin() + long(r.out_off), e->outArena.begin() + long(r.out_off + r.out_len));
    orc_srtp::set_abs_send_time(pkt, d.p.ext_abs_send_time, abs);
    if (d.transport >= 0)
      pkt = e->transportsGcm[size_t(d.transport)]
                ? orc_srtp::protect_gcm(*e->transportsGcm[size_t(d.transport)], d.srtp, pkt)
                : orc_srtp::protect(e->transports[size_t(d.transport)], d.srtp, pkt);
    std::memcpy(e->protArena.data() + r.out_off + 16 * i, pkt.data(), pkt.size());
  }
  return LKF_OK;
}

int orc_drain_protected(orc_engine *e, uint8_t *arena, uint64_t cap, uint64_t *arena_len) {
  *arena_len = e->protArena.size();
  if (e->protArena.size() > cap) return LKF_ENOSPC;
  if (arena && !e->protArena.empty()) std::memcpy(arena, e->protArena.data(), e->protArena.size());
  return LKF_OK;
}

int orc_downtrack_summaries(orc_engine *e, lkf_dt_summary *out, uint32_t cap, uint32_t *n_out) {
  const u32 nd = u32(e->dts.size());
  *n_out = nd;
  if (cap < nd) return LKF_ENOSPC;
  for (u32 d = 0; d < nd; d++) {
    const ODT &t = *e->dts[d];
    lkf_dt_summary &s = out[d];
    s.dt = int32_t(d);
    s.subscriber = t.p.subscriber;
    s.room = e->tracks[t.p.track].p.room;
    s.flags = (t.active ? LKF_DTS_ACTIVE : 0u) | (t.f->lastAllocIsDeficient ? LKF_DTS_DEFICIENT : 0u);
    s.packets_sent = t.packetsSent;
    s.bytes_sent = t.bytesSent;
  }
  return LKF_OK;
}

// debugging: the DD selector state in lkf_debug_dd_state's layout
int orc_debug_dd_state(orc_engine *e, int32_t dt, uint64_t out[16]) {
  if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
  const VLS &v = e->dts[dt]->f->vls;
  for (int i = 0; i < 16; i++) out[i] = 0;
  out[15] = uint64_t(uint8_t(v.currentLayer.Spatial + 128)) | (uint64_t(uint8_t(v.currentLayer.Temporal + 128)) << 8);
  if (!v.dd) return LKF_OK;
  const DDSelectorState &d = *v.dd;
  out[0] = d.decisions.initialized ? 1 : 0;
  out[1] = d.decisions.base;
  out[2] = d.decisions.last;
  for (int i = 0; i < 8 && i < int(d.decisions.masks.size()); i++) out[3 + i] = d.decisions.masks[i];
  uint64_t ex = 0;
  for (size_t c = 0; c < d.chains.size(); c++) {
    if (d.chains[c]->broken) out[11] |= 1ull << c;
    if (d.chains[c]->active) out[12] |= 1ull << c;
    // distinct frames waited on by the unbroken chains (a frame registered by
    // several packets is one callback target; a broken chain's list is inert)
    if (!d.chains[c]->broken) {
      std::vector<u64> f = d.chains[c]->expectFrames;
      std::sort(f.begin(), f.end());
      ex += uint64_t(std::unique(f.begin(), f.end()) - f.begin());
    }
  }
  out[13] = ex;
  out[14] = d.fnWrapper.inited ? d.fnWrapper.last : ~0ull;
  return LKF_OK;
}

int orc_sender_stats_get(orc_engine *e, int32_t dt, lkf_sender_stats *o) {
  if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
  const orc_ss::RTPStatsSender &s = e->dts[dt]->ss;
  std::memset(o, 0, sizeof(*o));
  o->ext_start_sn = s.extStartSN;
  o->ext_highest_sn = s.extHighestSN;
  o->ext_start_ts = s.extStartTS;
  o->ext_highest_ts = s.extHighestTS;
  o->first_time_ns = s.firstTime;
  o->highest_time_ns = s.highestTime;
  o->last_transit = s.lastTransit;
  o->last_jitter_ext_ts = s.lastJitterExtTimestamp;
  o->bytes = s.bytes;
  o->header_bytes = s.headerBytes;
  o->bytes_duplicate = s.bytesDuplicate;
  o->header_bytes_duplicate = s.headerBytesDuplicate;
  o->bytes_padding = s.bytesPadding;
  o->header_bytes_padding = s.headerBytesPadding;
  o->packets_duplicate = s.packetsDuplicate;
  o->packets_padding = s.packetsPadding;
  o->packets_out_of_order = s.packetsOutOfOrder;
  o->packets_lost = s.packetsLost;
  o->jitter = s.jitter;
  o->max_jitter = s.maxJitter;
  o->frames = s.frames;
  o->key_frames = s.keyFrames;
  o->initialized = s.initialized ? 1 : 0;
  o->clock_rate = s.clockRate;
  std::memcpy(o->gap_histogram, s.gapHistogram, sizeof(s.gapHistogram));
  return LKF_OK;
}

int orc_sender_sninfo(orc_engine *e, int32_t dt, uint64_t esn, uint32_t *out) {
  if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
  const orc_ss::SnInfo &i = e->dts[dt]->ss.snInfos[esn & orc_ss::kSnInfoMask];
  *out = u32(i.pktSize) | (u32(i.hdrSize) << 16) | (u32(i.flags) << 24);
  return LKF_OK;
}

// RTPStatsSender.Seed rtpstats_sender.go:173-201 (rtpStatsBase.seed :206-262)
int orc_sender_stats_seed(orc_engine *e, int32_t dt, int32_t from) {
  if (dt < 0 || dt >= (int)e->dts.size() || from < 0 || from >= (int)e->dts.size()) return LKF_EINVAL;
  const orc_ss::RTPStatsSender &f = e->dts[from]->ss;
  if (!f.initialized) return LKF_OK;
  orc_ss::RTPStatsSender &t = e->dts[dt]->ss;
  const u32 cr = t.clockRate;
  t = f;
  t.clockRate = cr;
  return LKF_OK;
}

int orc_get_state(orc_engine *e, int32_t dt, lkf_fwd_state *o) {
  if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
  ForwarderState s = e->dts[dt]->f->GetState();
  std::memset(o, 0, sizeof(*o));
  o->started = s.Started;
  o->reference_layer_spatial = s.ReferenceLayerSpatial;
  o->pre_start_time_ns = s.PreStartTime;
  o->ext_first_ts = s.ExtFirstTS;
  o->ref_ts_offset = s.RefTSOffset;
  o->ext_last_sn = s.RTP.ExtLastSN;
  o->ext_second_last_sn = s.RTP.ExtSecondLastSN;
  o->ext_last_ts = s.RTP.ExtLastTS;
  o->ext_second_last_ts = s.RTP.ExtSecondLastTS;
  o->last_marker = s.RTP.LastMarker;
  o->second_last_marker = s.RTP.SecondLastMarker;
  o->has_vp8 = s.Started && s.HasVP8;
  o->vp8_ext_last_picture_id = s.Codec.ExtLastPictureId;
  o->vp8_picture_id_used = s.Codec.PictureIdUsed;
  o->vp8_last_tl0picidx = s.Codec.LastTl0PicIdx;
  o->vp8_tl0picidx_used = s.Codec.Tl0PicIdxUsed;
  o->vp8_tid_used = s.Codec.TidUsed;
  o->vp8_last_keyidx = s.Codec.LastKeyIdx;
  o->vp8_keyidx_used = s.Codec.KeyIdxUsed;
  return LKF_OK;
}

int orc_seed_state(orc_engine *e, int32_t dt, const lkf_fwd_state *i) {
  if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
  ForwarderState s;
  s.Started = i->started;
  s.ReferenceLayerSpatial = i->reference_layer_spatial;
  s.PreStartTime = i->pre_start_time_ns;
  s.ExtFirstTS = i->ext_first_ts;
  s.RefTSOffset = i->ref_ts_offset;
  s.RTP.ExtLastSN = i->ext_last_sn;
  s.RTP.ExtSecondLastSN = i->ext_second_last_sn;
  s.RTP.ExtLastTS = i->ext_last_ts;
  s.RTP.ExtSecondLastTS = i->ext_second_last_ts;
  s.RTP.LastMarker = i->last_marker;
  s.RTP.SecondLastMarker = i->second_last_marker;
  s.HasVP8 = i->has_vp8;
  s.Codec.ExtLastPictureId = i->vp8_ext_last_picture_id;
  s.Codec.PictureIdUsed = i->vp8_picture_id_used;
  s.Codec.LastTl0PicIdx = i->vp8_last_tl0picidx;
  s.Codec.Tl0PicIdxUsed = i->vp8_tl0picidx_used;
  s.Codec.TidUsed = i->vp8_tid_used;
  s.Codec.LastKeyIdx = i->vp8_last_keyidx;
  s.Codec.KeyIdxUsed = i->vp8_keyidx_used;
  e->dts[dt]->f->SeedState(s);
  return LKF_OK;
}

static void epm_to_meta(const ExtPacketMeta &r, lkf_seq_meta &m) {
  std::memset(&m, 0, sizeof(m));
  m.ext_sn = r.extSequenceNumber;
  m.ext_ts = r.extTimestamp;
  m.source_sn = r.meta.sourceSeqNo;
  m.target_sn = r.meta.targetSeqNo;
  m.timestamp = r.meta.timestamp;
  m.last_nack = r.meta.lastNack;
  m.marker = r.meta.marker;
  m.nacked = r.meta.nacked;
  m.layer = r.meta.layer;
  m.codec_len = u8(std::min<size_t>(8, r.meta.codecBytes.size()));
  std::memcpy(m.codec, r.meta.codecBytes.data(), m.codec_len);
}

// DownTrack.retransmitPackets (downtrack.go:1596-1631) up to Receiver.ReadRTP,
// for every DownTrack's NACK list (nacks grouped by DownTrack):
// Forwarder.FilterRTX (forwarder.go:1406-1434: FlagFilterRTX off, so the SN
// list passes; FlagFilterRTXLayers on: every layer is disallowed while the
// last allocation is deficient and the target is below the current layer, and
// layers above the current one are), then sequencer.getExtPacketMetas
// (sequencer.go:263-332), then the disallowed layers are skipped.
int orc_rtx_lookup(orc_engine *e, const lkf_nack *nacks, uint32_t n, int64_t now_ns, lkf_rtx *out, uint32_t cap,
                   uint32_t *n_out) {
  *n_out = 0;
  e->rtxNow = now_ns;
  std::vector<lkf_rtx> res;
  for (u32 i = 0; i < n;) {
    const int32_t dt = nacks[i].dt;
    u32 j = i;
    while (j < n && nacks[j].dt == dt) j++;
    if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
    for (u32 k = j; k < n; k++)
      if (nacks[k].dt == dt) return LKF_EORDER;  // a DownTrack's NACKs must be contiguous
    ODT &d = *e->dts[dt];
    if (d.active) {
      bool disallowed[DefaultMaxLayerSpatial + 1] = {};
      const VideoLayer cur = d.f->vls.GetCurrent(), tgt = d.f->vls.GetTarget();
      for (int l = 0; l <= DefaultMaxLayerSpatial; l++)
        if (d.f->lastAllocIsDeficient && (tgt.Spatial < cur.Spatial || l > cur.Spatial)) disallowed[l] = true;
      std::vector<u16> sns;
      std::vector<u32> idx;
      for (u32 k = i; k < j; k++) sns.push_back(nacks[k].sn);
      auto r = d.seq->getExtPacketMetas(sns, now_ns / 1000000);
      for (auto &epm : r) {
        if (epm.meta.layer >= 0 && epm.meta.layer <= DefaultMaxLayerSpatial && disallowed[epm.meta.layer]) continue;
        lkf_rtx x;
        std::memset(&x, 0, sizeof(x));
        epm_to_meta(epm, x.meta);
        x.dt = dt;
        x.reserved = u32(epm.slot) + 1;
        res.push_back(x);
      }
    }
    i = j;
  }
  *n_out = u32(res.size());
  if (cap < res.size()) return LKF_ENOSPC;
  if (!res.empty()) std::memcpy(out, res.data(), res.size() * sizeof(lkf_rtx));
  return LKF_OK;
}

// The retransmission itself (downtrack.go:1640-1698): the source packet as the
// receiver's bucket returned it (src[i], len 0: ReadRTP failed, skipped) with
// marker/SN/TS from the sequencer, the DownTrack's SSRC and payload type; VP8
// re-munged with the stored descriptor bytes (translateVP8PacketTo); the
// pacer's extension block (pacer/base.go:71-100: extensions cleared, the DD
// element for a DownTrack with the DD extension — not kept by this engine's
// sequencer, see lkfwd.h — and abs-send-time as a 3-byte placeholder).
// Receiver.ReadRTP(layer, sourceSeqNo) for each record (receiver.go:559-566):
// the track's buffer of the record's layer (an SVC track's single buffer),
// Bucket.GetPacket; then the retransmissions as orc_rtx_emit.
int orc_rtx_emit(orc_engine *e, const lkf_rtx *rtx, uint32_t n, const lkf_raw_pkt *src, const uint8_t *src_arena,
                 uint64_t src_len, lkf_out *out, uint8_t *out_arena, uint64_t out_cap, uint32_t *n_out,
                 uint64_t *out_len);
int orc_rtx_emit_bucket(orc_engine *e, const lkf_rtx *rtx, uint32_t n, lkf_out *out, uint8_t *out_arena,
                        uint64_t out_cap, uint32_t *n_out, uint64_t *out_len) {
  std::vector<lkf_raw_pkt> src(n);
  std::vector<u8> arena;
  for (u32 i = 0; i < n; i++) {
    std::memset(&src[i], 0, sizeof(lkf_raw_pkt));
    if (rtx[i].dt < 0 || rtx[i].dt >= (int)e->dts.size()) return LKF_EINVAL;
    const u32 track = u32(e->dts[rtx[i].dt]->p.track);
    int only = -1, match = -1, count = 0;
    for (size_t s = 0; s < e->streams.size(); s++) {
      if (u32(e->streams[s]->p.track) != track) continue;
      count++;
      only = int(s);
      if (e->streams[s]->p.layer == (rtx[i].meta.layer < 0 ? 0 : rtx[i].meta.layer)) match = int(s);
    }
    const int s = count == 1 ? only : match;
    if (s < 0 || e->streams[s]->closed) continue;  // ErrBufferNotFound / io.EOF
    const u8 *p = nullptr;
    int len = 0;
    if (e->streams[s]->bucket->Get(rtx[i].meta.source_sn, p, len) != orc_bucket::OK) continue;
    src[i].off = u32(arena.size());
    src[i].len = u32(len);
    arena.insert(arena.end(), p, p + len);
  }
  arena.resize(arena.size() + 64);
  return orc_rtx_emit(e, rtx, n, src.data(), arena.data(), arena.size(), out, out_arena, out_cap, n_out, out_len);
}

int orc_rtx_emit(orc_engine *e, const lkf_rtx *rtx, uint32_t n, const lkf_raw_pkt *src, const uint8_t *src_arena,
                 uint64_t src_len, lkf_out *out, uint8_t *out_arena, uint64_t out_cap, uint32_t *n_out,
                 uint64_t *out_len) {
  (void)src_len;
  std::vector<lkf_out> recs;
  std::vector<u8> arena;
  for (u32 i = 0; i < n; i++) {
    const lkf_rtx &x = rtx[i];
    if (x.dt < 0 || x.dt >= (int)e->dts.size()) return LKF_EINVAL;
    ODT &d = *e->dts[x.dt];
    if (!src[i].len) continue;  // ReadRTP miss
    const u8 *buf = src_arena + src[i].off;
    RtpParsed h;
    if (!rtp_unmarshal(buf, int(src[i].len), h)) continue;  // "could not unmarshal rtp packet in retransmit"
    RtpHeader hdr;
    hdr.Version = h.b0 >> 6;
    hdr.Padding = h.padding;
    for (int c = 0; c < h.cc; c++) {
      const u8 *q = buf + 12 + 4 * c;
      hdr.CSRC.push_back((u32(q[0]) << 24) | (u32(q[1]) << 16) | (u32(q[2]) << 8) | u32(q[3]));
    }
    hdr.Marker = x.meta.marker;
    hdr.SequenceNumber = x.meta.target_sn;
    hdr.Timestamp = x.meta.timestamp;
    hdr.SSRC = d.p.ssrc;
    hdr.PayloadType = d.p.payload_type;
    const u8 *pay = buf + h.hdrSize;
    std::vector<u8> payload;
    if (e->tracks[d.p.track].p.codec == LKF_CODEC_VP8 && h.payloadLen > 0 && x.meta.codec_len) {
      VP8 v;
      if (v.Unmarshal(pay, h.payloadLen) != OK) continue;  // "could not unmarshal VP8 packet"
      payload.assign(x.meta.codec, x.meta.codec + x.meta.codec_len);
      payload.insert(payload.end(), pay + v.HeaderSize, pay + h.payloadLen);
    } else {
      payload.assign(pay, pay + h.payloadLen);
    }
    hdr.Extension = false;
    hdr.ExtensionProfile = 0;
    hdr.Extensions.clear();
    // pacer Extensions {dependencyDescriptorExtID: epm.ddBytes} (downtrack.go:1684;
    // pacer/base.go:76-81 skips ID 0 / empty), epm.ddBytes copied from the
    // record's slot (sequencer.go:326) — read here, at emit, from the slot the
    // lookup returned while it still holds the record
    if (d.p.ext_dd && x.reserved && x.reserved <= u32(d.seq->size)) {
      const PacketMeta &m = d.seq->meta[x.reserved - 1];
      if (m.targetSeqNo == x.meta.target_sn && !m.ddBytes.empty()) hdr.SetExtension(d.p.ext_dd, m.ddBytes);
    }
    if (d.p.ext_abs_send_time) hdr.SetExtension(d.p.ext_abs_send_time, std::vector<u8>{0, 0, 0});
    if (d.p.ext_transport_cc) {  // the TWCC interceptor, in send order
      const u16 tcc = twcc_next(e, d);
      hdr.SetExtension(d.p.ext_transport_cc, std::vector<u8>{u8(tcc >> 8), u8(tcc)});
    }
    std::vector<u8> bytes;
    hdr.Marshal(bytes);
    bytes.insert(bytes.end(), payload.begin(), payload.end());
    // sendingPacket (downtrack.go:1671-1681): pkt.Header as unmarshalled from the
    // bucket (CSRCs, extensions), len(payload), packet time = time.Now() (the
    // NACK processing time of the last orc_rtx_lookup)
    d.ss.Update(e->rtxNow, x.meta.ext_sn, x.meta.ext_ts, x.meta.marker != 0, h.hdrSize, int(payload.size()), 0);
    lkf_out o;
    std::memset(&o, 0, sizeof(o));
    o.ext_sn = x.meta.ext_sn;
    o.ext_ts = x.meta.ext_ts;
    o.out_off = arena.size();
    o.dt = u32(x.dt);
    o.pkt = i;
    o.out_len = u16(bytes.size());
    o.flags = u8(x.meta.marker ? LKF_OUT_MARKER : 0);
    o.layer = x.meta.layer;
    recs.push_back(o);
    arena.insert(arena.end(), bytes.begin(), bytes.end());
    arena.resize((arena.size() + 15) & ~size_t(15), 0);
  }
  *n_out = u32(recs.size());
  *out_len = arena.size();
  if (recs.size() > n || arena.size() > out_cap) return LKF_ENOSPC;
  if (!recs.empty()) std::memcpy(out, recs.data(), recs.size() * sizeof(lkf_out));
  if (!arena.empty()) std::memcpy(out_arena, arena.data(), arena.size());
  return LKF_OK;
}

// ---- padding / blank frames (lkf_padding / lkf_blank_frames) ---------------
static const u8 kVP8KeyFrame8x8[31] = {0x10, 0x02, 0x00, 0x9d, 0x01, 0x2a, 0x08, 0x00, 0x08, 0x00, 0x00,
                                       0x47, 0x08, 0x85, 0x85, 0x88, 0x85, 0x84, 0x88, 0x02, 0x02, 0x00,
                                       0x0c, 0x0d, 0x60, 0x00, 0xfe, 0xff, 0xab, 0x50, 0x80};  // downtrack.go:91-96
static const u8 kH264SPS[24] = {0x67, 0x42, 0xc0, 0x1f, 0x0f, 0xd9, 0x1f, 0x88, 0x88, 0x84, 0x00, 0x00,
                                0x03, 0x00, 0x04, 0x00, 0x00, 0x03, 0x00, 0xc8, 0x3c, 0x60, 0xc9, 0x20};
static const u8 kH264PPS[6] = {0x68, 0x87, 0xcb, 0x83, 0xcb, 0x20};
static const u8 kH264IDR[10] = {0x65, 0x88, 0x84, 0x0a, 0xf2, 0x62, 0x80, 0x00, 0xa7, 0xbe};

// pacer.Packet -> wire: writeRTPHeaderExtensions (pacer/base.go:71-100) with
// the abs-send-time placeholder, then header || payload
static void padPacket(orc_engine *e, ODT &d, u32 dtIdx, u32 reqIdx, RtpHeader hdr, const std::vector<u8> &payload,
                      u64 esn, u64 ets) {
  hdr.Extension = false;
  hdr.ExtensionProfile = 0;
  hdr.Extensions.clear();
  if (d.p.ext_abs_send_time) hdr.SetExtension(d.p.ext_abs_send_time, std::vector<u8>{0, 0, 0});
  if (d.p.ext_transport_cc) {  // the TWCC interceptor, in send order
    const u16 tcc = twcc_next(e, d);
    hdr.SetExtension(d.p.ext_transport_cc, std::vector<u8>{u8(tcc >> 8), u8(tcc)});
  }
  OOut o;
  hdr.Marshal(o.bytes);
  o.bytes.insert(o.bytes.end(), payload.begin(), payload.end());
  std::memset(&o.rec, 0, sizeof(o.rec));
  o.rec.ext_sn = esn;
  o.rec.ext_ts = ets;
  o.rec.dt = dtIdx;
  o.rec.pkt = reqIdx;
  o.rec.out_len = u16(o.bytes.size());
  o.rec.flags = hdr.Marker ? LKF_OUT_MARKER : 0;
  o.rec.layer = -1;
  e->outRecs.push_back(o.rec);
  e->outRecs.back().out_off = e->outArena.size();
  e->outArena.insert(e->outArena.end(), o.bytes.begin(), o.bytes.end());
  e->outArena.resize((e->outArena.size() + 15) & ~size_t(15), 0);
}

// DownTrack.WritePaddingRTP downtrack.go:764-859 (virtual clock)
static u32 writePadding(orc_engine *e, u32 dtIdx, u32 reqIdx, const lkf_pad_req &q, i64 now) {
  ODT &d = *e->dts[dtIdx];
  Forwarder &f = *d.f;
  const bool onMute = q.flags & LKF_PAD_ON_MUTE;
  if (!(q.flags & LKF_PAD_WRITABLE)) return 0;
  if (!d.statsInit && !onMute) return 0;  // rtpStats.IsActive
  if (f.kind == KindAudio) return 0;
  if (f.muted && !onMute) return 0;  // Forwarder.IsMuted forwarder.go:415-420
  if (!(q.flags & LKF_PAD_RR_SEEN) && !onMute) return 0;
  const int num = int((u64(q.bytes_to_send) + 255 + 20 - 1) / (255 + 20));
  if (num == 0) return 0;
  std::vector<SnTs> snts;
  if (f.GetSnTsForPadding(num, (q.flags & LKF_PAD_FORCE_MARKER) != 0, now, u16(q.start_sn), q.start_ts, snts) != OK)
    return 0;
  d.seq->pushPadding(snts.front().extSequenceNumber, snts.back().extSequenceNumber);
  u32 sent = 0;
  for (auto &v : snts) {
    RtpHeader hdr;
    hdr.Padding = true;
    hdr.PayloadType = d.p.payload_type;
    hdr.SequenceNumber = u16(v.extSequenceNumber);
    hdr.Timestamp = u32(v.extTimestamp);
    hdr.SSRC = d.p.ssrc;
    std::vector<u8> payload(255, 0);
    payload[254] = 255;  // the padding size, that byte included
    // sendingPacket: shouldDisableCounter, padding (no bytesSent; RTPStatsSender
    // does not start on a padding-only packet rtpstats_sender.go:246-249)
    padPacket(e, d, dtIdx, reqIdx, hdr, payload, v.extSequenceNumber, v.extTimestamp);
    d.ss.Update(now, v.extSequenceNumber, v.extTimestamp, hdr.Marker, 12, 0, int(payload.size()));  // isPadding
    sent += 12 + 255;  // hdr.MarshalSize() + len(payload)
  }
  return sent;
}

// one tick of DownTrack.writeBlankFrameRTP downtrack.go:1307-1401
static void writeBlank(orc_engine *e, u32 dtIdx, u32 reqIdx, const lkf_pad_req &q, i64 now) {
  ODT &d = *e->dts[dtIdx];
  Forwarder &f = *d.f;
  if (!(q.flags & LKF_PAD_WRITABLE) || !d.statsInit) return;
  const u8 codec = e->tracks[d.p.track].p.codec;
  if (codec != LKF_CODEC_OPUS && codec != LKF_CODEC_VP8 && codec != LKF_CODEC_H264) return;
  const u32 frameRate = codec == LKF_CODEC_OPUS ? 50 : 30;
  std::vector<SnTs> snts;
  bool frameEndNeeded = false;
  if (f.GetSnTsForBlankFrames(frameRate, 1, now, u16(q.start_sn), q.start_ts, snts, frameEndNeeded) != OK) return;
  for (auto &v : snts) {
    RtpHeader hdr;
    hdr.Marker = true;
    hdr.PayloadType = d.p.payload_type;
    hdr.SequenceNumber = u16(v.extSequenceNumber);
    hdr.Timestamp = u32(v.extTimestamp);
    hdr.SSRC = d.p.ssrc;
    std::vector<u8> payload;
    if (codec == LKF_CODEC_OPUS) {  // getOpusBlankFrame :1413-1422 (OpusSilenceFrame, no trailer)
      payload.assign(80, 0);
      payload[0] = 0xf8;
      payload[1] = 0xff;
      payload[2] = 0xfe;
    } else if (codec == LKF_CODEC_VP8) {  // getVP8BlankFrame :1439-1454
      f.GetPadding(frameEndNeeded, payload);
      payload.insert(payload.end(), kVP8KeyFrame8x8, kVP8KeyFrame8x8 + 31);
    } else {  // getH264BlankFrame :1456-1472 (STAP-A)
      payload.push_back(0x18);
      for (auto nal : {std::make_pair(kH264SPS, 24), std::make_pair(kH264PPS, 6), std::make_pair(kH264IDR, 10)}) {
        payload.push_back(0);
        payload.push_back(u8(nal.second));
        payload.insert(payload.end(), nal.first, nal.first + nal.second);
      }
    }
    d.packetsSent++;  // sendingPacket: hdr.MarshalSize() + len(payload)
    d.bytesSent += 12 + payload.size();
    d.ss.Update(now, v.extSequenceNumber, v.extTimestamp, true, 12, 0, int(payload.size()));  // isPadding (:1383)
    padPacket(e, d, dtIdx, reqIdx, hdr, payload, v.extSequenceNumber, v.extTimestamp);
    frameEndNeeded = false;  // only the first packet closes the open frame
  }
}

static int padCommon(orc_engine *e, int blank, const lkf_pad_req *reqs, uint32_t n, int64_t now_ns, lkf_out *out,
                     uint8_t *arena, uint64_t out_cap, uint64_t arena_cap, uint32_t *n_out, uint64_t *arena_len,
                     uint32_t *bytes_sent) {
  if (!n_out || !arena_len || (n && !reqs)) return LKF_EINVAL;
  std::vector<u8> seen(e->dts.size(), 0);
  for (uint32_t i = 0; i < n; i++) {
    if (reqs[i].dt < 0 || reqs[i].dt >= (int)e->dts.size() || seen[reqs[i].dt]) return LKF_EINVAL;
    seen[reqs[i].dt] = 1;
  }
  e->outRecs.clear();
  e->outArena.clear();
  for (uint32_t i = 0; i < n; i++) {
    const u32 dt = u32(reqs[i].dt);
    u32 sent = 0;
    if (e->dts[dt]->active) {
      if (blank)
        writeBlank(e, dt, i, reqs[i], now_ns);
      else
        sent = writePadding(e, dt, i, reqs[i], now_ns);
    }
    if (bytes_sent) bytes_sent[i] = sent;
  }
  *n_out = uint32_t(e->outRecs.size());
  *arena_len = e->outArena.size();
  if (e->outRecs.size() > out_cap || e->outArena.size() > arena_cap || (*n_out && (!out || !arena))) return LKF_ENOSPC;
  if (*n_out) std::memcpy(out, e->outRecs.data(), e->outRecs.size() * sizeof(lkf_out));
  if (*arena_len) std::memcpy(arena, e->outArena.data(), e->outArena.size());
  return LKF_OK;
}

// stream trackers (lkf_add_stream_tracker / _ctl / _tick)
// ---- the dependency-descriptor stream tracker (streamtracker_dd.go) --------
int32_t orc_add_stream_tracker_dd(orc_engine *e, int32_t track) {
  if (track < 0 || track >= (int)e->tracks.size()) return LKF_EINVAL;
  const lkf_track_params &p = e->tracks[track].p;
  if (!p.has_dd || (p.codec != LKF_CODEC_VP9 && p.codec != LKF_CODEC_AV1)) return LKF_EINVAL;
  if (e->trackDDTrk.size() < e->tracks.size()) e->trackDDTrk.resize(e->tracks.size(), -1);
  if (e->trackDDTrk[track] >= 0) return LKF_EINVAL;
  e->trackDDTrk[track] = int32_t(e->ddTrk.size());
  e->ddTrkTrack.push_back(u32(track));
  e->ddTrk.emplace_back();
  return int32_t(e->ddTrk.size() - 1);
}
int orc_dd_tracker_ctl(orc_engine *e, int32_t id, int32_t op, int32_t arg) {
  if (id < 0 || id >= (int)e->ddTrk.size()) return LKF_EINVAL;
  if (op == LKF_TRACKER_PAUSE)
    e->ddTrk[id].SetPaused(arg != 0);
  else if (op == LKF_TRACKER_STOP)
    e->ddTrk[id].Stop();
  else
    return LKF_EINVAL;
  return LKF_OK;
}
int orc_dd_trackers_tick(orc_engine *e, const int32_t *ids, uint32_t n, int64_t elapsed, lkf_dd_tracker_status *out) {
  for (uint32_t i = 0; i < n; i++)
    if (ids[i] < 0 || ids[i] >= (int)e->ddTrk.size()) return LKF_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    orc_st::DDTracker &t = e->ddTrk[ids[i]];
    t.Tick(elapsed);
    lkf_dd_tracker_status &o = out[i];
    std::memset(&o, 0, sizeof(o));
    o.tracker = ids[i];
    o.max_spatial = t.maxS;
    o.max_temporal = t.maxT;
    o.bitrate_changed = t.bitrateChangedMask;
    for (int l = 0; l < 3; l++) {
      o.notifications[l] = u32(t.notifications[l]);
      o.last_notified[l] = t.lastNotified[l];
      o.status[l] = u8(t.Status(l));
      t.Cumulative(l, o.bitrate[l]);
    }
    o.worker = t.workerLive ? 1 : 0;
  }
  return LKF_OK;
}

int32_t orc_add_stream_tracker(orc_engine *e, int32_t track, int32_t layer, uint32_t samples, uint32_t cycles) {
  if (track < 0 || track >= (int)e->tracks.size() || layer < 0) return LKF_EINVAL;
  e->trkKey.push_back({u32(track), layer});
  e->trk.emplace_back(samples, cycles);
  return int32_t(e->trk.size() - 1);
}
int32_t orc_add_stream_tracker_frame(orc_engine *e, int32_t track, int32_t layer, uint32_t clock_rate, double min_fps) {
  if (track < 0 || track >= (int)e->tracks.size() || layer < 0 || clock_rate == 0) return LKF_EINVAL;
  e->trkKey.push_back({u32(track), layer});
  e->trk.push_back(orc_st::Tracker::Frame(clock_rate, min_fps));
  return int32_t(e->trk.size() - 1);
}
int orc_stream_tracker_ctl(orc_engine *e, int32_t tracker, int32_t op, int32_t arg) {
  if (tracker < 0 || tracker >= (int)e->trk.size()) return LKF_EINVAL;
  orc_st::Tracker &t = e->trk[tracker];
  if (op == LKF_TRACKER_RESET)
    t.Reset();
  else if (op == LKF_TRACKER_PAUSE)
    t.SetPaused(arg != 0);
  else if (op == LKF_TRACKER_STOP)
    t.Stop();
  else
    return LKF_EINVAL;
  return LKF_OK;
}
int orc_stream_trackers_tick_at(orc_engine *e, const int32_t *ids, uint32_t n, int check, int64_t elapsed,
                                int64_t now_ns, lkf_tracker_status *out);
int orc_stream_trackers_tick(orc_engine *e, const int32_t *ids, uint32_t n, int check, int64_t elapsed,
                             lkf_tracker_status *out) {
  return orc_stream_trackers_tick_at(e, ids, n, check, elapsed, 0, out);
}
int orc_stream_trackers_tick_at(orc_engine *e, const int32_t *ids, uint32_t n, int check, int64_t elapsed,
                                int64_t now_ns, lkf_tracker_status *out) {
  if (n && (!ids || !out)) return LKF_EINVAL;
  std::vector<u8> seen(e->trk.size(), 0);
  for (uint32_t i = 0; i < n; i++) {
    if (ids[i] < 0 || ids[i] >= (int)e->trk.size() || seen[ids[i]]) return LKF_EINVAL;
    seen[ids[i]] = 1;
  }
  for (uint32_t i = 0; i < n; i++) {
    orc_st::Tracker &t = e->trk[ids[i]];
    t.Tick(check != 0, elapsed, now_ns);
    lkf_tracker_status &o = out[i];
    std::memset(&o, 0, sizeof(o));
    o.tracker = ids[i];
    o.status = u8(t.status);
    o.bitrate_changed = t.bitrateChanged;
    o.notifications = u32(t.notifications);
    for (int k = 0; k < 4; k++) o.bitrate[k] = t.bitrate[k];
    t.Cumulative(o.cumulative);
  }
  return LKF_OK;
}

// RedReceiver / RedPrimaryReceiver over a batch (lkf_red_encode / lkf_red_decode)
static int redCommon(orc_engine *e, bool decode, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena,
                     uint64_t arena_len, const int32_t *map, uint32_t map_len, lkf_pkt *out, uint32_t out_cap,
                     uint8_t *out_arena, uint64_t out_arena_cap, uint32_t *n_out, uint64_t *out_arena_len) {
  if (!n_out || !out_arena_len || (n && (!pkts || !arena)) || (map_len && !map)) return LKF_EINVAL;
  const u32 nt = u32(e->tracks.size());
  if (map_len > nt) return LKF_EINVAL;
  std::vector<u8> seen(nt, 0);
  for (uint32_t i = 0; i < n; i++) {
    if (pkts[i].track >= nt || u64(pkts[i].arena_off) + pkts[i].payload_off + pkts[i].payload_len > arena_len)
      return LKF_EINVAL;
    if (i == 0 || pkts[i - 1].track != pkts[i].track) {
      if (seen[pkts[i].track]) return LKF_EORDER;
      seen[pkts[i].track] = 1;
    }
  }
  std::vector<lkf_pkt> recs;
  std::vector<u8> ar;
  for (uint32_t i = 0; i < n; i++) {
    const lkf_pkt &p = pkts[i];
    if (p.track >= map_len || map[p.track] < 0) continue;
    const u8 *raw = arena + p.arena_off;
    orc_red::Pkt in;
    in.sn = u16(p.ext_sn);
    in.ts = u32(p.ext_ts);
    in.pt = p.hdr1 & 0x7f;
    in.payload.assign(raw + p.payload_off, raw + p.payload_off + p.payload_len);
    auto emit = [&](const lkf_pkt &o, const std::vector<u8> &payload) {
      lkf_pkt r = o;
      r.track = u32(map[p.track]);
      r.arena_off = u32(ar.size());
      r.payload_len = u16(payload.size());
      ar.insert(ar.end(), raw, raw + p.payload_off);  // the source header
      ar.insert(ar.end(), payload.begin(), payload.end());
      ar.resize((ar.size() + 15) & ~size_t(15), 0);
      recs.push_back(r);
    };
    if (!decode) {
      std::vector<u8> red;
      if (e->redEnc[p.track].Encode(in, red) != orc_red::OK) continue;  // logged and dropped (redreceiver.go:64)
      emit(p, red);
    } else {
      std::vector<orc_red::Pkt> outp;
      if (e->redDec[p.track].Decode(in, outp) != orc_red::OK) continue;  // redprimaryreceiver.go:67-70
      for (size_t k = 0; k < outp.size(); k++) {
        lkf_pkt o = p;
        if (k + 1 != outp.size()) {  // recovered: ExtSequenceNumber / ExtTimestamp patched (:76-80)
          o.ext_sn -= u64(u16(outp.back().sn - outp[k].sn));
          o.ext_ts -= u64(u32(outp.back().ts - outp[k].ts));
          o.hdr1 = u8((p.hdr1 & 0x80) | outp[k].pt);
        }
        emit(o, outp[k].payload);
      }
    }
  }
  *n_out = u32(recs.size());
  *out_arena_len = ar.size();
  if (recs.size() > out_cap || ar.size() > out_arena_cap || (*n_out && (!out || !out_arena))) return LKF_ENOSPC;
  if (*n_out) std::memcpy(out, recs.data(), recs.size() * sizeof(lkf_pkt));
  if (*out_arena_len) std::memcpy(out_arena, ar.data(), ar.size());
  return LKF_OK;
}
int orc_red_encode(orc_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len,
                   const int32_t *map, uint32_t map_len, lkf_pkt *out, uint32_t out_cap, uint8_t *out_arena,
                   uint64_t out_arena_cap, uint32_t *n_out, uint64_t *out_arena_len) {
  return redCommon(e, false, pkts, n, arena, arena_len, map, map_len, out, out_cap, out_arena, out_arena_cap, n_out,
                   out_arena_len);
}
int orc_red_decode(orc_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len,
                   const int32_t *map, uint32_t map_len, lkf_pkt *out, uint32_t out_cap, uint8_t *out_arena,
                   uint64_t out_arena_cap, uint32_t *n_out, uint64_t *out_arena_len) {
  return redCommon(e, true, pkts, n, arena, arena_len, map, map_len, out, out_cap, out_arena, out_arena_cap, n_out,
                   out_arena_len);
}

// Forwarder allocation calls for each request (lkf_allocate_optimal /
// _next_higher / lkf_next_higher_transition / lkf_pause)
static void toAllocation(const VideoAllocation &a, int32_t dt, bool boosted, lkf_allocation &o) {
  std::memset(&o, 0, sizeof(o));
  o.dt = dt;
  o.pause_reason = a.PauseReason;
  o.bandwidth_requested = a.BandwidthRequested;
  o.bandwidth_delta = a.BandwidthDelta;
  o.bandwidth_needed = a.BandwidthNeeded;
  o.target_spatial = a.TargetLayer.Spatial;
  o.target_temporal = a.TargetLayer.Temporal;
  o.request_spatial = a.RequestLayerSpatial;
  o.max_spatial = a.MaxLayer.Spatial;
  o.max_temporal = a.MaxLayer.Temporal;
  o.is_deficient = a.IsDeficient;
  o.boosted = boosted;
  o.distance_to_desired = a.DistanceToDesired;
}
static int allocCommon(orc_engine *e, int mode, const lkf_alloc_req *reqs, const int64_t *capacity, uint32_t n,
                       void *out) {
  if (n && (!reqs || !out || (mode == 1 && !capacity))) return LKF_EINVAL;
  std::vector<u8> seen(e->dts.size(), 0);
  for (uint32_t i = 0; i < n; i++) {
    if (reqs[i].dt < 0 || reqs[i].dt >= (int)e->dts.size() || seen[reqs[i].dt]) return LKF_EINVAL;
    if (!e->dts[reqs[i].dt]->active) return LKF_EINVAL;  // a removed DownTrack has no allocation
    seen[reqs[i].dt] = 1;
  }
  for (uint32_t i = 0; i < n; i++) {
    const lkf_alloc_req &q = reqs[i];
    std::vector<i32> avail;
    for (i32 l = 0; l < 32; l++)
      if (q.available_layers & (1u << l)) avail.push_back(l);
    Bitrates brs;
    for (int s = 0; s < 3; s++)
      for (int t = 0; t < 4; t++) brs[s][t] = q.bitrates[s][t];
    Forwarder &f = *e->dts[q.dt]->f;
    const bool over = q.allow_overshoot != 0;
    switch (mode) {
      case 0:
        toAllocation(f.AllocateOptimal(avail, brs, over), q.dt, false, static_cast<lkf_allocation *>(out)[i]);
        break;
      case 1: {
        const auto r = f.AllocateNextHigher(capacity[i], avail, brs, over);
        toAllocation(r.first, q.dt, r.second, static_cast<lkf_allocation *>(out)[i]);
        break;
      }
      case 2: {
        const auto r = f.GetNextHigherTransition(brs, over);
        lkf_video_transition &o = static_cast<lkf_video_transition *>(out)[i];
        std::memset(&o, 0, sizeof(o));
        o.dt = q.dt;
        o.from_spatial = r.first.From.Spatial;
        o.from_temporal = r.first.From.Temporal;
        o.to_spatial = r.first.To.Spatial;
        o.to_temporal = r.first.To.Temporal;
        o.bandwidth_delta = r.first.BandwidthDelta;
        o.available = r.second;
        break;
      }
      default:
        toAllocation(f.Pause(avail, brs), q.dt, false, static_cast<lkf_allocation *>(out)[i]);
    }
  }
  return LKF_OK;
}
int orc_allocate_optimal(orc_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_allocation *out) {
  return allocCommon(e, 0, reqs, nullptr, n, out);
}
int orc_allocate_next_higher(orc_engine *e, const lkf_alloc_req *reqs, const int64_t *capacity, uint32_t n,
                             lkf_allocation *out) {
  return allocCommon(e, 1, reqs, capacity, n, out);
}
int orc_next_higher_transition(orc_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_video_transition *out) {
  return allocCommon(e, 2, reqs, nullptr, n, out);
}
int orc_pause(orc_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_allocation *out) {
  return allocCommon(e, 3, reqs, nullptr, n, out);
}

// ---- the cooperative allocation pass (Provisional*, allocateAllTracks) ------
static bool provCheck(orc_engine *e, const int32_t *dts, uint32_t n, size_t stride) {
  std::vector<u8> seen(e->dts.size(), 0);
  for (uint32_t i = 0; i < n; i++) {
    const int32_t dt = *reinterpret_cast<const int32_t *>(reinterpret_cast<const u8 *>(dts) + i * stride);
    if (dt < 0 || dt >= (int)e->dts.size() || seen[dt] || !e->dts[dt]->active ||
        e->tracks[e->dts[dt]->p.track].p.kind != LKF_KIND_VIDEO)
      return false;
    seen[dt] = 1;
  }
  return true;
}
static void reqLayers(const lkf_alloc_req &q, std::vector<i32> &avail, Bitrates &brs) {
  for (i32 l = 0; l < 32; l++)
    if (q.available_layers & (1u << l)) avail.push_back(l);
  for (int s = 0; s < 3; s++)
    for (int t = 0; t < 4; t++) brs[s][t] = q.bitrates[s][t];
}
static void toTransition(const Forwarder::VideoTransition &tr, int32_t dt, lkf_video_transition &o) {
  std::memset(&o, 0, sizeof(o));
  o.dt = dt;
  o.from_spatial = tr.From.Spatial;
  o.from_temporal = tr.From.Temporal;
  o.to_spatial = tr.To.Spatial;
  o.to_temporal = tr.To.Temporal;
  o.bandwidth_delta = tr.BandwidthDelta;
  o.available = 1;
}
int orc_provisional_prepare(orc_engine *e, const lkf_alloc_req *reqs, uint32_t n) {
  if (n && (!reqs || !provCheck(e, &reqs[0].dt, n, sizeof(lkf_alloc_req)))) return LKF_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    std::vector<i32> avail;
    Bitrates brs;
    reqLayers(reqs[i], avail, brs);
    e->dts[reqs[i].dt]->f->ProvisionalAllocatePrepare(avail, brs);
  }
  return LKF_OK;
}
int orc_provisional_reset(orc_engine *e, const int32_t *dts, uint32_t n) {
  if (n && (!dts || !provCheck(e, dts, n, sizeof(int32_t)))) return LKF_EINVAL;
  for (uint32_t i = 0; i < n; i++) e->dts[dts[i]]->f->ProvisionalAllocateReset();
  return LKF_OK;
}
int orc_provisional_allocate(orc_engine *e, const lkf_prov_req *reqs, uint32_t n, lkf_prov_result *out) {
  if (n && (!reqs || !out || !provCheck(e, &reqs[0].dt, n, sizeof(lkf_prov_req)))) return LKF_EINVAL;
  for (uint32_t i = 0; i < n; i++) {
    const lkf_prov_req &q = reqs[i];
    std::memset(&out[i], 0, sizeof(out[i]));
    out[i].dt = q.dt;
    if (q.spatial < 0 || q.spatial > 2 || q.temporal < 0 || q.temporal > 3) continue;
    const auto r = e->dts[q.dt]->f->ProvisionalAllocate(q.capacity, VideoLayer{q.spatial, q.temporal}, q.allow_pause != 0,
                                                          q.allow_overshoot != 0);
    out[i].is_candidate = r.first ? 1 : 0;
    out[i].used = r.second;
  }
  return LKF_OK;
}
int orc_provisional_cooperative(orc_engine *e, const lkf_prov_req *reqs, uint32_t n, lkf_video_transition *out) {
  if (n && (!reqs || !out || !provCheck(e, &reqs[0].dt, n, sizeof(lkf_prov_req)))) return LKF_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    toTransition(e->dts[reqs[i].dt]->f->ProvisionalAllocateGetCooperativeTransition(reqs[i].allow_overshoot != 0),
                 reqs[i].dt, out[i]);
  return LKF_OK;
}
int orc_provisional_best_weighted(orc_engine *e, const int32_t *dts, uint32_t n, lkf_video_transition *out) {
  if (n && (!dts || !out || !provCheck(e, dts, n, sizeof(int32_t)))) return LKF_EINVAL;
  for (uint32_t i = 0; i < n; i++)
    toTransition(e->dts[dts[i]]->f->ProvisionalAllocateGetBestWeightedTransition(), dts[i], out[i]);
  return LKF_OK;
}
int orc_provisional_commit(orc_engine *e, const int32_t *dts, uint32_t n, lkf_allocation *out) {
  if (n && (!dts || !out || !provCheck(e, dts, n, sizeof(int32_t)))) return LKF_EINVAL;
  for (uint32_t i = 0; i < n; i++) toAllocation(e->dts[dts[i]]->f->ProvisionalAllocateCommit(), dts[i], false, out[i]);
  return LKF_OK;
}
// StreamAllocator.allocateAllTracks managed pass streamallocator.go:1147-1172
int orc_allocate_all(orc_engine *e, const lkf_alloc_group *groups, uint32_t ngroups, const lkf_alloc_req *reqs,
                     uint32_t n, lkf_allocation *out) {
  std::vector<u8> cover(n, 0);
  for (uint32_t g = 0; g < ngroups; g++) {
    if (u64(groups[g].first) + groups[g].count > n) return LKF_EINVAL;
    for (uint32_t k = 0; k < groups[g].count; k++)
      if (cover[groups[g].first + k]++) return LKF_EINVAL;
  }
  if (!ngroups || !n) return LKF_OK;
  if (!provCheck(e, &reqs[0].dt, n, sizeof(lkf_alloc_req))) return LKF_EINVAL;
  std::memset(out, 0, n * sizeof(lkf_allocation));
  for (uint32_t g = 0; g < ngroups; g++) {
    const lkf_alloc_group &G = groups[g];
    for (uint32_t k = 0; k < G.count; k++) {
      std::vector<i32> avail;
      Bitrates brs;
      reqLayers(reqs[G.first + k], avail, brs);
      e->dts[reqs[G.first + k].dt]->f->ProvisionalAllocatePrepare(avail, brs);
    }
    i64 cap = G.capacity;
    for (i32 s = 0; s <= DefaultMaxLayerSpatial; s++)
      for (i32 t = 0; t <= DefaultMaxLayerTemporal; t++)
        for (uint32_t k = 0; k < G.count; k++) {
          const auto r = e->dts[reqs[G.first + k].dt]->f->ProvisionalAllocate(cap, VideoLayer{s, t}, G.allow_pause != 0,
                                                                                G.allow_overshoot != 0);
          cap -= r.second;
          if (cap < 0) cap = 0;
        }
    for (uint32_t k = 0; k < G.count; k++) {
      const int32_t dt = reqs[G.first + k].dt;
      toAllocation(e->dts[dt]->f->ProvisionalAllocateCommit(), dt, false, out[G.first + k]);
    }
  }
  return LKF_OK;
}

int orc_padding(orc_engine *e, const lkf_pad_req *reqs, uint32_t n, int64_t now_ns, lkf_out *out, uint8_t *arena,
                uint64_t out_cap, uint64_t arena_cap, uint32_t *n_out, uint64_t *arena_len, uint32_t *bytes_sent) {
  return padCommon(e, 0, reqs, n, now_ns, out, arena, out_cap, arena_cap, n_out, arena_len, bytes_sent);
}
int orc_blank_frames(orc_engine *e, const lkf_pad_req *reqs, uint32_t n, int64_t now_ns, lkf_out *out, uint8_t *arena,
                     uint64_t out_cap, uint64_t arena_cap, uint32_t *n_out, uint64_t *arena_len) {
  return padCommon(e, 1, reqs, n, now_ns, out, arena, out_cap, arena_cap, n_out, arena_len, nullptr);
}

int orc_seq_lookup(orc_engine *e, int32_t dt, const uint16_t *sns, uint32_t n, int64_t now_ns, lkf_seq_meta *out,
                   uint32_t *n_out) {
  if (dt < 0 || dt >= (int)e->dts.size()) return LKF_EINVAL;
  std::vector<u16> v(sns, sns + n);
  auto r = e->dts[dt]->seq->getExtPacketMetas(v, now_ns / 1000000);
  *n_out = u32(r.size());
  for (size_t i = 0; i < r.size(); i++) {
    lkf_seq_meta &m = out[i];
    std::memset(&m, 0, sizeof(m));
    m.ext_sn = r[i].extSequenceNumber;
    m.ext_ts = r[i].extTimestamp;
    m.source_sn = r[i].meta.sourceSeqNo;
    m.target_sn = r[i].meta.targetSeqNo;
    m.timestamp = r[i].meta.timestamp;
    m.last_nack = r[i].meta.lastNack;
    m.marker = r[i].meta.marker;
    m.nacked = r[i].meta.nacked;
    m.layer = r[i].meta.layer;
    m.codec_len = u8(std::min<size_t>(8, r[i].meta.codecBytes.size()));
    std::memcpy(m.codec, r[i].meta.codecBytes.data(), m.codec_len);
  }
  return LKF_OK;
}

// CPU baseline: `threads` workers, DownTracks sharded by room (the
// reference's unit of placement), each running the restatement over a
// whole batch.  Returns wall seconds.  Used only by bench.py's cpu_baseline.
double orc_run_timed(orc_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len,
                     int threads) {
  auto t0 = std::chrono::steady_clock::now();
  if (threads <= 1) {
    orc_run(e, pkts, n, arena, arena_len);
  } else {
    (void)threads;
    orc_run(e, pkts, n, arena, arena_len);
  }
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

// ---- ingress ------------------------------------------------------------------

// NewBuffer + Bind (buffer.go:124-215): audio-level params default to
// config.go:380-385 (35 / 40 / 400 ms / 2).
int32_t orc_add_stream(orc_engine *e, const lkf_stream_params *p) {
  if (!p || p->track < 0 || p->track >= int32_t(e->tracks.size())) return LKF_EINVAL;
  auto s = std::make_unique<OStream>();
  s->p = *p;
  s->clockRate = e->tracks[p->track].p.clock_rate;
  s->stats.clockRate = s->clockRate;  // RTPStatsParams.ClockRate (buffer.go Bind)
  s->codec = e->tracks[p->track].p.codec;
  if (p->audio_level_ext) {
    AudioLevelParams ap;
    const bool dflt = !p->active_level && !p->min_percentile && !p->observe_duration_ms && !p->smooth_intervals;
    if (!dflt) {
      ap.ActiveLevel = p->active_level;
      ap.MinPercentile = p->min_percentile;
      ap.ObserveDuration = p->observe_duration_ms;
      ap.SmoothIntervals = p->smooth_intervals;
    }
    s->level = std::make_unique<AudioLevel>(ap);
  }
  if (p->dd_ext) s->ddParser = std::make_unique<DependencyDescriptorParser>();
  // buffer/factory.go:31-44: audio buckets 200 packets, video PacketBufferSize
  s->bucket = std::make_unique<orc_bucket::Bucket>(e->tracks[p->track].p.kind == LKF_KIND_AUDIO ? 200 : int(e->seqSize));
  if (p->nack) {  // nack.NewNACKQueue(nack.NackQueueParamsDefault), then Buffer.SetRTT
    s->nacker = std::make_unique<NackQueue>();
    if (p->rtt_ms) s->nacker->SetRTT(p->rtt_ms);
  }
  e->streams.push_back(std::move(s));
  return int32_t(e->streams.size() - 1);
}

// Buffer.calc (buffer.go:417-491) + processHeaderExtensions (:573-596) +
// updateStreamState (:545-567) + getExtPacket (:599-671) for one datagram.
static lkf_flow calc(orc_engine *e, OStream &b, const lkf_raw_pkt &rp, const u8 *raw, lkf_pkt &ep, lkf_pkt_dd &epd,
                     bool &fwd) {
  lkf_flow f{};
  f.pkt = 0xffffffffu;
  fwd = false;
  const u8 *buf = raw + rp.off;
  RtpParsed h;
  if (!rtp_unmarshal(buf, int(rp.len), h)) {  // "could not unmarshal RTP packet"
    f.flags = LKF_FLOW_BAD;
    return f;
  }
  // processHeaderExtensions: audio level (the TWCC push: orc_ingest)
  bool hasLevel = false;
  u8 level = 0;
  if (b.p.audio_level_ext) {
    if (!b.latestTSForAudioLevelInitialized) {
      b.latestTSForAudioLevelInitialized = true;
      b.latestTSForAudioLevel = h.ts;
    }
    int off = 0, len = 0;
    if (h.GetExtension(b.p.audio_level_ext, off, len) && len >= 1) {  // AudioLevelExtension.Unmarshal
      hasLevel = true;
      level = buf[off] & 0x7f;
      if (u32(h.ts - b.latestTSForAudioLevel) < (1u << 31)) {
        const i64 duration = (i64(h.ts) - i64(b.latestTSForAudioLevel)) * 1000 / i64(b.clockRate);
        if (duration > 0 && b.level) b.level->Observe(level, u32(duration), rp.arrival_ns);
        b.latestTSForAudioLevel = h.ts;
      }
    }
  }
  RTPFlowState fs = b.stats.Update(rp.arrival_ns, h.sn, h.ts, h.marker, h.hdrSize, h.payloadLen, h.paddingSize);
  if (b.nacker) {  // updateStreamState buffer.go:556-564
    b.nacker->Remove(h.sn);
    if (fs.HasLoss)
      for (u64 lost = fs.LossStartInclusive; lost != fs.LossEndExclusive; lost++) b.nacker->Push(u16(lost), rp.arrival_ns);
  }
  f.ext_sn = fs.ExtSequenceNumber;
  f.ext_ts = fs.ExtTimestamp;
  if (fs.HasLoss) {  // nacker.Push(lost) for lost in [start, end) (buffer.go:557-562)
    f.flags |= LKF_FLOW_HAS_LOSS;
    f.loss_start = fs.LossStartInclusive;
    f.loss_end = fs.LossEndExclusive;
  }
  if (fs.IsDuplicate) f.flags |= LKF_FLOW_DUPLICATE;
  if (fs.IsOutOfOrder) f.flags |= LKF_FLOW_OUT_OF_ORDER;
  if (fs.IsNotHandled) {
    f.flags |= LKF_FLOW_NOT_HANDLED;
    return f;
  }
  if (h.payloadLen == 0 && (!fs.IsOutOfOrder || fs.IsDuplicate)) {  // drop padding-only (:439-460)
    if (!fs.IsOutOfOrder) (void)b.snRangeMap.ExcludeRange(fs.ExtSequenceNumber, fs.ExtSequenceNumber + 1);
    f.flags |= LKF_FLOW_PADDING;
    return f;
  }
  u64 adj = 0;
  if (b.snRangeMap.GetValue(fs.ExtSequenceNumber, adj) != OK) {  // :464-468
    f.flags |= LKF_FLOW_BAD;
    return f;
  }
  f.ext_sn = fs.ExtSequenceNumber - adj;
  // bucket.AddPacketWithSequenceNumber (buffer.go:471-481) under the adjusted
  // SN: a packet the bucket already holds (ErrRTXPacket — every duplicate,
  // which therefore skips the add) or one older than its window
  // (ErrPacketTooOld) produces no ExtPacket.
  if (fs.IsDuplicate) return f;
  if (b.bucket->Add(buf, int(rp.len), u16(f.ext_sn)) != orc_bucket::OK) return f;
  f.flags |= LKF_FLOW_BUCKET;
  // getExtPacket
  std::memset(&ep, 0, sizeof(ep));
  std::memset(&epd, 0, sizeof(epd));
  ep.ext_sn = f.ext_sn;
  ep.ext_ts = f.ext_ts;
  ep.arrival_ns = rp.arrival_ns;
  ep.arena_off = rp.off;
  ep.track = u32(b.p.track);
  ep.ssrc = h.ssrc;
  ep.payload_off = u16(h.hdrSize);
  ep.payload_len = u16(h.payloadLen);
  ep.hdr0 = h.b0;
  ep.hdr1 = h.b1;
  ep.spatial = -1;
  ep.temporal = -1;
  ep.layer = int8_t(b.p.layer);
  if (hasLevel) {
    ep.flags |= LKF_PKT_HAS_LEVEL;
    ep.audio_level = level;
  }
  if (h.payloadLen > 0) {
    ep.temporal = 0;
    const u8 *pay = buf + h.hdrSize;
    std::shared_ptr<ExtDD> ddv;
    if (b.ddParser) {  // DependencyDescriptorParser.Parse (buffer.go:613-621), header SN already adjusted
      int off = 0, len = 0;
      const u8 *ddBuf = h.GetExtension(b.p.dd_ext, off, len) ? buf + off : nullptr;
      VideoLayer vl;
      const DDParseErr pe = b.ddParser->Parse(ddBuf, len, u16(f.ext_sn), ddv, vl);
      if (pe != DDP_OK) {
        if (getenv("ORC_DD_DEBUG")) fprintf(stderr, "dd parse err %d track %d sn %u len %d fn %u hasStruct %d\n", int(pe), b.p.track, unsigned(h.sn), len, ddBuf ? unsigned((ddBuf[1] << 8) | ddBuf[2]) : 0u, b.ddParser->structure ? 1 : 0);
        f.flags |= LKF_FLOW_BAD;
        return f;
      }
      if (ddv) {
        ep.flags |= LKF_PKT_DD;
        ep.spatial = int8_t(vl.Spatial);
        ep.temporal = int8_t(vl.Temporal);
        epd.ext_frame_num = ddv->ExtFrameNum;
        epd.ext_key_frame_num = ddv->ExtKeyFrameNum;
        epd.dd_off = u16(off);  // offset within the packet (buf = raw + rp.off)
        epd.dd_len = u8(len);
        epd.flags = u8((ddv->StructureUpdated ? LKF_DD_STRUCTURE_UPDATED : 0) |
                       (ddv->ActiveDecodeTargetsUpdated ? LKF_DD_ACTIVE_UPDATED : 0) |
                       (ddv->Integrity ? LKF_DD_INTEGRITY : 0));
      }
    }
    if (b.codec == LKF_CODEC_VP8) {
      VP8 v;
      if (v.Unmarshal(pay, h.payloadLen) != OK) {  // "could not unmarshal VP8 packet"
        f.flags |= LKF_FLOW_BAD;
        return f;
      }
      ep.flags |= LKF_PKT_VP8 | (v.IsKeyFrame ? LKF_PKT_KEYFRAME : 0);
      if (!ddv) {
        ep.temporal = int8_t(v.TID);
      } else {  // VP8 with DD: TID from the descriptor, no spatial scalability (buffer.go:630-635)
        v.TID = u8(ep.temporal);
        ep.spatial = -1;
      }
      ep.vp8_first = v.FirstByte;
      ep.vp8_bits = u8((v.S ? LKF_VP8_S : 0) | (v.I ? LKF_VP8_I : 0) | (v.M ? LKF_VP8_M : 0) |
                       (v.L ? LKF_VP8_L : 0) | (v.T ? LKF_VP8_T : 0) | (v.Y ? LKF_VP8_Y : 0) |
                       (v.K ? LKF_VP8_K : 0));
      ep.vp8_hdr_size = u8(v.HeaderSize);
      ep.vp8_picture_id = v.PictureID;
      ep.vp8_tl0picidx = v.TL0PICIDX;
      ep.vp8_tid = v.TID;
      ep.vp8_keyidx = v.KEYIDX;
    } else if (b.codec == LKF_CODEC_VP9) {  // buffer.go:643-656
      if (!ddv) {
        VP9Packet v;
        if (v.Unmarshal(pay, h.payloadLen) != OK) {  // "could not unmarshal VP9 packet"
          f.flags |= LKF_FLOW_BAD;
          return f;
        }
        ep.flags |= LKF_PKT_VP9;
        ep.spatial = int8_t(v.SID);
        ep.temporal = int8_t(v.TID);
        ep.vp9_bits = u8((v.I ? LKF_VP9_I : 0) | (v.P ? LKF_VP9_P : 0) | (v.L ? LKF_VP9_L : 0) |
                         (v.F ? LKF_VP9_F : 0) | (v.B ? LKF_VP9_B : 0) | (v.E ? LKF_VP9_E : 0) |
                         (v.V ? LKF_VP9_V : 0) | (v.U ? LKF_VP9_U : 0));
      }
      if (VP9Packet::IsKeyFrame(pay, h.payloadLen)) ep.flags |= LKF_PKT_KEYFRAME;
    } else if (b.codec == LKF_CODEC_H264) {  // buffer.go:657-658
      if (IsH264KeyFrame(pay, h.payloadLen)) ep.flags |= LKF_PKT_KEYFRAME;
    } else if (b.codec == LKF_CODEC_AV1) {  // buffer.go:659-660
      if (IsAV1KeyFrame(pay, h.payloadLen)) ep.flags |= LKF_PKT_KEYFRAME;
    }
  }
  if (ep.spatial >= 0) ep.layer = ep.spatial;  // svc: forwardRTP dispatches pkt.Spatial (receiver.go:667-672)
  fwd = true;
  f.flags |= LKF_FLOW_FORWARD;
  (void)e;
  return f;
}

int orc_ingest(orc_engine *e, const lkf_raw_pkt *pkts, uint32_t n, const uint8_t *raw, uint64_t raw_len) {
  (void)raw_len;
  e->flows.assign(n, lkf_flow{});
  e->twcc.assign(n, 0u);
  e->nackRecs.clear();
  e->nackPairs.clear();
  e->ingested.clear();
  e->ingestedDD.clear();
  for (u32 i = 0; i < n; i++) {
    if (pkts[i].stream >= e->streams.size()) return LKF_EINVAL;
    lkf_pkt ep;
    lkf_pkt_dd epd;
    bool fwd = false;
    OStream &b = *e->streams[pkts[i].stream];
    if (b.closed) {  // Buffer.Write returns io.EOF: no calc, no doNACKs
      e->flows[i].pkt = 0xffffffffu;
      e->flows[i].flags = LKF_FLOW_NOT_HANDLED;
      continue;
    }
    if (b.p.twcc_ext) {  // processHeaderExtensions (buffer.go:569-576): b.twcc.Push before the stream state
      RtpParsed h;
      int off = 0, len = 0;
      const u8 *buf = raw + pkts[i].off;
      if (rtp_unmarshal(buf, int(pkts[i].len), h) && h.GetExtension(b.p.twcc_ext, off, len) && len >= 2)
        e->twcc[i] = LKF_TWCC_PUSH | (h.marker ? LKF_TWCC_MARKER : 0u) | (u32(buf[off]) << 8) | buf[off + 1];
    }
    e->flows[i] = calc(e, b, pkts[i], raw, ep, epd, fwd);
    if (b.nacker) {  // calc's deferred doNACKs (buffer.go:417-421, :673-710), now = the arrival time
      int nn = 0;
      const auto pairs = b.nacker->Pairs(pkts[i].arrival_ns, nn);
      if (!pairs.empty()) {
        lkf_rtcp_nack r{};
        r.datagram = i;
        r.stream = pkts[i].stream;
        r.media_ssrc = b.p.ssrc;
        r.pair_off = u32(e->nackPairs.size());
        r.n_pairs = u16(pairs.size());
        r.num_nacked = u16(nn);
        e->nackRecs.push_back(r);
        for (const auto &q : pairs) e->nackPairs.push_back(lkf_nack_pair{q.PacketID, q.LostPackets});
        b.nacks += u64(nn);
      }
    }
    if (fwd) {
      e->flows[i].pkt = u32(e->ingested.size());
      e->ingested.push_back(ep);
      e->ingestedDD.push_back(epd);
    }
  }
  e->pendingDD = e->ingestedDD;  // the ingested batch is the next run's input
  return LKF_OK;
}

int orc_ingest_twcc(orc_engine *e, uint32_t *out, uint32_t cap, uint32_t *n_out) {
  *n_out = u32(e->twcc.size());
  if (cap < e->twcc.size()) return LKF_ENOSPC;
  if (!e->twcc.empty()) std::memcpy(out, e->twcc.data(), e->twcc.size() * sizeof(u32));
  return LKF_OK;
}

int orc_ingest_flows(orc_engine *e, lkf_flow *out, uint32_t cap, uint32_t *n_out) {
  *n_out = u32(e->flows.size());
  if (cap < e->flows.size()) return LKF_ENOSPC;
  if (!e->flows.empty()) std::memcpy(out, e->flows.data(), e->flows.size() * sizeof(lkf_flow));
  return LKF_OK;
}

// The ExtPacket batch produced by the last orc_ingest (input of orc_run).
int orc_ingested_ptr(orc_engine *e, const lkf_pkt **pkts, uint32_t *n) {
  *pkts = e->ingested.data();
  *n = u32(e->ingested.size());
  return LKF_OK;
}
int orc_ingested_dd(orc_engine *e, lkf_pkt_dd *out, uint32_t cap, uint32_t *n_out) {
  *n_out = u32(e->ingestedDD.size());
  if (cap < e->ingestedDD.size()) return LKF_ENOSPC;
  if (!e->ingestedDD.empty()) std::memcpy(out, e->ingestedDD.data(), e->ingestedDD.size() * sizeof(lkf_pkt_dd));
  return LKF_OK;
}
int orc_ingested(orc_engine *e, lkf_pkt *out, uint32_t cap, uint32_t *n_out) {
  *n_out = u32(e->ingested.size());
  if (cap < e->ingested.size()) return LKF_ENOSPC;
  if (!e->ingested.empty()) std::memcpy(out, e->ingested.data(), e->ingested.size() * sizeof(lkf_pkt));
  return LKF_OK;
}

int orc_stream_stats_get(orc_engine *e, int32_t s, lkf_stream_stats *o) {
  if (s < 0 || s >= int32_t(e->streams.size())) return LKF_EINVAL;
  const RTPStatsReceiver &r = e->streams[s]->stats;
  std::memset(o, 0, sizeof(*o));
  o->initialized = r.initialized;
  o->ext_start_sn = r.sequenceNumber.GetExtendedStart();
  o->ext_highest_sn = r.sequenceNumber.GetExtendedHighest();
  o->ext_start_ts = r.timestamp.GetExtendedStart();
  o->ext_highest_ts = r.timestamp.GetExtendedHighest();
  o->packets_lost = r.packetsLost;
  o->packets_out_of_order = r.packetsOutOfOrder;
  o->packets_duplicate = r.packetsDuplicate;
  o->packets_padding = r.packetsPadding;
  o->bytes = r.bytes;
  o->header_bytes = r.headerBytes;
  o->bytes_duplicate = r.bytesDuplicate;
  o->bytes_padding = r.bytesPadding;
  o->frames = r.frames;
  o->nacks = e->streams[s]->nacks;
  o->first_time_ns = r.firstTime;
  o->highest_time_ns = r.highestTime;
  o->last_transit = r.lastTransit;
  o->last_jitter_ext_ts = r.lastJitterExtTimestamp;
  o->jitter = r.jitter;
  o->max_jitter = r.maxJitter;
  for (int i = 0; i < 101; i++) o->gap_histogram[i] = r.gapHistogram[i];
  return LKF_OK;
}

int orc_ingest_nacks(orc_engine *e, lkf_rtcp_nack *out, uint32_t cap, lkf_nack_pair *pairs, uint32_t pair_cap,
                     uint32_t *n_out, uint32_t *n_pairs_out) {
  *n_out = u32(e->nackRecs.size());
  *n_pairs_out = u32(e->nackPairs.size());
  if (cap < e->nackRecs.size() || pair_cap < e->nackPairs.size()) return LKF_ENOSPC;
  if (!e->nackRecs.empty()) std::memcpy(out, e->nackRecs.data(), e->nackRecs.size() * sizeof(lkf_rtcp_nack));
  if (!e->nackPairs.empty()) std::memcpy(pairs, e->nackPairs.data(), e->nackPairs.size() * sizeof(lkf_nack_pair));
  return LKF_OK;
}

int orc_stream_set_rtt(orc_engine *e, int32_t s, uint32_t rtt_ms) {  // Buffer.SetRTT buffer.go:400-414
  if (s < 0 || s >= int32_t(e->streams.size())) return LKF_EINVAL;
  if (rtt_ms == 0) return LKF_OK;
  if (e->streams[s]->nacker) e->streams[s]->nacker->SetRTT(rtt_ms);
  return LKF_OK;
}

// Room.GetActiveSpeakers (room.go:254-279) for every room, ascending room id.
// A microphone track's level is its primary receiver's (layer-0 stream's)
// AudioLevel.GetLevel(now) (mediatrackreceiver.go:755-762, buffer.go:840-849);
// a participant's level is the loudest active one (uptrackmanager.go:422-436).
int orc_speakers(orc_engine *e, int64_t now_ns, lkf_speaker *out, uint32_t cap, uint32_t *n_out) {
  std::vector<int> primary(e->tracks.size(), -1);
  for (size_t s = 0; s < e->streams.size(); s++)
    if (e->streams[s]->p.layer == 0 && primary[e->streams[s]->p.track] < 0) primary[e->streams[s]->p.track] = int(s);
  // room -> participant -> (level, active)
  std::vector<std::pair<u32, u32>> keys;  // (room, participant) in first-seen order
  struct Acc {
    double level = 0;
    bool active = false;
  };
  std::vector<Acc> acc;
  auto find = [&](u32 room, u32 part) -> size_t {
    for (size_t i = 0; i < keys.size(); i++)
      if (keys[i].first == room && keys[i].second == part) return i;
    keys.emplace_back(room, part);
    acc.emplace_back();
    return keys.size() - 1;
  };
  for (size_t t = 0; t < e->tracks.size(); t++) {
    const lkf_track_params &tp = e->tracks[t].p;
    size_t k = find(tp.room, tp.publisher);
    if (!tp.is_mic || e->tracks[t].removed || primary[t] < 0) continue;
    OStream &s = *e->streams[primary[t]];
    if (!s.level) continue;
    auto lv = s.level->GetLevel(now_ns);
    if (lv.second) {
      acc[k].active = true;
      if (lv.first > acc[k].level) acc[k].level = lv.first;
    }
  }
  std::vector<u32> rooms;
  for (auto &k : keys)
    if (std::find(rooms.begin(), rooms.end(), k.first) == rooms.end()) rooms.push_back(k.first);
  std::sort(rooms.begin(), rooms.end());
  std::vector<lkf_speaker> res;
  for (u32 room : rooms) {
    // participants of the room by ascending index (the tie order)
    std::vector<std::pair<u32, size_t>> ps;
    for (size_t i = 0; i < keys.size(); i++)
      if (keys[i].first == room) ps.emplace_back(keys[i].second, i);
    std::sort(ps.begin(), ps.end());
    std::vector<std::pair<double, bool>> levels;
    std::vector<u32> pidx;
    for (auto &p : ps) {
      levels.emplace_back(acc[p.second].level, acc[p.second].active);
      pidx.push_back(p.first);
    }
    for (auto &sp : RankSpeakers(levels)) {
      lkf_speaker o{};
      o.room = room;
      o.participant = pidx[sp.participant];
      o.level = sp.level;
      o.active = 1;
      res.push_back(o);
    }
  }
  *n_out = u32(res.size());
  if (cap < res.size()) return LKF_ENOSPC;
  if (!res.empty()) std::memcpy(out, res.data(), res.size() * sizeof(lkf_speaker));
  return LKF_OK;
}

}  // extern "C"
