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
#include <memory>
#include <thread>

#include "../include/lkfwd.h"
#include "lkf_oracle.h"

using namespace orc;

namespace {

struct OTrack {
  lkf_track_params p;
};

struct OOut {
  lkf_out rec;
  std::vector<u8> bytes;
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
};

struct OEv {
  int32_t dt, op;
  int64_t a[4];
  uint32_t at;
};

}  // namespace

struct orc_engine {
  u32 seqSize = 500;
  std::vector<OTrack> tracks;
  std::vector<std::unique_ptr<ODT>> dts;
  std::vector<OEv> pending;
  lkf_stats stats{};
  std::vector<lkf_out> outRecs;
  std::vector<u8> outArena;
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

static ExtPacket toExt(const lkf_pkt &d, const u8 *arena) {
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
  }
  return p;
}

// DownTrack.WriteRTP downtrack.go:680-760 on the virtual clock.
static void writeRTP(orc_engine *e, u32 dtIdx, ODT &d, const ExtPacket &ep, u32 pktIdx, int8_t layer) {
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
  // pacer Base.writeRTPHeaderExtensions pacer/base.go:71-100 (DD bytes are
  // never produced by the VP8/Opus selectors; abs-send-time is a 3-byte
  // placeholder the sender stamps — wall clock excluded from parity)
  hdr.Extension = false;
  hdr.ExtensionProfile = 0;
  hdr.Extensions.clear();
  if (d.p.ext_playout && !d.playoutAcked)
    hdr.SetExtension(d.p.ext_playout, std::vector<u8>(d.p.playout_delay, d.p.playout_delay + 3));
  if (d.p.ext_abs_send_time) hdr.SetExtension(d.p.ext_abs_send_time, std::vector<u8>{0, 0, 0});
  // sequencer.push downtrack.go:724-735
  i64 arrivalMs = ep.Arrival / 1000000;
  d.seq->push(arrivalMs, ep.ExtSequenceNumber, tp.rtp.extSequenceNumber, tp.rtp.extTimestamp, hdr.Marker, i8(layer),
              tp.codecBytes, {});
  // sendingPacket -> RTPStatsSender.Update init (rtpstats_sender.go:245-262)
  if (!d.statsInit && !payload.empty()) {
    d.statsInit = true;
    d.firstTime = ep.Arrival;
    d.extStartTS = tp.rtp.extTimestamp;
  }
  OOut o;
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
  e->tracks.push_back(OTrack{*p});
  return int32_t(e->tracks.size() - 1);
}

int32_t orc_add_downtrack(orc_engine *e, const lkf_downtrack_params *p) {
  if (p->track < 0 || p->track >= (int)e->tracks.size()) return LKF_EINVAL;
  auto d = std::make_unique<ODT>();
  d->p = *p;
  const lkf_track_params &tp = e->tracks[p->track].p;
  Kind k = tp.kind == LKF_KIND_VIDEO ? KindVideo : KindAudio;
  d->f = std::make_unique<Forwarder>(k);
  Mime m = tp.codec == LKF_CODEC_VP8 ? MimeVP8 : tp.codec == LKF_CODEC_H264 ? MimeH264 : MimeOpus;
  d->f->DetermineCodec(m, tp.clock_rate);
  d->seq = std::make_unique<Sequencer>(int(e->seqSize), k == KindVideo, p->bind_time_ns / 1000000);
  ODT *dp = d.get();
  int32_t track = p->track;
  if (tp.has_ref_ts) {
    // StreamTrackerManager.GetReferenceLayerRTPTimestamp streamtrackermanager.go:660-679
    dp->f->getReferenceLayerRTPTimestamp = [e, track](u32 ts, i32 layer, i32 ref, u32 &out) -> Err {
      if (layer < 0 || layer >= 3 || ref < 0 || ref >= 3) return ErrRefLayerUnavailable;
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

int orc_set_layer_offsets(orc_engine *e, int32_t track, const uint32_t *offs) {
  if (track < 0 || track >= (int)e->tracks.size()) return LKF_EINVAL;
  std::memcpy(e->tracks[track].p.layer_offsets, offs, sizeof(uint32_t) * 9);
  return LKF_OK;
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

// Runs one batch; pkts grouped by track (lkf_submit contract).
int orc_run(orc_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len) {
  (void)arena_len;
  std::memset(&e->stats, 0, sizeof(e->stats));
  const u32 ndt = u32(e->dts.size());
  std::vector<std::vector<OEv>> evq(ndt);
  for (auto &ev : e->pending) evq[ev.dt].push_back(ev);
  e->pending.clear();
  for (auto &q : evq)
    std::stable_sort(q.begin(), q.end(), [](const OEv &a, const OEv &b) { return a.at < b.at; });
  std::vector<size_t> evc(ndt, 0);
  std::vector<std::vector<u32>> trackDts(e->tracks.size());
  for (u32 d = 0; d < ndt; d++) {
    e->dts[d]->outs.clear();
    if (e->dts[d]->active) trackDts[e->dts[d]->p.track].push_back(d);
  }
  for (u32 i = 0; i < n; i++) {
    const lkf_pkt &pd = pkts[i];
    if (pd.track >= e->tracks.size()) return LKF_EINVAL;
    ExtPacket ep = toExt(pd, arena);
    for (u32 d : trackDts[pd.track]) {
      ODT &dt = *e->dts[d];
      while (evc[d] < evq[d].size() && evq[d][evc[d]].at <= i) applyCtl(e, dt, evq[d][evc[d]++]);
      writeRTP(e, d, dt, ep, i, pd.layer);
    }
  }
  for (u32 d = 0; d < ndt; d++)
    while (evc[d] < evq[d].size()) applyCtl(e, *e->dts[d], evq[d][evc[d]++]);
  // Output order: by track, then DownTrack handle, then packet; wire packets
  // 16-B aligned.  (An engine-defined batch layout: the reference hands each
  // packet to its DownTrack's pacer directly.)
  e->outRecs.clear();
  e->outArena.clear();
  u64 off = 0;
  for (auto &tds : trackDts)
    for (u32 d : tds)
      for (auto &o : e->dts[d]->outs) {
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

}  // extern "C"
