// synth.cpp — deterministic synthetic RTP workloads.
//
// Media model: VP8 3-layer simulcast L1T3 at 30 fps
// (q: 1 pkt/frame ~600 B, h: 2 pkt/frame ~1000 B, f: 7 pkt/frame ~1100 B),
// Opus 50 pkt/s 40-160 B.  Raw packets carry a one-byte header-extension
// block (transport-cc seq for video, RFC 6464 audio level for audio), as a
// browser publisher sends them.  Control scripts mirror what the reference's
// control plane drives into the Forwarder (SetMax*, updateAllocation, Mute).
#include "synth.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

struct Rng {
  u64 s;
  explicit Rng(u64 seed) : s(seed) {}
  u64 next() {  // splitmix64
    u64 z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
  u32 below(u32 n) { return u32(uni() * n) % (n ? n : 1); }
};

constexpr i64 NS = 1000000000LL;
constexpr i64 MS = 1000000LL;
constexpr u16 kPayloadOff = 20;  // 12-byte header + 8-byte one-byte-ext block

struct Plan {
  std::vector<u8> dd;  // dependency-descriptor extension payload (DD tracks)
  u64 extFn;           // unwrapped frame number (DD tracks)
  u8 ddAttach;         // structure attached
  u8 ddActive;         // active decode targets bitmask present
  u32 ddMask;
  u8 frameId;          // frame identity within a track for the integrity model: (superframe, spatial)
  u8 framePkts;
  i64 arrival;
  u64 ext_sn;
  u64 ext_ts;
  u32 ssrc;
  u16 payload_len;
  u16 pid;
  u16 twcc;
  int8_t layer;
  u8 tid;
  u8 tl0;
  u8 marker;
  u8 keyframe;  // S && P==0 (first packet of a key frame)
  u8 s_bit;
  u8 y_bit;
  u8 level;
  u8 pt;
  u8 vp9;  // LKF_VP9_* flags (config 5 SVC packets)
  u8 lost; // (svc_dd = 3) lost by the scripted burst, whatever the random loss draws
};

struct TrackGen {
  lkf_track_params p;
  int nlayers = 1;
  bool svc = false;         // VP9 SVC: all spatial layers in one stream (one SSRC)
  bool dd = false;          // dependency descriptor on every packet (AV1, or VP9 with DD)
  u32 ssrc[3] = {0, 0, 0};  // per received layer (one ingress stream each)
  std::vector<Plan> plans;  // merged arrival order
};

struct Ev {
  int32_t dt;
  int32_t op;
  int64_t a[4];
  i64 t;  // virtual time; < 0 = before the first packet
};

const int kPktsPerFrame[3] = {1, 2, 7};
const int kPayloadMean[3] = {600, 1000, 1100};

}  // namespace

struct lkfs_trace {
  std::vector<lkf_track_params> tracks;
  std::vector<lkf_downtrack_params> dts;
  std::vector<u64> batch_pkt_off;    // nb+1
  std::vector<u64> batch_raw_off;    // nb+1 (raw datagrams: a superset of the ExtPackets)
  std::vector<u64> batch_arena_off;  // nb+1
  std::vector<lkf_pkt> pkts;
  std::vector<lkf_raw_pkt> raws;  // the same datagrams as raw ingress input
  std::vector<lkf_stream_params> streams;
  std::vector<u8> arena;
  std::vector<u64> batch_ev_off;
  std::vector<lkfs_event> events;
  std::vector<lkf_pkt_dd> dds;  // parallel to pkts
  u32 max_batch_pkts = 0;
  u64 max_batch_arena = 0;
  u64 max_batch_tuples = 0;
  u64 max_batch_out_bytes = 0;  // bound on one batch's output arena (every tuple forwarded)
};

static void fill_payload(u8 *dst, int n, u64 key) {
  u64 x = key * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    std::memcpy(dst + i, &x, 8);
  }
  for (; i < n; i++) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    dst[i] = u8(x);
  }
}

// ---- dependency-descriptor encoder (the publisher side of config 5) -----------
// L3T3 with inter-layer prediction: per spatial layer s four templates (key T0,
// T0, T1, T2), 9 decode targets (s*3 + t) protected by chain s (chain c = the
// T0 frames of spatial layer c), resolutions 320x180 / 640x360 / 1280x720.
// Frames that deviate from their template (chain diffs after a skipped layer,
// the second reference of odd T2 frames) carry custom fields.
// The wide form (svc_dd = 2) takes the reader to the reference's maxima: one
// chain per decode target (chain c follows spatial layer c / 3, so 9 chains),
// T2 templates with 17 frame diffs, custom frame-diff lists of 9 and 18.
struct DDTmplGen {
  int sid, tid;
  std::vector<int> fd, chains, dtis;
};
static std::vector<DDTmplGen> dd_templates(bool wide) {
  static const int ch[3][4][3] = {{{0, 0, 0}, {12, 11, 10}, {6, 5, 4}, {3, 2, 1}},
                                  {{1, 0, 0}, {1, 12, 11}, {7, 6, 5}, {4, 3, 2}},
                                  {{2, 1, 0}, {2, 1, 12}, {8, 7, 6}, {5, 4, 3}}};
  std::vector<DDTmplGen> v;
  for (int sp = 0; sp < 3; sp++)
    for (int k = 0; k < 4; k++) {
      DDTmplGen t;
      t.sid = sp;
      t.tid = k <= 1 ? 0 : k - 1;
      static const int base[4] = {0, 12, 6, 3};
      if (k > 0) t.fd.push_back(base[k]);
      if (sp > 0) t.fd.push_back(1);
      static const int more[4] = {6, 12, 9, 3};
      if (wide && k == 3)
        for (int j = 0; t.fd.size() < 17; j++) t.fd.push_back(more[j % 4]);
      if (wide)
        for (int c = 0; c < 9; c++) t.chains.push_back(ch[sp][k][c / 3]);
      else
        t.chains.assign(ch[sp][k], ch[sp][k] + 3);
      for (int tg = 0; tg < 9; tg++) {
        const int s2 = tg / 3, t2 = tg % 3;
        int x = 0;
        if (s2 >= t.sid && t2 >= t.tid) x = (k == 0) ? 2 : (k == 3 ? 1 : (s2 == t.sid ? 2 : 3));
        t.dtis.push_back(x);
      }
      v.push_back(t);
    }
  return v;
}
struct BitOut {
  std::vector<u8> b;
  int n = 0;
  void put(u64 v, int bits) {
    for (int i = bits - 1; i >= 0; i--) {
      if ((n >> 3) >= int(b.size())) b.push_back(0);
      if ((v >> i) & 1) b[size_t(n >> 3)] |= u8(0x80u >> (n & 7));
      n++;
    }
  }
  void ns(u32 v, u32 numValues) {  // av1 ns(n)
    if (numValues == 1) return;
    int w = 0;
    for (u32 x = numValues; x; x >>= 1) w++;
    const u32 m = (1u << w) - numValues;
    if (v < m)
      put(v, w - 1);
    else
      put(v + m, w);
  }
};
static std::vector<u8> dd_encode(const std::vector<DDTmplGen> &T, int structureId, bool first, bool last, int tmpl,
                                 u16 fn, bool attach, bool active, u32 mask, const std::vector<int> &fd,
                                 const std::vector<int> &chains) {
  const DDTmplGen &t = T[size_t(tmpl)];
  const bool cFd = fd != t.fd, cCh = chains != t.chains;
  BitOut o;
  o.put(first, 1);
  o.put(last, 1);
  o.put(u64((tmpl + structureId) % 64), 6);
  o.put(fn, 16);
  if (attach || active || cFd || cCh) {
    o.put(attach, 1);
    o.put(active, 1);
    o.put(0, 1);
    o.put(cFd, 1);
    o.put(cCh, 1);
    if (attach) {
      o.put(u64(structureId), 6);
      o.put(9 - 1, 5);
      for (size_t i = 1; i < T.size(); i++) {
        const int idc = (T[i].sid == T[i - 1].sid && T[i].tid == T[i - 1].tid) ? 0 : (T[i].sid == T[i - 1].sid) ? 1 : 2;
        o.put(u64(idc), 2);
      }
      o.put(3, 2);
      for (auto &x : T)
        for (int d : x.dtis) o.put(u64(d), 2);
      for (auto &x : T) {
        for (int f : x.fd) o.put((1u << 4) | u32(f - 1), 5);
        o.put(0, 1);
      }
      const u32 nch = u32(T[0].chains.size());
      o.ns(nch, 9 + 1);
      for (int tg = 0; tg < 9; tg++) o.ns(nch == 9 ? u32(tg) : u32(tg / 3), nch);
      for (auto &x : T)
        for (int c : x.chains) o.put(u64(c), 4);
      o.put(1, 1);
      static const int W[3] = {320, 640, 1280}, H[3] = {180, 360, 720};
      for (int i = 0; i < 3; i++) {
        o.put(u64(W[i] - 1), 16);
        o.put(u64(H[i] - 1), 16);
      }
    }
    if (active) o.put(mask, 9);
    if (cFd) {
      for (int f : fd) {
        if (f <= 16)
          o.put((1u << 4) | u32(f - 1), 6);
        else if (f <= 256)
          o.put((2u << 8) | u32(f - 1), 10);
        else
          o.put((3u << 12) | u32(f - 1), 14);
      }
      o.put(0, 2);
    }
    if (cCh)
      for (int c : chains) o.put(u64(c & 0xff), 8);
  }
  return o.b;
}

extern "C" lkfs_trace *lkfs_generate(const lkfs_cfg *cfg) {
  if (!cfg || cfg->config < 1 || cfg->config > 5) return nullptr;
  const int C = cfg->config;
  // Every room and every track draws from its own splitmix64 stream keyed by
  // its global id, so a shard (room_base, rooms) generates exactly the rooms
  // the full trace would: room sharding across GPUs changes no packet.
  const u64 seedBase = cfg->seed ? cfg->seed : (0x4C4Bull + u64(C));
  auto keyed = [&](u64 key) {
    Rng k(seedBase ^ (key * 0xD6E8FEB86659FD93ull));
    k.next();
    return Rng(k.next());
  };
  const double dur = cfg->duration_s > 0 ? cfg->duration_s : 10.0;
  const double bs = cfg->batch_s > 0 ? cfg->batch_s : 1.0;
  const i64 durNs = i64(dur * NS);
  const i64 batchNs = i64(bs * NS);
  const bool withEvents = cfg->with_events != 0;
  const bool cb = cfg->has_callbacks != 0;
  const bool svcDD = cfg->svc_dd != 0;
  const bool ddWide = cfg->svc_dd == 2;
  // svc_dd = 3: as 1, with chain 0 following every frame (custom chain diffs:
  // the previous frame number) and, for 2 s of every 3, every other frame
  // number lost: each arriving frame then waits on the lost one before it, so
  // a chain holds dozens of expected frames (FrameChain.expectFrames) until
  // the oldest ages out of the decision cache's NACK window and breaks it
  const bool ddBurst = cfg->svc_dd == 3;
  const bool h264 = cfg->h264 > 0;

  u32 rooms = cfg->rooms, parts = cfg->participants;
  double loss = cfg->loss, reorder = cfg->reorder;
  switch (C) {
    case 1:
      if (!rooms) rooms = 1;
      if (!parts) parts = 10;
      if (loss < 0) loss = 0;
      if (reorder < 0) reorder = 0;
      break;
    case 2:
      if (!rooms) rooms = 100;
      if (!parts) parts = 10;
      if (loss < 0) loss = 0.02;
      if (reorder < 0) reorder = 0.01;
      break;
    case 3:
      if (!rooms) rooms = 125;
      if (!parts) parts = 50;
      if (loss < 0) loss = 0.0;
      if (reorder < 0) reorder = 0.0;
      break;
    case 4:
      if (!rooms) rooms = 10;
      if (!parts) parts = 5000;
      if (loss < 0) loss = 0.0;
      if (reorder < 0) reorder = 0.0;
      break;
    case 5:  // VP9 L3T3 SVC + Opus DTX, congestion-driven layer changes
      if (!rooms) rooms = 2000;
      if (!parts) parts = 5;
      if (loss < 0) loss = 0.01;
      if (reorder < 0) reorder = 0.005;
      break;
  }

  auto *tr = new lkfs_trace();
  std::vector<TrackGen> tg;
  std::vector<Ev> evs;
  const i64 t0 = 1700000000LL * NS;  // virtual epoch

  // ---- topology -------------------------------------------------------
  struct RoomTracks {
    std::vector<int> video;  // track handles
    std::vector<u32> videoPub;
    std::vector<int> audio;
    std::vector<u32> audioPub;
  };
  for (u32 r = 0; r < rooms; r++) {
    const u32 room = cfg->room_ids ? cfg->room_ids[r] : cfg->room_base + r;
    Rng rng = keyed((1ull << 40) + room);
    const size_t dt0 = tr->dts.size();
    RoomTracks rt;
    u32 npub = (C == 1 || C == 4) ? 1 : parts;
    for (u32 p = 0; p < npub; p++) {
      bool hasVideo = (C != 3) || (p < 5);
      if (hasVideo) {
        TrackGen g{};
        g.p.track_id = (u64(room) << 32) | (u64(p) << 8) | 1;
        g.p.room = room;
        g.p.publisher = p;
        g.p.kind = LKF_KIND_VIDEO;
        g.p.codec = C == 5 ? LKF_CODEC_VP9 : LKF_CODEC_VP8;
        g.svc = C == 5;
        if (h264 && C <= 3 && (p % 3) == (C == 1 ? 0u : 1u)) g.p.codec = LKF_CODEC_H264;
        // configs[4]: AV1 (DD only) and VP9 with DD beside VP9-descriptor publishers
        if (C == 5 && svcDD && (p % 4) != 3) {
          g.dd = true;
          g.p.has_dd = 1;
          if ((p % 4) != 2) g.p.codec = LKF_CODEC_AV1;
        }
        g.p.has_ref_ts = cb ? 1 : 0;
        g.p.is_mic = 0;
        g.p.clock_rate = 90000;
        g.nlayers = (C == 3) ? 1 : 3;
        rt.video.push_back((int)tg.size());
        rt.videoPub.push_back(p);
        tg.push_back(g);
      }
      TrackGen a{};
      a.p.track_id = (u64(room) << 32) | (u64(p) << 8) | 2;
      a.p.room = room;
      a.p.publisher = p;
      a.p.kind = LKF_KIND_AUDIO;
      a.p.codec = LKF_CODEC_OPUS;
      a.p.has_ref_ts = cb ? 1 : 0;
      a.p.is_mic = 1;
      a.p.clock_rate = 48000;
      a.nlayers = 1;
      rt.audio.push_back((int)tg.size());
      rt.audioPub.push_back(p);
      tg.push_back(a);
    }
    // subscribers
    u32 nsub = (C == 1 || C == 4) ? parts : parts;
    for (u32 s = 0; s < nsub; s++) {
      u32 subId = (C == 1 || C == 4) ? (1000000 + s) : s;
      auto addDT = [&](int track, bool video) {
        lkf_downtrack_params d{};
        d.track = track;
        d.subscriber = subId;
        d.ssrc = u32(rng.next()) | 1u;
        d.payload_type = video ? 96 : 111;
        d.ext_dd = (video && tg[track].dd && (s % 3) != 2) ? 9 : 0;  // some subscribers lack the DD extension
        d.ext_playout = 0;
        d.ext_abs_send_time = video ? 3 : 0;
        if (video && (cfg->twcc >= 2 || (cfg->twcc == 1 && (s % 2) == 0))) {  // send-side BWE subscriber
          d.ext_abs_send_time = 0;
          d.ext_transport_cc = 5;
        }
        d.has_expected_ts = cb ? 1 : 0;
        d.bind_time_ns = t0 - 50 * MS;
        int dt = (int)tr->dts.size();
        tr->dts.push_back(d);
        if (!video) return;
        // subscription settings + publisher layer info (control plane)
        evs.push_back(Ev{dt, LKF_CTL_SET_MAX_SPATIAL, {tg[track].nlayers - 1, 0, 0, 0}, -1});
        evs.push_back(Ev{dt, LKF_CTL_SET_MAX_TEMPORAL, {2, 0, 0, 0}, -1});
        evs.push_back(Ev{dt, LKF_CTL_SET_MAX_SEEN_SPATIAL, {tg[track].nlayers - 1, 0, 0, 0}, -1});
        evs.push_back(Ev{dt, LKF_CTL_SET_MAX_SEEN_TEMPORAL, {2, 0, 0, 0}, -1});
        int nl = tg[track].nlayers;
        int ts;
        if (C == 1)
          ts = s < 5 ? 2 : (s < 8 ? 1 : 0);
        else if (C == 4)
          ts = rng.uni() < 0.8 ? 2 : int(rng.below(2));
        else
          ts = int(rng.below(u32(nl)));
        if (ts > nl - 1) ts = nl - 1;
        evs.push_back(Ev{dt, LKF_CTL_SET_ALLOCATION, {ts, 2, ts, 0}, -1});
        if (withEvents && (C == 2 || C == 5)) {
          // congestion/subscription script: new target every 2 s (config 5:
          // every 1 s, spatial and temporal) per DT; deficient on downgrades
          const i64 period = C == 5 ? NS : 2 * NS;
          i64 phase = i64(rng.uni() * double(period));
          int cur = ts;
          for (i64 t = phase; t < durNs; t += period) {
            int ns = int(rng.below(u32(nl)));
            int nt = C == 5 ? int(rng.below(3)) : 1 + int(rng.below(2));
            bool deficient = ns < cur;
            evs.push_back(Ev{dt, LKF_CTL_SET_ALLOCATION, {ns, nt, ns, deficient ? 1 : 0}, t0 + t});
            cur = ns;
          }
        }
      };
      for (size_t i = 0; i < rt.video.size(); i++)
        if (C == 1 || C == 4 || rt.videoPub[i] != s) addDT(rt.video[i], true);
      for (size_t i = 0; i < rt.audio.size(); i++)
        if (C == 1 || C == 4 || rt.audioPub[i] != s) addDT(rt.audio[i], false);
    }
    // occasional subscriber mute/unmute (exercises resync + resume path)
    if (withEvents && (C == 2 || C == 3)) {
      for (int dt = int(dt0); dt < (int)tr->dts.size(); dt++) {
        if (rng.uni() < 0.05) {
          i64 t = i64(rng.uni() * (durNs * 0.7));
          i64 len = i64((0.3 + rng.uni()) * NS);
          evs.push_back(Ev{dt, LKF_CTL_MUTE, {1, 1, 0, 0}, t0 + t});
          evs.push_back(Ev{dt, LKF_CTL_MUTE, {0, 1, 0, 0}, t0 + t + len});
        }
      }
    }
  }

  // ---- keyframe schedule (periodic + PLI-triggered, throttled) --------
  // PLI: every allocation event that changes the target spatial layer asks
  // for a key frame on that layer 100 ms later; pli_throttle 500 ms/layer.
  std::vector<std::vector<std::vector<i64>>> kfReq(tg.size());
  for (size_t t = 0; t < tg.size(); t++) kfReq[t].assign(3, {});
  for (auto &e : evs) {
    if (e.op != LKF_CTL_SET_ALLOCATION || e.t < 0) continue;
    int track = tr->dts[e.dt].track;
    int l = int(e.a[0]);
    if (l >= 0 && l < 3) kfReq[track][l].push_back(e.t - t0 + 100 * MS);
  }

  // ---- per-track packet plans -------------------------------------------
  for (size_t ti = 0; ti < tg.size(); ti++) {
    TrackGen &g = tg[ti];
    Rng rng = keyed(g.p.track_id);
    std::vector<std::vector<Plan>> streams(g.nlayers);
    i64 netDelay = 20 * MS + i64(rng.below(10)) * MS;
    if (g.p.kind == LKF_KIND_VIDEO && g.svc) {
      // VP9 L3T3 SVC, 30 fps: every frame carries spatial layers 0..2 in one
      // RTP stream (one SSRC, one sequence, one timestamp per superframe).
      // Temporal pattern T0 T2 T1 T2; U (switching-up point) on T1/T2 frames;
      // B/E on the first/last packet of a layer frame; P unless the
      // superframe is a key superframe; marker on the superframe's last packet.
      static const int kSvcPkts[3] = {1, 2, 3};
      static const int kSvcPayload[3] = {300, 600, 1000};
      u32 ssrc = u32(rng.next()) | 1u;
      g.ssrc[0] = ssrc;
      u64 sn = u64(u16(rng.next()));
      u32 tsBase = u32(rng.next());
      u16 pid0 = u16(rng.next() & 0x7fff);
      u8 tl00 = u8(rng.next());
      u16 twcc = u16(rng.next());
      // dependency descriptor (DD tracks only: the RNG stream of VP9 tracks is unchanged)
      static const std::vector<DDTmplGen> ddT3 = dd_templates(false), ddT9 = dd_templates(true);
      const std::vector<DDTmplGen> &ddT = ddWide ? ddT9 : ddT3;
      int structureId = 0;
      u64 fn0 = 0;
      bool reducedTrack = false;
      if (g.dd) {
        structureId = int(rng.below(64));
        fn0 = u64(ti % 5 == 0 ? u16(65536 - 40 - rng.below(40)) : u16(rng.next()));  // some wrap early
        reducedTrack = (ti % 2) == 0;  // publisher drops S2 (active targets 0x3F) for 1 s
      }
      u64 lastChain[3] = {0, 0, 0};
      u64 lastAny = 0;  // (svc_dd = 3) the previous frame number
      bool wasReduced = false;
      std::vector<i64> reqs;
      for (int l = 0; l < 3; l++) reqs.insert(reqs.end(), kfReq[ti][l].begin(), kfReq[ti][l].end());
      std::sort(reqs.begin(), reqs.end());
      size_t ri = 0;
      i64 lastKf = -10 * NS;
      int nframes = int(dur * 30.0);
      for (int f = 0; f < nframes; f++) {
        i64 cap = i64(f) * NS / 30;
        bool kf = (f % 60) == 0;
        while (ri < reqs.size() && reqs[ri] <= cap) {
          if (cap - lastKf >= 500 * MS) kf = true;
          ri++;
        }
        if (kf) lastKf = cap;
        int tid = (f % 4 == 0) ? 0 : ((f % 4 == 2) ? 1 : 2);
        const bool reduced = g.dd && reducedTrack && cap >= 2 * NS && cap < 3 * NS;
        const bool sendMask = g.dd && (reduced || wasReduced);  // the change and the period
        wasReduced = reduced;
        int k = 0;
        for (int sl = 0; sl < 3; sl++) {
          if (reduced && sl == 2) continue;  // S2 not encoded
          // the layer frame's descriptor (same template/custom fields on each packet)
          std::vector<int> fdv, chv;
          int tmpl = 0;
          const u64 efn = fn0 + u64(f) * 3 + u64(sl);
          if (g.dd) {
            const int kk = kf ? 0 : (tid == 0 ? 1 : (tid == 1 ? 2 : 3));
            tmpl = sl * 4 + kk;
            fdv = ddT[size_t(tmpl)].fd;
            if (!kf && tid == 2 && f % 4 == 3) fdv.push_back(9);
            if (ddWide && !kf && tid == 1 && f % 8 == 2)  // a custom list of 9-10
              for (int j = 0; j < 8; j++) fdv.push_back(j % 2 ? 6 : 12);
            const int nch = int(ddT[size_t(tmpl)].chains.size());
            if (kf) {
              chv = ddT[size_t(tmpl)].chains;
            } else {
              for (int c = 0; c < nch; c++) chv.push_back(int(std::min<u64>(255, efn - lastChain[nch == 9 ? c / 3 : c])));
              if (ddBurst && efn > lastAny && lastAny) chv[0] = int(std::min<u64>(255, efn - lastAny));
            }
            if (kf || tid == 0) lastChain[sl] = efn;
            lastAny = efn;
          }
          for (int q = 0; q < kSvcPkts[sl]; q++, k++) {
            Plan pl{};
            pl.arrival = t0 + cap + netDelay + i64(k) * 150000 + i64(rng.below(2000000));
            pl.ext_sn = sn++;
            pl.ext_ts = u64(tsBase) + u64(f) * 3000;
            pl.ssrc = ssrc;
            int m = kSvcPayload[sl];
            pl.payload_len = u16(m - m / 10 + int(rng.below(u32(m / 5))));
            pl.pid = u16((pid0 + f) & 0x7fff);
            pl.twcc = twcc++;
            pl.layer = int8_t(sl);
            pl.tid = u8(tid);
            pl.tl0 = u8(tl00 + f / 4);
            pl.marker = sl == 2 && q == kSvcPkts[sl] - 1;
            pl.s_bit = q == 0;
            pl.keyframe = kf && sl == 0 && q == 0;  // IsVP9KeyFrame (helpers.go:317-336)
            pl.vp9 = u8(LKF_VP9_I | LKF_VP9_L | (kf ? 0 : LKF_VP9_P) | (q == 0 ? LKF_VP9_B : 0) |
                        (q == kSvcPkts[sl] - 1 ? LKF_VP9_E : 0) | (tid > 0 ? LKF_VP9_U : 0));
            pl.pt = g.p.codec == LKF_CODEC_AV1 ? 35 : 98;
            pl.lost = u8(ddBurst && g.dd && !kf && (f % 90) >= 15 && (f % 90) < 75 && (efn & 1));
            if (g.dd) {
              const bool attach = kf && sl == 0 && q == 0;
              pl.tid = u8(ddT[size_t(tmpl)].tid);  // the descriptor's TemporalId (key superframes: T0)
              const bool act = q == 0 && sl == 0 && (sendMask || (attach && reduced));
              pl.extFn = efn;
              pl.ddAttach = attach;
              pl.ddActive = act;
              pl.ddMask = reduced ? 0x3Fu : 0x1FFu;
              pl.frameId = u8(sl);
              pl.framePkts = u8(kSvcPkts[sl]);
              pl.dd = dd_encode(ddT, structureId, q == 0, q == kSvcPkts[sl] - 1, tmpl, u16(efn), attach, act,
                                pl.ddMask, fdv, chv);
            }
            streams[0].push_back(pl);
          }
        }
      }
    } else if (g.p.kind == LKF_KIND_VIDEO) {
      u32 tsBase[3];
      for (int l = 0; l < g.nlayers; l++) tsBase[l] = u32(rng.next());
      for (int r = 0; r < 3; r++)
        for (int l = 0; l < 3; l++)
          g.p.layer_offsets[r][l] = (r < g.nlayers && l < g.nlayers && r != l) ? u32(tsBase[r] - tsBase[l]) : 0;
      for (int l = 0; l < g.nlayers; l++) {
        int lq = g.nlayers == 1 ? 0 : l;
        u32 ssrc = u32(rng.next()) | 1u;
        g.ssrc[l] = ssrc;
        u64 sn = u64(u16(rng.next()));
        u16 pid0 = u16(rng.next() & 0x7fff);
        u8 tl00 = u8(rng.next());
        u16 twcc = u16(rng.next());
        auto &reqs = kfReq[ti][l];
        std::sort(reqs.begin(), reqs.end());
        size_t ri = 0;
        i64 lastKf = -10 * NS;
        int nframes = int(dur * 30.0);
        for (int f = 0; f < nframes; f++) {
          i64 cap = i64(f) * NS / 30;
          bool kf = (f % 60) == 0;
          while (ri < reqs.size() && reqs[ri] <= cap) {
            if (cap - lastKf >= 500 * MS) kf = true;
            ri++;
          }
          if (kf) lastKf = cap;
          int tid = (f % 4 == 0) ? 0 : ((f % 4 == 2) ? 1 : 2);
          bool y = (f % 4 == 1) || (f % 4 == 2);
          int np = kPktsPerFrame[lq];
          for (int k = 0; k < np; k++) {
            Plan pl{};
            pl.arrival = t0 + cap + netDelay + i64(k) * 150000 + i64(rng.below(2000000));
            pl.ext_sn = sn++;
            pl.ext_ts = u64(tsBase[l]) + u64(f) * 3000;
            pl.ssrc = ssrc;
            int m = kPayloadMean[lq];
            pl.payload_len = u16(m - m / 10 + int(rng.below(u32(m / 5))));
            pl.pid = u16((pid0 + f) & 0x7fff);
            pl.twcc = twcc++;
            pl.layer = int8_t(l);
            pl.tid = u8(tid);
            pl.tl0 = u8(tl00 + f / 4);
            pl.marker = k == np - 1;
            pl.s_bit = k == 0;
            pl.keyframe = kf && k == 0;
            pl.y_bit = y;
            pl.pt = 96;
            streams[l].push_back(pl);
          }
        }
      }
    } else {
      u32 ssrc = u32(rng.next()) | 1u;
      g.ssrc[0] = ssrc;
      u64 sn = u64(u16(rng.next()));
      u32 ts0 = u32(rng.next());
      int npk = int(dur * 50.0);
      bool talking = rng.uni() < 0.33;
      i64 nextFlip = i64((talking ? 2.0 : 4.0) * -std::log(1.0 - rng.uni()) * NS);
      for (int k = 0; k < npk; k++) {
        i64 cap = i64(k) * 20 * MS;
        while (cap >= nextFlip) {
          talking = !talking;
          nextFlip += i64((talking ? 2.0 : 4.0) * -std::log(1.0 - rng.uni()) * NS) + 1;
        }
        if (C == 5 && !talking && (k % 20) != 0) continue;  // Opus DTX: one frame per 400 ms in silence
        Plan pl{};
        pl.arrival = t0 + cap + netDelay + i64(rng.below(2000000));
        pl.ext_sn = sn++;
        pl.ext_ts = u64(ts0) + u64(k) * 960;
        pl.ssrc = ssrc;
        pl.payload_len = u16(40 + rng.below(121));
        pl.layer = 0;
        pl.marker = 0;
        pl.level = talking ? u8(20 + rng.below(21)) : u8(90 + rng.below(38));
        pl.pt = 111;
        streams[0].push_back(pl);
      }
    }
    // per-stream reorder (depth <= 3) and loss, then merge by arrival
    for (auto &st : streams) {
      // monotonic arrivals in send order
      for (size_t i = 1; i < st.size(); i++)
        if (st[i].arrival <= st[i - 1].arrival) st[i].arrival = st[i - 1].arrival + 1000;
      if (reorder > 0) {
        for (size_t i = 0; i + 1 < st.size(); i++) {
          // DD streams keep their first packets in order: a packet older than
          // the stream's first one is not handled at ingress
          // (rtpstats_receiver.go), and the dependency descriptor of the
          // opening key frame must reach the parser for the stream to be readable
          if (rng.uni() < reorder && !(g.dd && i < 8)) {
            size_t j = std::min(st.size() - 1, i + 1 + rng.below(3));
            std::swap(st[i].arrival, st[j].arrival);
          }
        }
      }
      std::vector<Plan> kept;
      kept.reserve(st.size());
      for (auto &pl : st)
        if (!(loss > 0 && rng.uni() < loss) && !pl.lost) kept.push_back(pl);
      st.swap(kept);
      std::stable_sort(st.begin(), st.end(), [](const Plan &a, const Plan &b) { return a.arrival < b.arrival; });
    }
    for (auto &st : streams) g.plans.insert(g.plans.end(), st.begin(), st.end());
    std::stable_sort(g.plans.begin(), g.plans.end(), [](const Plan &a, const Plan &b) {
      if (a.arrival != b.arrival) return a.arrival < b.arrival;
      return a.layer < b.layer;
    });
  }

  for (auto &g : tg) tr->tracks.push_back(g.p);
  // ingress streams: one per received SSRC (video layer / audio), in track order
  std::vector<u32> streamBase(tg.size());
  for (size_t ti = 0; ti < tg.size(); ti++) {
    streamBase[ti] = u32(tr->streams.size());
    for (int l = 0; l < (tg[ti].svc ? 1 : tg[ti].nlayers); l++) {
      lkf_stream_params sp{};
      sp.track = int32_t(ti);
      sp.layer = l;
      sp.ssrc = tg[ti].ssrc[l];
      sp.audio_level_ext = tg[ti].p.kind == LKF_KIND_AUDIO ? 1 : 0;
      sp.dd_ext = tg[ti].dd ? 8 : 0;
      sp.twcc_ext = 5;  // transport-cc (video datagrams carry it; audio ones do not)
      // publishers negotiate NACK feedback for Opus and every video codec
      // (pkg/rtc/config.go:92-101): each Buffer gets a NackQueue; RTTs vary
      // (a quarter keep the queue's default), keyed by the track's SSRC so a
      // room draws the same RTTs in any shard of rooms
      sp.nack = 1;
      const u32 rk = tg[ti].ssrc[0];
      sp.rtt_ms = (rk % 4 == 0) ? 0u : u32(20 + (rk * 37u + u32(l) * 11) % 130);
      tr->streams.push_back(sp);
    }
  }

  // ---- batches ------------------------------------------------------------
  const u32 nb = u32((durNs + batchNs - 1) / batchNs + 1);  // +1: network delay tail
  std::vector<size_t> cursor(tg.size(), 0);
  // per (batch, track) index range for event mapping
  std::vector<std::vector<std::pair<u32, u32>>> trackRange(nb, std::vector<std::pair<u32, u32>>(tg.size()));
  // header size of a raw packet: DD tracks carry the DD element before the
  // transport-cc one (two-byte profile when the DD exceeds 16 bytes)
  auto hdrSize = [](const TrackGen &g, const Plan &pl) -> u32 {
    if (!g.dd) return kPayloadOff;
    const u32 eh = pl.dd.size() > 16 ? 2 : 1;
    const u32 el = eh + u32(pl.dd.size()) + eh + 2;
    return 12 + 4 + ((el + 3) & ~3u);
  };
  u64 totalArena = 0, totalPkts = 0;
  for (auto &g : tg)
    for (auto &pl : g.plans) {
      totalPkts++;
      totalArena += (u64(hdrSize(g, pl)) + pl.payload_len + 15) & ~u64(15);
    }
  // the ingress parser's view of each DD track, in arrival order (persists across batches)
  struct DDTrackView {
    bool hasStructure = false;
    u64 structureFn = 0, activeSeq = 0;
    u32 mask = 0;
    std::vector<std::pair<u64, int>> arrived;  // (extFn, packets seen)
  };
  std::vector<DDTrackView> ddv(tg.size());
  tr->pkts.reserve(totalPkts);
  tr->arena.resize(totalArena);
  u64 aoff = 0;
  tr->batch_pkt_off.push_back(0);
  tr->batch_raw_off.push_back(0);
  tr->batch_arena_off.push_back(0);
  for (u32 b = 0; b < nb; b++) {
    i64 end = (b + 1 == nb) ? INT64_MAX : t0 + i64(b + 1) * batchNs;
    u64 batchA0 = aoff;
    u64 batchP0 = tr->pkts.size();
    for (size_t ti = 0; ti < tg.size(); ti++) {
      TrackGen &g = tg[ti];
      u32 rb = u32(tr->pkts.size() - batchP0);
      while (cursor[ti] < g.plans.size() && g.plans[cursor[ti]].arrival < end) {
        const Plan &pl = g.plans[cursor[ti]++];
        lkf_pkt d{};
        lkf_pkt_dd dd{};
        bool keep = true;  // an ExtPacket is produced for this datagram
        const u32 hsz = hdrSize(g, pl);
        d.ext_sn = pl.ext_sn;
        d.ext_ts = pl.ext_ts;
        d.arrival_ns = pl.arrival;
        d.arena_off = u32(aoff - batchA0);
        d.track = u32(ti);
        d.ssrc = pl.ssrc;
        d.payload_off = u16(hsz);
        d.payload_len = pl.payload_len;
        d.hdr0 = 0x90;  // V=2, X=1, CC=0
        d.hdr1 = u8((pl.marker ? 0x80 : 0) | pl.pt);
        d.layer = pl.layer;
        u8 *raw = tr->arena.data() + aoff;
        raw[0] = d.hdr0;
        raw[1] = d.hdr1;
        raw[2] = u8(pl.ext_sn >> 8);
        raw[3] = u8(pl.ext_sn);
        u32 ts32 = u32(pl.ext_ts);
        raw[4] = u8(ts32 >> 24);
        raw[5] = u8(ts32 >> 16);
        raw[6] = u8(ts32 >> 8);
        raw[7] = u8(ts32);
        raw[8] = u8(pl.ssrc >> 24);
        raw[9] = u8(pl.ssrc >> 16);
        raw[10] = u8(pl.ssrc >> 8);
        raw[11] = u8(pl.ssrc);
        raw[12] = 0xBE;
        raw[13] = 0xDE;
        raw[14] = 0x00;
        raw[15] = 0x01;
        u8 *pay = raw + hsz;
        fill_payload(pay, pl.payload_len, (u64(pl.ssrc) << 32) ^ pl.ext_sn);
        if (g.dd) {
          // extension block: DD (id 8) then transport-cc (id 5)
          const bool two = pl.dd.size() > 16;
          const u32 words = (hsz - 16) / 4;
          raw[12] = two ? 0x10 : 0xBE;
          raw[13] = two ? 0x00 : 0xDE;
          raw[14] = u8(words >> 8);
          raw[15] = u8(words);
          u32 o = 16;
          if (two) {
            raw[o++] = 8;
            raw[o++] = u8(pl.dd.size());
          } else {
            raw[o++] = u8((8 << 4) | (pl.dd.size() - 1));
          }
          dd.dd_off = u16(o);
          dd.dd_len = u8(pl.dd.size());
          for (u8 x : pl.dd) raw[o++] = x;
          if (two) {
            raw[o++] = 5;
            raw[o++] = 2;
          } else {
            raw[o++] = 0x51;
          }
          raw[o++] = u8(pl.twcc >> 8);
          raw[o++] = u8(pl.twcc);
          while (o < hsz) raw[o++] = 0;
          if (g.p.codec == LKF_CODEC_AV1) {
            // AV1 aggregation header; the key superframe's first packet holds a
            // sequence header OBU and a KEY_FRAME OBU_FRAME (IsAV1KeyFrame)
            if (pl.keyframe && pl.payload_len > 16) {
              pay[0] = 0x28;  // Z=0 Y=0 W=2 N=1
              pay[1] = 8;     // OBU_SEQUENCE_HEADER, 8 bytes
              pay[2] = 0x08;
              pay[10] = 0x30;  // OBU_FRAME
              pay[11] = 0x10;  // show_existing_frame 0, KEY_FRAME, show_frame
            } else {
              pay[0] = u8((pl.s_bit ? 0x00 : 0x80) | 0x10);  // Z (continuation) W=1 N=0
            }
          } else {  // VP9 with DD: the VP9 payload descriptor is still there (IsVP9KeyFrame)
            pay[0] = u8((pl.vp9 & (LKF_VP9_I | LKF_VP9_P | LKF_VP9_L | LKF_VP9_F | LKF_VP9_B | LKF_VP9_E | LKF_VP9_V)));
            pay[1] = u8(0x80 | (pl.pid >> 8));
            pay[2] = u8(pl.pid);
            pay[3] = u8((pl.tid << 5) | ((pl.vp9 & LKF_VP9_U) ? 0x10 : 0) | (u8(pl.layer) << 1));
            pay[4] = pl.tl0;
            if (pl.vp9 & LKF_VP9_B) pay[5] = pl.keyframe ? 0x82 : 0x86;
          }
          d.flags = LKF_PKT_DD | (pl.keyframe ? LKF_PKT_KEYFRAME : 0);
          d.spatial = pl.layer;  // VideoLayer from the DD (dependencydescriptorparser.go:101-103)
          d.temporal = int8_t(pl.tid);
          // the ingress parser's metadata, in arrival order (dependencydescriptorparser.go:99-162);
          // a packet the parser rejects produces no ExtPacket (buffer.go:613-616): no
          // structure yet, or a frame older than the current structure's
          DDTrackView &v = ddv[ti];
          if ((!v.hasStructure && !pl.ddAttach) || (v.hasStructure && pl.extFn < v.structureFn)) keep = false;
          dd.ext_frame_num = pl.extFn;
          if (keep && pl.ddAttach) {
            v.hasStructure = true;
            v.structureFn = pl.extFn;
            dd.flags |= LKF_DD_STRUCTURE_UPDATED | LKF_DD_ACTIVE_UPDATED;
          }
          const bool maskPresent = keep && (pl.ddAttach || pl.ddActive);
          const u32 mask = pl.ddActive ? pl.ddMask : 0x1FFu;
          if (maskPresent && pl.ext_sn > v.activeSeq) {
            v.activeSeq = pl.ext_sn;
            if (mask != v.mask) {
              v.mask = mask;
              dd.flags |= LKF_DD_ACTIVE_UPDATED;
            }
          }
          dd.ext_key_frame_num = v.structureFn;
          int seen = 1;
          bool found = !keep;
          for (auto &a : v.arrived) {
            if (found) break;
            if (a.first == pl.extFn) {
              seen = ++a.second;
              found = true;
            }
          }
          if (!found) {
            v.arrived.push_back({pl.extFn, 1});
            if (v.arrived.size() > 256) v.arrived.erase(v.arrived.begin());
          }
          if (seen == pl.framePkts) dd.flags |= LKF_DD_INTEGRITY;
        } else if (g.p.kind == LKF_KIND_VIDEO && g.svc) {
          raw[16] = 0x51;  // id 5 (transport-cc), len 2
          raw[17] = u8(pl.twcc >> 8);
          raw[18] = u8(pl.twcc);
          raw[19] = 0;
          // VP9 payload descriptor (non-flexible mode): I|P|L|F|B|E|V|Z,
          // M|PID(15), TID|U|SID|D, TL0PICIDX; then on B packets the first
          // byte of the VP9 uncompressed header (frame marker 10, profile 0,
          // show_existing 0, frame_type 0 = key / 1 = inter, show_frame 1)
          pay[0] = u8((pl.vp9 & (LKF_VP9_I | LKF_VP9_P | LKF_VP9_L | LKF_VP9_F | LKF_VP9_B | LKF_VP9_E | LKF_VP9_V)));
          pay[1] = u8(0x80 | (pl.pid >> 8));
          pay[2] = u8(pl.pid);
          pay[3] = u8((pl.tid << 5) | ((pl.vp9 & LKF_VP9_U) ? 0x10 : 0) | (u8(pl.layer) << 1));
          pay[4] = pl.tl0;
          if (pl.vp9 & LKF_VP9_B) pay[5] = pl.keyframe ? 0x82 : 0x86;
          d.flags = LKF_PKT_VP9 | (pl.keyframe ? LKF_PKT_KEYFRAME : 0);
          d.vp9_bits = pl.vp9;
          d.spatial = pl.layer;  // VideoLayer{SID, TID} (buffer.go:645-655)
          d.temporal = int8_t(pl.tid);
        } else if (g.p.kind == LKF_KIND_VIDEO && g.p.codec == LKF_CODEC_H264) {
          raw[16] = 0x51;  // id 5 (transport-cc), len 2
          raw[17] = u8(pl.twcc >> 8);
          raw[18] = u8(pl.twcc);
          raw[19] = 0;
          // RFC 6184 packetization; a key frame's first packet carries the SPS
          // (IsH264KeyFrame), in one of the four aggregation forms by picture id
          const u32 n = pl.payload_len;
          bool sps = false;
          if (pl.keyframe && pl.s_bit) {
            const u32 form = n >= 16 ? pl.pid % 4 : 0;
            if (form == 0) {
              pay[0] = 0x67;  // single NALU, type 7
            } else if (form == 1) {
              pay[0] = 0x78;  // STAP-A: [len 10][SPS ...][len ...][PPS ...]
              pay[1] = 0;
              pay[2] = 10;
              pay[3] = 0x67;
              pay[13] = 0;
              pay[14] = u8(n - 15);
              pay[15] = 0x68;
            } else if (form == 2) {
              pay[0] = 0x7C;  // FU-A start fragment of an SPS
              pay[1] = 0x87;
            } else {
              pay[0] = 0x79;  // STAP-B: DON, then [len 4][AUD][len ..][SPS]
              pay[1] = 0;
              pay[2] = 1;
              pay[3] = 0;
              pay[4] = 4;
              pay[5] = 0x09;
              pay[9] = 0;
              pay[10] = u8(n - 11);
              pay[11] = 0x67;
            }
            sps = true;
          } else if (pl.s_bit) {
            if (pl.pid % 7 == 3 && n >= 4) {
              pay[0] = 0x78;  // truncated STAP-A (length beyond the payload)
              pay[1] = 0xFF;
              pay[2] = 0xFF;
            } else if (pl.pid % 2) {
              pay[0] = 0x41;  // single NALU, non-IDR slice
            } else {
              pay[0] = 0x7C;  // FU-A start, non-IDR slice
              pay[1] = 0x81;
            }
          } else {
            pay[0] = 0x7C;  // FU-A continuation
            pay[1] = pl.keyframe ? 0x05 : 0x01;
          }
          d.flags = sps ? LKF_PKT_KEYFRAME : 0;
          d.spatial = -1;
          d.temporal = 0;  // buffer.go:616: no temporal layers without a descriptor
        } else if (g.p.kind == LKF_KIND_VIDEO) {
          raw[16] = 0x51;  // id 5 (transport-cc), len 2
          raw[17] = u8(pl.twcc >> 8);
          raw[18] = u8(pl.twcc);
          raw[19] = 0;
          // VP8 payload descriptor (RFC 7741): X|S, I|L|T, M|PID(15), TL0, TID|Y
          pay[0] = u8(0x80 | (pl.s_bit ? 0x10 : 0));
          pay[1] = 0xE0;
          pay[2] = u8(0x80 | (pl.pid >> 8));
          pay[3] = u8(pl.pid);
          pay[4] = pl.tl0;
          pay[5] = u8((pl.tid << 6) | (pl.y_bit ? 0x20 : 0));
          pay[6] = u8((pay[6] & 0xFE) | (pl.keyframe ? 0 : 1));  // VP8 P bit
          d.flags = LKF_PKT_VP8 | (pl.keyframe ? LKF_PKT_KEYFRAME : 0);
          d.vp8_first = pay[0];
          d.vp8_bits = u8((pl.s_bit ? LKF_VP8_S : 0) | LKF_VP8_I | LKF_VP8_M | LKF_VP8_L | LKF_VP8_T |
                          (pl.y_bit ? LKF_VP8_Y : 0));
          d.vp8_hdr_size = 6;
          d.vp8_picture_id = pl.pid;
          d.vp8_tl0picidx = pl.tl0;
          d.vp8_tid = pl.tid;
          d.vp8_keyidx = 0;
          d.spatial = -1;  // VP8 without DD: buffer.go:605-636
          d.temporal = int8_t(pl.tid);
        } else {
          raw[16] = 0x10;  // id 1 (ssrc-audio-level), len 1
          raw[17] = u8(0x80 | pl.level);
          raw[18] = 0;
          raw[19] = 0;
          d.flags = LKF_PKT_HAS_LEVEL;
          d.audio_level = pl.level;
          d.spatial = -1;
          d.temporal = 0;  // buffer.go:616
        }
        lkf_raw_pkt rp{};
        rp.arrival_ns = pl.arrival;
        rp.stream = streamBase[ti] + u32((g.nlayers == 1 || g.svc) ? 0 : pl.layer);
        rp.off = d.arena_off;
        rp.len = hsz + pl.payload_len;
        tr->raws.push_back(rp);
        aoff += (u64(hsz) + pl.payload_len + 15) & ~u64(15);
        if (keep) {
          tr->pkts.push_back(d);
          tr->dds.push_back(dd);
        }
      }
      trackRange[b][ti] = {rb, u32(tr->pkts.size() - batchP0)};
    }
    tr->batch_pkt_off.push_back(tr->pkts.size());
    tr->batch_raw_off.push_back(tr->raws.size());
    tr->batch_arena_off.push_back(aoff);
    tr->max_batch_pkts = std::max(tr->max_batch_pkts, u32(tr->raws.size() - tr->batch_raw_off[b]));
    tr->max_batch_arena = std::max(tr->max_batch_arena, aoff - batchA0);
  }

  {
    std::vector<u64> dtsPerTrack(tg.size(), 0);
    for (auto &d : tr->dts) dtsPerTrack[d.track]++;
    for (u32 b = 0; b < nb; b++) {
      u64 tup = 0, ob = 0;
      const lkf_pkt *bp = tr->pkts.data() + tr->batch_pkt_off[b];
      for (size_t ti = 0; ti < tg.size(); ti++) {
        tup += u64(trackRange[b][ti].second - trackRange[b][ti].first) * dtsPerTrack[ti];
        u64 tb = 0;  // wire packet <= payload + 12-B header + 12-B extension block + 1 (descriptor growth), 16-B aligned
        const u64 extra = tg[ti].dd ? 25 + 2 + 255 : 25;  // + a DD element up to 255 bytes
        for (u32 i = trackRange[b][ti].first; i < trackRange[b][ti].second; i++)
          tb += (u64(bp[i].payload_len) + extra + 15) & ~u64(15);
        ob += tb * dtsPerTrack[ti];
      }
      tr->max_batch_tuples = std::max(tr->max_batch_tuples, tup);
      tr->max_batch_out_bytes = std::max(tr->max_batch_out_bytes, ob);
    }
  }
  // ---- events -> (batch, at_pkt) -------------------------------------
  std::vector<std::vector<lkfs_event>> bev(nb);
  std::stable_sort(evs.begin(), evs.end(), [](const Ev &a, const Ev &b) { return a.t < b.t; });
  for (auto &e : evs) {
    lkfs_event o{};
    o.dt = e.dt;
    o.op = e.op;
    for (int i = 0; i < 4; i++) o.a[i] = e.a[i];
    if (e.t < 0) {
      o.at_pkt = 0;
      bev[0].push_back(o);
      continue;
    }
    u32 b = u32(std::min<i64>(i64(nb) - 1, (e.t - t0) / batchNs));
    int track = tr->dts[e.dt].track;
    auto rg = trackRange[b][track];
    const lkf_pkt *bp = tr->pkts.data() + tr->batch_pkt_off[b];
    u32 at = rg.second;
    for (u32 i = rg.first; i < rg.second; i++)
      if (bp[i].arrival_ns >= e.t) {
        at = i;
        break;
      }
    o.at_pkt = at;
    bev[b].push_back(o);
  }
  tr->batch_ev_off.push_back(0);
  for (u32 b = 0; b < nb; b++) {
    tr->events.insert(tr->events.end(), bev[b].begin(), bev[b].end());
    tr->batch_ev_off.push_back(tr->events.size());
  }
  return tr;
}

extern "C" void lkfs_free(lkfs_trace *t) { delete t; }
extern "C" uint32_t lkfs_num_tracks(const lkfs_trace *t) { return u32(t->tracks.size()); }
extern "C" uint32_t lkfs_num_downtracks(const lkfs_trace *t) { return u32(t->dts.size()); }
extern "C" const lkf_track_params *lkfs_tracks(const lkfs_trace *t) { return t->tracks.data(); }
extern "C" const lkf_downtrack_params *lkfs_downtracks(const lkfs_trace *t) { return t->dts.data(); }
extern "C" uint32_t lkfs_num_batches(const lkfs_trace *t) { return u32(t->batch_pkt_off.size() - 1); }
extern "C" int lkfs_batch(const lkfs_trace *t, uint32_t b, const lkf_pkt **pkts, uint32_t *n, const uint8_t **arena,
                          uint64_t *arena_len) {
  if (b + 1 >= t->batch_pkt_off.size()) return LKF_EINVAL;
  *pkts = t->pkts.data() + t->batch_pkt_off[b];
  *n = u32(t->batch_pkt_off[b + 1] - t->batch_pkt_off[b]);
  *arena = t->arena.data() + t->batch_arena_off[b];
  *arena_len = t->batch_arena_off[b + 1] - t->batch_arena_off[b];
  return LKF_OK;
}

extern "C" int lkfs_batch_dd(const lkfs_trace *t, uint32_t b, const lkf_pkt_dd **dd, uint32_t *n) {
  if (b + 1 >= t->batch_pkt_off.size()) return LKF_EINVAL;
  *dd = t->dds.data() + t->batch_pkt_off[b];
  *n = u32(t->batch_pkt_off[b + 1] - t->batch_pkt_off[b]);
  return LKF_OK;
}
extern "C" uint32_t lkfs_num_streams(const lkfs_trace *t) { return u32(t->streams.size()); }
extern "C" const lkf_stream_params *lkfs_streams(const lkfs_trace *t) { return t->streams.data(); }
extern "C" int lkfs_batch_raw(const lkfs_trace *t, uint32_t b, const lkf_raw_pkt **raws, uint32_t *n) {
  if (b + 1 >= t->batch_pkt_off.size()) return -1;
  *raws = t->raws.data() + t->batch_raw_off[b];
  *n = u32(t->batch_raw_off[b + 1] - t->batch_raw_off[b]);
  return 0;
}
extern "C" int lkfs_batch_events(const lkfs_trace *t, uint32_t b, const lkfs_event **ev, uint32_t *n) {
  if (b + 1 >= t->batch_ev_off.size()) return LKF_EINVAL;
  *ev = t->events.data() + t->batch_ev_off[b];
  *n = u32(t->batch_ev_off[b + 1] - t->batch_ev_off[b]);
  return LKF_OK;
}
extern "C" uint64_t lkfs_total_pkts(const lkfs_trace *t) { return t->pkts.size(); }
extern "C" uint64_t lkfs_total_arena(const lkfs_trace *t) { return t->arena.size(); }
extern "C" uint32_t lkfs_max_batch_pkts(const lkfs_trace *t) { return t->max_batch_pkts; }
extern "C" uint64_t lkfs_max_batch_arena(const lkfs_trace *t) { return t->max_batch_arena; }
extern "C" uint64_t lkfs_max_batch_tuples(const lkfs_trace *t) { return t->max_batch_tuples; }
extern "C" uint64_t lkfs_max_batch_out_bytes(const lkfs_trace *t) { return t->max_batch_out_bytes; }
