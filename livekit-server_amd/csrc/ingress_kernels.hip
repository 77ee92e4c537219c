// ingress_kernels.hip — gfx950 kernels of the ingress path (Buffer.calc) and
// the active-speaker ranking.
//
// Per raw batch (lkf_ingest):
//   k_ing_parse    thread per datagram: rtp.Packet.Unmarshal (pion/rtp
//                  v1.8.3, restated), the ssrc-audio-level extension
//                  (RFC 6464) and the VP8 payload descriptor
//                  (buffer/helpers.go:76-162); datagrams grouped by track
//                  -> [begin, end) per track
//   k_ing_stream_wave  one wave per received stream (buffer.Buffer), its
//                  datagrams in order: processHeaderExtensions ->
//                  AudioLevel.Observe (buffer.go:573-596, audiolevel.go:70-102),
//                  RTPStatsReceiver.Update (rtpstats_receiver.go:76-241) with
//                  its WrapArounds and 4096-bit history, NACK loss ranges
//                  (buffer.go:545-567), padding exclusion + SN adjustment
//                  (buffer.go:439-471), the RTX bucket's
//                  AddPacketWithSequenceNumber (:471-481), getExtPacket's
//                  dependency descriptor (:599-671); in-order runs lane-parallel
//   k_ing_nack     (side stream) the NackQueue per stream
//   scan           positions of the ExtPackets produced
//   k_ing_out      thread per datagram: the ExtPacket (getExtPacket
//                  buffer.go:599-671) as an lkf_pkt of the forwarding batch
// Speakers (lkf_speakers):
//   k_speakers     one wave per room, lane per participant: loudest active
//                  microphone (AudioLevel.GetLevel audiolevel.go:105-112,
//                  uptrackmanager.go:422-436), rank, quantise (room.go:254-279)
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <hip/hip_runtime.h>

#include "../../include/lkfwd.h"
#include "dd_device.h"
#include "fwd_state.h"
#include "kernels.h"

namespace lkf {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i16 = int16_t;
using i32 = int32_t;
using i64 = int64_t;

// ---------------------------------------------------------------------------
// k_ing_parse
// ---------------------------------------------------------------------------
// A datagram's bytes for the parsers: the first n staged in LDS, the rest read
// from HBM (the parsers walk the header, extensions and codec descriptor byte
// by byte; from LDS those dependent reads cost LDS latency, not HBM latency).
typedef const __attribute__((address_space(3))) u8 *LdsBytes;  // (ds_read, not a flat load)
struct StagedBytes {
  LdsBytes lds;
  const u8 *g;
  int n;
  __device__ __forceinline__ u8 operator[](int i) const {
    u8 v;
    if (i < n)
      v = lds[i];
    else
      v = g[i];
    return v;
  }
  __device__ __forceinline__ StagedBytes operator+(int k) const { return StagedBytes{lds + k, g + k, n - k}; }
};

template <typename BP>
__device__ __forceinline__ bool rtp_parse(BP buf, int len, u8 levelExt, u8 ddExt, IngParsed &q,
                                          int &levelOff, u8 twccExt = 0, int *twccOff = nullptr,
                                          int *twccLen = nullptr) {
  levelOff = -1;
  if (len < 12) return false;
  q.b0 = buf[0];
  q.b1 = buf[1];
  const bool padding = (buf[0] >> 5) & 1, extension = (buf[0] >> 4) & 1;
  const int cc = buf[0] & 0xf;
  int n = 12 + 4 * cc;
  if (len < n) return false;
  q.sn = u16((u32(buf[2]) << 8) | buf[3]);
  q.ts = (u32(buf[4]) << 24) | (u32(buf[5]) << 16) | (u32(buf[6]) << 8) | buf[7];
  q.ssrc = (u32(buf[8]) << 24) | (u32(buf[9]) << 16) | (u32(buf[10]) << 8) | buf[11];
  if (extension) {
    if (len < n + 4) return false;
    const u32 profile = (u32(buf[n]) << 8) | buf[n + 1];
    n += 2;
    const int extLen = int((u32(buf[n]) << 8) | buf[n + 1]) * 4;
    n += 2;
    const int extEnd = n + extLen;
    if (len < extEnd) return false;
    if (profile == 0xBEDE || profile == 0x1000) {
      bool seen = false, seenDD = false, seenTw = false;  // Header.GetExtension: the first element with the id
      while (n < extEnd) {
        if (buf[n] == 0x00) {
          n++;
          continue;
        }
        u8 id;
        int pl;
        if (profile == 0xBEDE) {
          id = buf[n] >> 4;
          pl = (buf[n] & 0x0f) + 1;
          n++;
          if (id == 15) break;
        } else {
          id = buf[n];
          n++;
          if (len <= n) return false;
          pl = buf[n];
          n++;
        }
        if (len <= n + pl) return false;
        if (levelExt && id == levelExt && !seen) {
          seen = true;
          if (pl >= 1) levelOff = n;  // AudioLevelExtension.Unmarshal needs 1 byte
        }
        if (ddExt && id == ddExt && !seenDD) {
          seenDD = true;
          q.ddOff = u16(n);
          q.ddLen = u8(pl);
        }
        if (twccExt && id == twccExt && !seenTw) {
          seenTw = true;
          *twccOff = n;
          *twccLen = pl;
        }
        n += pl;
      }
    } else {  // RFC 3550 extension: a single element with id 0 (never the level id)
      n = extEnd;
    }
  }
  int end = len;
  int padSize = 0;
  if (padding) {
    if (end <= n) return false;
    padSize = buf[end - 1];
    end -= padSize;
  }
  if (end < n) return false;
  q.hdrSize = u16(n);
  q.payloadLen = u16(end - n);
  q.paddingSize = u8(padSize);
  if (buf[1] & 0x80) q.flags |= IP_MARKER;
  return true;
}

// buffer.VP8.Unmarshal helpers.go:76-162
template <typename BP>
__device__ __forceinline__ bool vp8_parse(BP p, int len, IngParsed &q) {
  if (len < 1) return false;
  int idx = 0;
  q.vfirst = p[0];
  const bool S = (p[0] & 0x10) != 0;
  bool I = false, L = false, T = false, K = false, M = false, Y = false;
  u16 pid = 0;
  u8 tl0 = 0, tid = 0, keyidx = 0;
  bool kf;
  if (p[0] & 0x80) {
    idx++;
    if (len < idx + 1) return false;
    I = (p[idx] & 0x80) != 0;
    L = (p[idx] & 0x40) != 0;
    T = (p[idx] & 0x20) != 0;
    K = (p[idx] & 0x10) != 0;
    if (L && !T) return false;
    if (I) {
      idx++;
      if (len < idx + 1) return false;
      const u8 lo7 = p[idx] & 0x7f;
      M = (p[idx] & 0x80) != 0;
      if (M) {
        idx++;
        if (len < idx + 1) return false;
        pid = u16((u16(lo7) << 8) | p[idx]);
      } else {
        pid = lo7;
      }
    }
    if (L) {
      idx++;
      if (len < idx + 1) return false;
      tl0 = p[idx];
    }
    if (T || K) {
      idx++;
      if (len < idx + 1) return false;
      if (T) {
        tid = (p[idx] & 0xc0) >> 6;
        Y = (p[idx] & 0x20) != 0;
      }
      if (K) keyidx = p[idx] & 0x1f;
    }
    idx++;
    if (len < idx + 1) return false;
    kf = (p[idx] & 0x01) == 0 && S;
  } else {
    idx++;
    if (len < idx + 1) return false;
    kf = (p[idx] & 0x01) == 0 && S;
  }
  q.vbits = u8((S ? LKF_VP8_S : 0) | (I ? LKF_VP8_I : 0) | (M ? LKF_VP8_M : 0) | (L ? LKF_VP8_L : 0) |
               (T ? LKF_VP8_T : 0) | (Y ? LKF_VP8_Y : 0) | (K ? LKF_VP8_K : 0));
  q.vhs = u8(idx);
  q.pid = pid;
  q.tl0 = tl0;
  q.tid = tid;
  q.keyidx = keyidx;
  if (kf) q.flags |= IP_KF;
  return true;
}

// buffer.IsH264KeyFrame helpers.go:248-309
template <typename BP>
__device__ inline bool h264_keyframe(BP p, int n) {
  if (n < 1) return false;
  const int nalu = p[0] & 0x1F;
  if (nalu == 0) return false;
  if (nalu <= 23) return nalu == 7;
  if (nalu >= 24 && nalu <= 27) {  // STAP-A/B, MTAP16/24
    int i = 1;
    if (nalu != 24) i += 2;  // DON
    while (i < n) {
      if (i + 2 > n) return false;
      const int length = (int(p[i]) << 8) | int(p[i + 1]);
      i += 2;
      if (i + length > n) return false;
      const int offset = nalu == 26 ? 3 : nalu == 27 ? 4 : 0;
      if (offset >= length) return false;
      if ((p[i + offset] & 0x1F) == 7) return true;
      i += length;
    }
    return false;
  }
  if (nalu == 28 || nalu == 29) {  // FU-A/B: starting fragment of an SPS
    if (n < 2) return false;
    if ((p[1] & 0x80) == 0) return false;
    return (p[1] & 0x1F) == 7;
  }
  return false;
}

// buffer.IsAV1KeyFrame helpers.go:343-420: walk the aggregation's OBUs (W
// field: the last one carries no length) to the first frame header
template <typename BP>
__device__ inline bool av1_keyframe(BP payload, int n) {
  if (n < 2) return false;
  if ((payload[0] & 0x88) != 0x08) return false;  // Z=0, N=1
  const int w = (payload[0] & 0x30) >> 4;
  int offset = 1;
  for (int i = 0;; i++) {
    const BP data = payload + offset;
    const int dn = n - offset;
    BP obu = data;
    int olen, length;
    bool truncated = false;
    if (w == i + 1) {
      obu = data;
      olen = dn;
      length = dn;
    } else {
      int off = 0, len = 0;
      bool done = false;
      for (;;) {
        if (dn <= off) {
          done = true;
          break;
        }
        const u8 l = data[off];
        len |= int(l & 0x7f) << (off * 7);
        off++;
        if ((l & 0x80) == 0) break;
      }
      if (done) return false;  // no OBU
      if (dn < off + len) {
        obu = data + off;
        olen = dn - off;
        length = dn;
        truncated = true;
      } else {
        obu = data + off;
        olen = len;
        length = off + len;
      }
    }
    if (olen < 1) return false;
    const int tpe = (obu[0] & 0x38) >> 3;
    if (i == 0) {
      if (tpe != 1) return false;  // OBU_SEQUENCE_HEADER
    } else if (tpe == 3 || tpe == 6) {
      if (olen < 2) return false;
      if ((obu[1] & 0x80) != 0) return false;  // show_existing_frame
      return (obu[1] & 0x60) == 0;             // KEY_FRAME
    }
    if (truncated || i >= w) return false;
    offset += length;
  }
}

// codecs.VP9Packet.Unmarshal (pion/rtp v1.8.3 codecs/vp9_packet.go; not in
// the reference tree: restated from the published descriptor layout, parity
// unpinned) + buffer.IsVP9KeyFrame helpers.go:317-336.  Layer info, flexible
// mode reference indices and scalability-structure data are walked for their
// lengths; the selector reads I/P/L/F/B/E/V, TID/U/SID.
template <typename BP>
__device__ __forceinline__ bool vp9_parse(BP p, int len, IngParsed &q) {
  if (len < 1) return false;
  const u8 b0 = p[0];
  const bool I = b0 & 0x80, P = b0 & 0x40, L = b0 & 0x20, F = b0 & 0x10, V = b0 & 0x02;
  int pos = 1;
  u8 tid = 0, sid = 0;
  bool U = false;
  if (I) {  // parsePictureID
    if (len <= pos) return false;
    if (p[pos] & 0x80) {
      pos++;
      if (len <= pos) return false;
    }
    pos++;
  }
  if (L) {  // parseLayerInfo
    if (len <= pos) return false;
    tid = p[pos] >> 5;
    U = (p[pos] & 0x10) != 0;
    sid = (p[pos] >> 1) & 0x7;
    if (sid >= 5) return false;  // errTooManySpatialLayers (maxSpatialLayers 5)
    pos++;
    if (!F) {  // non-flexible mode: TL0PICIDX
      if (len <= pos) return false;
      pos++;
    }
  }
  if (F && P) {  // parseRefIndices (maxVP9RefPics 3)
    int nref = 0;
    for (;;) {
      if (len <= pos) return false;
      nref++;
      if ((p[pos] & 0x01) == 0) break;
      if (nref >= 3) return false;
      pos++;
    }
    pos++;
  }
  if (V) {  // parseSSData
    if (len <= pos) return false;
    const int ns = (p[pos] >> 5) + 1;
    const bool Y = p[pos] & 0x10, G = p[pos] & 0x08;
    pos++;
    if (Y) {
      if (len <= pos + ns * 4 - 1) return false;
      pos += ns * 4;
    }
    int ng = 0;
    if (G) {
      if (len <= pos) return false;
      ng = p[pos];
      pos++;
    }
    for (int i = 0; i < ng; i++) {
      if (len <= pos) return false;
      const int r = (p[pos] >> 2) & 0x3;
      pos++;
      if (len <= pos + r - 1) return false;
      pos += r;
    }
  }
  q.vp9bits = u8((b0 & (LKF_VP9_I | LKF_VP9_P | LKF_VP9_L | LKF_VP9_F | LKF_VP9_B | LKF_VP9_E | LKF_VP9_V)) |
                 (U ? LKF_VP9_U : 0));
  q.sid = sid;
  q.tid = tid;
  // IsVP9KeyFrame: B, frame marker 10, profile -> show_existing_frame / frame_type
  bool kf = false;
  if ((b0 & 0x08) && len > pos) {
    const u8 h = p[pos];
    if ((h & 0xc0) == 0x80) {
      const u8 profile = (h >> 4) & 0x3;
      kf = profile != 3 ? (h & 0xC) == 0 : (h & 0x6) == 0;
    }
  }
  if (kf) q.flags |= IP_KF;
  return true;
}

constexpr int kParseT = 64;       // k_ing_parse block (8 KB of LDS: fits beside the decide waves)
constexpr int kParseStage = 128;  // bytes of each datagram staged in LDS
constexpr int kStageW = kParseStage / 4 + 1;  // dwords per thread: a dword-aligned window (odd stride: no bank conflicts)
// (with the per-track datagram ranges: a datagram's track is its stream's,
// so the boundaries need no parse — k_ing_ranges' work, one dispatch fewer
// on the ingest chain)
__device__ __forceinline__ u32 raw_track(const lkf_raw_pkt *raws, const DevStream *streams, u32 nstreams, u32 i) {
  const u32 sid = raws[i].stream;
  return sid < nstreams ? streams[sid].track : 0xffffffffu;
}
__global__ void __launch_bounds__(kParseT) k_ing_parse(const lkf_raw_pkt *__restrict__ raws, u32 n,
                                                      const u8 *__restrict__ raw, const DevStream *__restrict__ streams,
                                                      u32 nstreams, IngParsed *__restrict__ out, u32 *__restrict__ twcc,
                                                      u32 *__restrict__ err, u32 ntracks, u32 *__restrict__ tBegin,
                                                      u32 *__restrict__ tEnd, u32 *__restrict__ tRuns) {
  __shared__ u32 sStage[kParseT * kStageW];
  const u32 lane = threadIdx.x;
  const u32 i = blockIdx.x * blockDim.x + lane;
  lkf_raw_pkt rp = {};
  if (i < n) rp = raws[i];
  // the block's datagrams' first bytes into LDS, one datagram per load
  // instruction (lane k loads dword k of its dword-aligned window: one or two
  // cache lines per instruction, where a thread-per-datagram load touched 64),
  // 16 datagrams' loads in flight.  Global loads need only dword alignment; a
  // dword holding a byte of the datagram lies in that byte's page.
  const int sl = int(rp.len) < kParseStage ? int(rp.len) : kParseStage;
  {
    const u32 wbase = rp.off & ~3u;
    const u32 nw = (u32(sl) + (rp.off & 3) + 3) >> 2;  // 0 for a lane past the batch
#pragma unroll
    for (int j0 = 0; j0 < kParseT; j0 += 16) {
      u32 w[16];
#pragma unroll
      for (int jj = 0; jj < 16; jj++) {
        const u32 b = __builtin_amdgcn_readlane(wbase, j0 + jj);
        const u32 c = __builtin_amdgcn_readlane(nw, j0 + jj);
        w[jj] = lane < c ? reinterpret_cast<const u32 *>(raw + b)[lane] : 0u;
      }
#pragma unroll
      for (int jj = 0; jj < 16; jj++)
        if (lane < u32(kStageW)) sStage[(j0 + jj) * kStageW + lane] = w[jj];
    }
  }
  __syncthreads();
  if (i >= n) return;
  {  // per-track ranges (k_ing_init zeroed them)
    const u32 t = raw_track(raws, streams, nstreams, i);
    if (t < ntracks) {
      const u32 tp = i > 0 ? raw_track(raws, streams, nstreams, i - 1) : 0xffffffffu;
      const u32 tn = i + 1 < n ? raw_track(raws, streams, nstreams, i + 1) : 0xffffffffu;
      if (tp != t) {
        tBegin[t] = i;
        if (atomicAdd(&tRuns[t], 1u) != 0) atomicOr(err, 2u);
      }
      if (tn != t) tEnd[t] = i + 1;
    } else {
      atomicOr(err, 1u);
    }
  }
  u32 *const st = sStage + lane * kStageW;
  IngParsed q = {};
  twcc[i] = 0;
  if (rp.stream >= nstreams) {
    atomicOr(err, 1u);
    q.track = 0xffffffffu;
    out[i] = q;
    return;
  }
  const DevStream s = streams[rp.stream];
  q.track = s.track;
  // (each thread reads its own datagram's staged window)
  const StagedBytes b{(LdsBytes)(reinterpret_cast<const u8 *>(st)) + (rp.off & 3), raw + rp.off, sl};
  int levelOff = -1, twOff = -1, twLen = 0;
  if (rtp_parse(b, int(rp.len), s.levelExt, s.ddExt, q, levelOff, s.twccExt, &twOff, &twLen)) {
    q.flags |= IP_OK;
    // processHeaderExtensions (buffer.go:569-576): the TWCC responder sees every
    // datagram that unmarshals (a closed Buffer takes none: Write returns first)
    if (twOff >= 0 && twLen >= 2 && !s.closed)
      twcc[i] = LKF_TWCC_PUSH | ((b[1] & 0x80) ? LKF_TWCC_MARKER : 0u) | (u32(b[twOff]) << 8) | b[twOff + 1];
    if (levelOff >= 0) {  // AudioLevelExtension.Unmarshal: level = b & 0x7f
      q.flags |= IP_LEVEL;
      q.level = b[levelOff] & 0x7f;
    }
    if (s.codec == LKF_CODEC_VP8 && q.payloadLen > 0) {
      if (vp8_parse(b + q.hdrSize, q.payloadLen, q))
        q.flags |= IP_VP8;
      else
        q.flags |= IP_VP8_BAD;
    } else if (s.codec == LKF_CODEC_VP9 && q.payloadLen > 0) {  // getExtPacket buffer.go:643-656
      if (vp9_parse(b + q.hdrSize, q.payloadLen, q))
        q.flags |= IP_VP9;
      else
        q.flags |= IP_VP8_BAD;
    } else if (s.codec == LKF_CODEC_H264 && q.payloadLen > 0) {  // buffer.go:657-658
      if (h264_keyframe(b + q.hdrSize, q.payloadLen)) q.flags |= IP_KF;
    } else if (s.codec == LKF_CODEC_AV1 && q.payloadLen > 0) {  // buffer.go:659-660
      if (av1_keyframe(b + q.hdrSize, q.payloadLen)) q.flags |= IP_KF;
    }
  }
  out[i] = q;
}

// ---------------------------------------------------------------------------
// k_ing_stream helpers: WrapAround (wraparound.go:68-180, restart disallowed),
// protocol utils.Bitmap (4096 bits), utils.RangeMap(100), AudioLevel.
// ---------------------------------------------------------------------------
struct WAResult {
  bool unhandled;
  u64 preHighest, extVal;
};

// WrapAround<uint16,uint64>{IsRestartAllowed: false}.Update
__device__ __forceinline__ WAResult wa16_update(StreamHot &h, u16 val) {
  WAResult r = {false, 0, 0};
  const u64 full = 1ull << 16;
  if (!(h.flags & S_SN_INIT)) {
    r.preHighest = u64(val) - 1;
    r.extVal = u64(val);
    h.snStart = val;
    h.snHighest = val;
    h.snExtHighest = h.snCycles + u64(val);
    h.flags |= S_SN_INIT;
    return r;
  }
  const u16 gap = u16(val - h.snHighest);
  if (gap > u16(full >> 1)) {  // maybeAdjustStart
    u64 cyc = h.snCycles;
    const u64 total = h.snExtHighest - u64(h.snStart) + 1;
    const bool wrapBack = u64(h.snHighest) < (full >> 1) && u64(val) >= (full >> 1);
    if (total > (full >> 1)) {
      if (wrapBack) cyc -= full;
      r.preHighest = h.snExtHighest;
      r.extVal = cyc + u64(val);
      return r;
    }
    if (u16(val - h.snStart) > u16(full >> 1)) {
      r.unhandled = true;  // restart not allowed
    } else if (wrapBack) {
      cyc -= full;
    }
    r.preHighest = h.snExtHighest;
    r.extVal = cyc + u64(val);
    return r;
  }
  r.preHighest = h.snExtHighest;
  if (val < h.snHighest) h.snCycles += full;
  h.snHighest = val;
  h.snExtHighest = h.snCycles + u64(val);
  r.extVal = h.snExtHighest;
  return r;
}

// WrapAround<uint32,uint64>{IsRestartAllowed: false}.Update
__device__ __forceinline__ WAResult wa32_update(StreamHot &h, u32 val) {
  WAResult r = {false, 0, 0};
  const u64 full = 1ull << 32;
  if (!(h.flags & S_TS_INIT)) {
    r.preHighest = u64(val) - 1;
    r.extVal = u64(val);
    h.tsStart = val;
    h.tsHighest = val;
    h.tsExtHighest = h.tsCycles + u64(val);
    h.flags |= S_TS_INIT;
    return r;
  }
  const u32 gap = val - h.tsHighest;
  if (gap > u32(full >> 1)) {
    u64 cyc = h.tsCycles;
    const u64 total = h.tsExtHighest - u64(h.tsStart) + 1;
    const bool wrapBack = u64(h.tsHighest) < (full >> 1) && u64(val) >= (full >> 1);
    if (total > (full >> 1)) {
      if (wrapBack) cyc -= full;
      r.preHighest = h.tsExtHighest;
      r.extVal = cyc + u64(val);
      return r;
    }
    if (u32(val - h.tsStart) > u32(full >> 1)) {
      r.unhandled = true;
    } else if (wrapBack) {
      cyc -= full;
    }
    r.preHighest = h.tsExtHighest;
    r.extVal = cyc + u64(val);
    return r;
  }
  r.preHighest = h.tsExtHighest;
  if (val < h.tsHighest) h.tsCycles += full;
  h.tsHighest = val;
  h.tsExtHighest = h.tsCycles + u64(val);
  r.extVal = h.tsExtHighest;
  return r;
}

// RTPStatsReceiver history (cHistorySize 4096 bits, rtpstats_receiver.go:30),
// staged in LDS for the ingest (HS: the word stride of the staged copy)
template <int HS = 1>
__device__ __forceinline__ bool hist_isset(const u64 *h, u64 v) {
  return (h[((v >> 6) & (kHistWords - 1)) * HS] >> (v & 63)) & 1;
}
template <int HS = 1>
__device__ __forceinline__ void hist_set(u64 *h, u64 v) { h[((v >> 6) & (kHistWords - 1)) * HS] |= 1ull << (v & 63); }
template <int HS = 1>
__device__ void hist_clear_range(u64 *h, u64 lo, u64 hi) {  // inclusive; lo > hi: no-op
  if (lo > hi) return;
  if (hi - lo + 1 >= u64(kHistWords) * 64) {
    for (int w = 0; w < kHistWords; w++) h[w * HS] = 0;
    return;
  }
  for (u64 v = lo;;) {  // a word at a time
    const u32 b = u32(v & 63);
    const u64 nb = min(u64(64 - b), hi - v + 1);
    const u64 m = (nb == 64 ? ~0ull : ((1ull << nb) - 1)) << b;
    h[((v >> 6) & (kHistWords - 1)) * HS] &= ~m;
    if (hi - v + 1 == nb) break;
    v += nb;
  }
}

// utils.RangeMap[uint64,uint64](100): ExcludeRange (rangemap.go:100-132)
__device__ __forceinline__ bool irm_exclude(StreamHot &h, RangeEntry *ring, u64 s, u64 e) {
  if (e == s || (e - s) > (1ull << 63)) return false;
  if (h.rmOpenStart > s) return false;
  const u64 nv = h.rmOpenValue + (e - s);
  if (h.rmOpenStart == s) {
    h.rmOpenStart = e;
    h.rmOpenValue = nv;
    return true;
  }
  RangeEntry c;
  c.start = h.rmOpenStart;
  c.end = s - 1;
  c.value = h.rmOpenValue;
  if (h.rmCount < kRangeCap) {
    ring[(h.rmHead + h.rmCount) % kRangeCap] = c;
    h.rmCount++;
  } else {
    ring[h.rmHead] = c;
    h.rmHead = u16((h.rmHead + 1) % kRangeCap);
  }
  h.rmOpenStart = e;
  h.rmOpenValue = nv;
  return true;
}
// GetValue (rangemap.go:134-169)
__device__ __forceinline__ bool irm_get(const StreamHot &h, const RangeEntry *ring, u64 key, u64 &out) {
  out = 0;
  if (key >= h.rmOpenStart) {
    out = h.rmOpenValue;
    return true;
  }
  const int nc = h.rmCount;
  const u64 firstStart = nc > 0 ? ring[h.rmHead].start : h.rmOpenStart;
  if (key < firstStart) return false;
  RangeEntry next;
  next.start = h.rmOpenStart;
  next.end = 0;
  next.value = h.rmOpenValue;
  const u64 half = 1ull << 63;
  for (int idx = nc; idx >= 0; idx--) {
    if (idx != nc) {
      const RangeEntry rv = next;
      if ((key - rv.start) < half && (rv.end - key) < half) {
        out = rv.value;
        return true;
      }
    }
    if (idx > 0) {
      const RangeEntry prev = ring[(h.rmHead + idx - 1) % kRangeCap];
      const u64 before = key - prev.end, after = next.start - key;
      if (before > 0 && before < half && after > 0 && after < half) return false;
      next = prev;
    }
  }
  return false;
}

// the window's smoothed level (audiolevel.go:88-96; once per observe window: out of line)
__device__ __noinline__ double level_smooth(double prev, u32 activeDuration, u8 loudest, u32 observeDuration,
                                            double smoothFactor) {
  const double activityWeight = 20.0 * log10(double(activeDuration) / double(observeDuration));
  const double adjusted = double(loudest) - activityWeight;
  const double linear = pow(10.0, adjusted * (-1.0 / 20));
  return prev + (linear - prev) * smoothFactor;
}
// AudioLevel.Observe audiolevel.go:70-102
__device__ __forceinline__ void level_observe(StreamHot &h, const DevStream &s, u8 level, u32 durationMs, i64 arrivalNs) {
  h.lastObservedNs = arrivalNs;
  h.observedDuration += durationMs;
  if (level <= s.activeLevel) {
    h.activeDuration += durationMs;
    if (h.loudest > level) h.loudest = level;
  }
  if (h.observedDuration >= s.observeDuration) {
    h.smoothedLevel = h.activeDuration >= s.minActiveDuration
                          ? level_smooth(h.smoothedLevel, h.activeDuration, h.loudest, s.observeDuration, s.smoothFactor)
                          : 0.0;
    h.loudest = 127;
    h.activeDuration = 0;
    h.observedDuration = 0;
  }
}

// processHeaderExtensions' audio level (buffer.go:573-596) for one datagram
__device__ __forceinline__ void level_step(StreamHot &h, const DevStream &s, u32 pflags, u32 ts, u8 level,
                                           i64 arrival) {
  if (!(h.flags & S_LVL_TS_INIT)) {
    h.flags |= S_LVL_TS_INIT;
    h.latestTSForAudioLevel = ts;
  }
  if (pflags & IP_LEVEL) {
    if (u32(ts - h.latestTSForAudioLevel) < (1u << 31)) {
      const i64 dur = (i64(ts) - i64(h.latestTSForAudioLevel)) * 1000 / i64(s.clockRate);
      if (dur > 0) level_observe(h, s, level, u32(dur), arrival);
      h.latestTSForAudioLevel = ts;
    }
  }
}

// ---------------------------------------------------------------------------
// k_ing_lists: per track, the datagrams of each of its streams (simulcast
// layer slot 0-2) in arrival order — the lane of a stream walks its own list
// instead of scanning the whole track's datagrams.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_ing_lists(const lkf_raw_pkt *__restrict__ raws,
                                                  const DevStream *__restrict__ streams, u32 nstreams,
                                                  const u32 *__restrict__ tBegin, const u32 *__restrict__ tEnd,
                                                  u32 stride, u32 *__restrict__ list, u32 *__restrict__ cnt) {
  const u32 t = blockIdx.x, lane = threadIdx.x;
  const u64 lt = (1ull << lane) - 1;
  const u32 b = tBegin[t], e = tEnd[t];
  u32 c[3] = {0, 0, 0};
  for (u32 base = b; base < e; base += 64) {
    const u32 i = base + lane;
    int l = -1;
    if (i < e) {
      const u32 sid = raws[i].stream;
      if (sid < nstreams) l = int(streams[sid].layer);
      if (l > 2) l = -1;
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const u64 m = __ballot(l == k);
      if (l == k) list[size_t(k) * stride + b + c[k] + u32(__popcll(m & lt))] = i;
      c[k] += u32(__popcll(m));
    }
  }
  if (lane == 0)
    for (int k = 0; k < 3; k++) cnt[t * 3 + k] = c[k];
}

// ---------------------------------------------------------------------------
// buffer.DependencyDescriptorParser (dependencydescriptorparser.go:75-163) and
// its FrameIntegrityChecker (frameintegrity.go), per stream
// ---------------------------------------------------------------------------
// WrapAround<uint16,uint64>{IsRestartAllowed: false}.Update -> ExtendedVal
__device__ inline u64 wa16_ext(u64 &cycles, u64 &extHighest, u16 &start, u16 &highest, u32 &flags, u32 initBit,
                               u16 val) {
  const u64 full = 1ull << 16;
  if (!(flags & initBit)) {
    start = val;
    highest = val;
    extHighest = cycles + u64(val);
    flags |= initBit;
    return u64(val);
  }
  const u16 gap = u16(val - highest);
  if (gap > u16(full >> 1)) {
    u64 cyc = cycles;
    const u64 total = extHighest - u64(start) + 1;
    const bool wrapBack = u64(highest) < (full >> 1) && u64(val) >= (full >> 1);
    if (total > (full >> 1)) {
      if (wrapBack) cyc -= full;
      return cyc + u64(val);
    }
    if (!(u16(val - start) > u16(full >> 1)) && wrapBack) cyc -= full;
    return cyc + u64(val);
  }
  if (val < highest) cycles += full;
  highest = val;
  extHighest = cycles + u64(val);
  return extHighest;
}

// PacketHistory frameintegrity.go:46-146
__device__ inline void ph_set(DDIngState &d, u64 seq, bool r) {
  const u64 i = (seq - d.phBase) % u64(kFICPktWords * 64);
  if (r)
    d.phBits[i >> 6] |= 1ull << (i & 63);
  else
    d.phBits[i >> 6] &= ~(1ull << (i & 63));
}
__device__ inline void ph_add(DDIngState &d, u64 seq) {
  if (!(d.flags & DI_PH_INIT)) {
    d.flags |= DI_PH_INIT;
    d.phBase = seq > 100 ? seq - 100 : 0;
    d.phLast = seq;
    ph_set(d, seq, true);
    return;
  }
  if (seq <= d.phBase) return;
  if (seq <= d.phLast) {
    if (d.phLast - seq < u64(kFICPktWords * 64)) ph_set(d, seq, true);
    return;
  }
  if (seq - d.phLast - 1 >= u64(kFICPktWords * 64)) {  // the clearing loop wraps the whole ring
    for (int w = 0; w < kFICPktWords; w++) d.phBits[w] = 0;
  } else {
    for (u64 i = d.phLast + 1; i < seq; i++) ph_set(d, i, false);
  }
  ph_set(d, seq, true);
  d.phLast = seq;
}
__device__ inline bool ph_consecutive(const DDIngState &d, u64 start, u64 end) {
  const u64 pc = u64(kFICPktWords * 64);
  if (start > end || end - start >= pc) return false;
  const u64 si = (start - d.phBase) % pc, ei = (end - d.phBase) % pc;
  const int sIdx = int(si >> 6), sOff = int(si & 63), eIdx = int(ei >> 6), eOff = int(ei & 63);
  if (sIdx == eIdx && end - start <= 64) {
    const int w = eOff - sOff + 1;
    const u64 tb = (w >= 64 ? ~0ull : ((1ull << w) - 1)) << sOff;
    return (d.phBits[sIdx] & tb) == tb;
  }
  const u64 lhs = (d.phBits[sIdx] >> sOff) + 1;
  const u64 rhs = (64 - sOff) >= 64 ? 0 : (1ull << (64 - sOff));
  if (lhs != rhs) return false;
  for (int i = sIdx + 1; i != eIdx; i++) {
    if (i == kFICPktWords) {
      i = 0;
      if (i == eIdx) break;
    }
    if (d.phBits[i] + 1 != 0) return false;
  }
  const u64 tb = eOff + 1 >= 64 ? ~0ull : ((1ull << (eOff + 1)) - 1);
  return (d.phBits[eIdx] & tb) == tb;
}
// FrameIntegrityChecker.AddPacket / FrameIntegrity
__device__ inline void fe_add(DDIngState &d, int slot, u64 seq, bool first, bool last) {
  u8 f = d.feFlags[slot];
  if (f & 4) return;
  if (!(f & 1) && first) {
    f |= 1;
    d.feStart[slot] = seq;
  }
  if (!(f & 2) && last) {
    f |= 2;
    d.feEnd[slot] = seq;
  }
  if ((f & 3) == 3 && ph_consecutive(d, d.feStart[slot], d.feEnd[slot])) f |= 4;
  d.feFlags[slot] = f;
}
__device__ inline void fc_add(DDIngState &d, u64 seq, u64 fn, bool first, bool last) {
  ph_add(d, seq);
  if (!(d.flags & DI_FC_INIT)) {
    d.flags |= DI_FC_INIT;
    d.fcBase = d.fcLast = fn;
  }
  if (fn < d.fcBase) return;
  if (fn <= d.fcLast) {
    if (d.fcLast - fn >= u64(kFICFrames)) return;
    fe_add(d, int((fn - d.fcBase) % u64(kFICFrames)), seq, first, last);
    return;
  }
  if (fn - d.fcLast >= u64(kFICFrames)) {  // the reset loop covers every slot
    for (int i = 0; i < kFICFrames; i++) d.feFlags[i] = 0;
  } else {
    for (u64 i = d.fcLast + 1; i <= fn; i++) d.feFlags[int((i - d.fcBase) % u64(kFICFrames))] = 0;
  }
  fe_add(d, int((fn - d.fcBase) % u64(kFICFrames)), seq, first, last);
  d.fcLast = fn;
}
__device__ inline bool fc_integrity(const DDIngState &d, u64 fn) {
  if (fn < d.fcBase || fn > d.fcLast || d.fcLast - fn >= u64(kFICFrames)) return false;
  return (d.feFlags[int((fn - d.fcBase) % u64(kFICFrames))] & 4) != 0;
}

// The fields of a parsed descriptor the parser state needs
struct DDLite {
  u16 frameNumber;
  u8 flags, sid, tid;  // flags: DP_*
  u32 activeMask;
  int err;  // dd_parse_lite's result
};
// The parser state's part of Parse (dependencydescriptorparser.go:100-162) for
// a descriptor already read: sequence / frame-number unwrap, the frame
// integrity checker, an attached structure, the active decode targets.
// false -> no ExtPacket (out as far as it was filled, as Parse leaves it)
__device__ bool dd_fold(DDIngState &d, u16 sn, const DDLite &o, bool att, IngDD &out) {
  const u64 extSeq = wa16_ext(d.seqCycles, d.seqExtHighest, d.seqStart, d.seqHighest, d.flags, DI_SEQ_INIT, sn);
  const u64 extFN = wa16_ext(d.fnCycles, d.fnExtHighest, d.fnStart, d.fnHighest, d.flags, DI_FN_INIT, o.frameNumber);
  if (extFN < d.structureExtFN) return false;  // ErrFrameEarlierThanKeyFrame
  fc_add(d, extSeq, extFN, o.flags & DP_FIRST, o.flags & DP_LAST);
  out.extFN = extFN;
  out.flags = fc_integrity(d, extFN) ? LKF_DD_INTEGRITY : 0;
  if (att) {
    if (!(o.flags & DP_FIRST)) return false;  // ErrDDStructureAttachedToNonFirstPacket
    d.flags ^= DI_CUR;
    d.flags |= DI_HAS_STRUCT;
    d.structureExtFN = extFN;
    out.flags |= LKF_DD_STRUCTURE_UPDATED | LKF_DD_ACTIVE_UPDATED;
  }
  if ((o.flags & DP_ACTIVE) && extSeq > d.activeExtSeq) {
    d.activeExtSeq = extSeq;
    if (o.activeMask != d.activeMask) {
      d.activeMask = o.activeMask;
      out.flags |= LKF_DD_ACTIVE_UPDATED;
    }
  }
  out.extKFN = d.structureExtFN;
  out.present = 1;
  out.sid = o.sid;
  out.tid = o.tid;
  return true;
}

// DependencyDescriptorExtension.Unmarshal against the structure in force
// (cur; nullptr before any) with no structure attached (the caller checked
// the flag): -> (error, the descriptor's DDLite), out of line (one call per
// lane of a run).
// (returned by value: a reference to the caller's copy would put it on every
// lane's private stack)
__device__ __noinline__ DDLite dd_parse_lite(const u8 *buf, int len, const DDStruct *cur) {
  DDPkt o = {};
  bool att = false;
  DDLite out;
  out.err = dd::dd_parse(buf, len, cur, nullptr, o, att);
  out.frameNumber = o.frameNumber;
  out.flags = o.flags;
  out.sid = o.sid;
  out.tid = o.tid;
  out.activeMask = o.activeMask;
  return out;
}
// a descriptor that attaches a structure (template_dependency_structure_present_flag)
__device__ __forceinline__ bool dd_attaches(const u8 *buf, int len) { return len > 3 && (buf[3] & 0x80); }

// Parse: false -> the packet produces no ExtPacket (a parse error); *limit
// when an engine limit (not the reference) refused it
__device__ __noinline__ bool dd_ingest(DDIngState &d, DDStruct *structs, const u8 *buf, int len, u16 sn, IngDD &out,
                                       bool &limit) {
  limit = false;
  const u32 cur = (d.flags & DI_CUR) ? 1u : 0u;
  DDPkt o = {};
  bool att = false;
  const int e = dd::dd_parse(buf, len, (d.flags & DI_HAS_STRUCT) ? structs + cur : nullptr, structs + (cur ^ 1u), o,
                             att);
  if (e) {
    limit = e == dd::LIMIT;
    return false;
  }
  DDLite l;
  l.frameNumber = o.frameNumber;
  l.flags = o.flags;
  l.sid = o.sid;
  l.tid = o.tid;
  l.activeMask = o.activeMask;
  return dd_fold(d, sn, l, att, out);
}

// The stream's RTX bucket inside the stream kernel (mediatransportutil
// bucket.AddPacketWithSequenceNumber as buffer.go:471-481 calls it; oracle
// bucket_oracle.h): the logical state (head, step) in LDS, the slot tags in
// HBM, and this ingest's writer of each slot (sOwn in LDS for rings of up to
// kBktLds slots, else the global owner words tagged with the ingest epoch) so
// a slot taken again later in the batch cancels the earlier datagram's copy.
constexpr int kBktLds = 2048;
constexpr u32 kNoOwner = 0xFFFFFFFFu;
struct BktCtx {
  BucketState *b;  // LDS
  u32 *tag;        // the stream's slot tags
  u64 *owner;      // the stream's owner words (rings above kBktLds)
  u64 *store;      // per datagram of the batch
  u32 *sOwn;       // LDS owner map (rings up to kBktLds)
  u64 ep;          // ingest epoch << 32
  bool lds;
};
__device__ __forceinline__ int bkt_wrap(int x, int M) {
  x %= M;
  return x < 0 ? x + M : x;
}
// the slot's previous writer in this ingest is not stored; ic takes it (kNoOwner: invalidated)
__device__ __forceinline__ void bkt_supersede(const BktCtx &k, int sl, u32 ic) {
  if (k.lds) {
    const u32 o = k.sOwn[sl];
    if (o != kNoOwner) k.store[o] = 0;
    k.sOwn[sl] = ic;
  } else {
    const u64 o = k.owner[sl];
    if ((o & 0xFFFFFFFF00000000ull) == k.ep) k.store[u32(o)] = 0;
    k.owner[sl] = ic == kNoOwner ? 0 : (k.ep | ic);
  }
}
// AddPacketWithSequenceNumber for one datagram (one lane): push (the skipped
// slots invalidated, the packet at the new head) or set (an older SN inside
// the window, unless the slot already holds it: ErrRTXPacket); too old or too
// large (> MaxPktSize - 2) is refused.  -> the slot, or -1 (no ExtPacket).
__device__ int bkt_add_one(const BktCtx &k, u16 sn, u32 len, u32 ic) {
  BucketState &b = *k.b;
  const int M = int(b.maxSteps);
  int slot = -1;
  if (len <= 1498) {
    if (!b.init) {
      b.head = u16(sn - 1);
      b.init = 1;
    }
    const u16 diff = u16(sn - b.head);
    if (diff == 0 || diff > (1u << 15)) {  // set
      const int back = int(u16(b.head - sn));
      if (back < M) {
        const int sl = bkt_wrap(int(b.step) - back - 1, M);
        const u32 t = k.tag[sl];
        if (!((t >> 16) != 0xFFFFu && u16(t) == sn)) slot = sl;  // (a duplicate is not overwritten)
      }
    } else {  // push
      const int gap = int(diff) - 1;
      b.head = sn;
      for (int i = 0; i < min(gap, M); i++) {
        const int sl = bkt_wrap(int(b.step) + i, M);
        k.tag[sl] = 0xFFFF0000u;
        bkt_supersede(k, sl, kNoOwner);
      }
      slot = bkt_wrap(int(b.step) + gap, M);
      b.step = u32(bkt_wrap(int(b.step) + gap + 1, M));
    }
  }
  if (slot >= 0) {
    k.tag[slot] = (len << 16) | sn;
    bkt_supersede(k, slot, ic);
    k.store[ic] = (1ull << 63) | (u64(sn) << 32) | u64(b.base + u32(slot));
  }
  return slot;
}

// rtpStatsBase.updateGapHistogram (rtpstats_base.go:871-882) of the receiver
__device__ __forceinline__ void rx_gap(u32 *gap, u64 g) {
  if (g < 2) return;
  const u64 missing = g - 1;
  atomicAdd(&gap[missing > u64(kGapBins) ? kGapBins - 1 : u32(missing - 1)], 1u);
}
// rtpStatsBase.updateJitter (rtpstats_base.go:775-810) of the receiver (Go's
// int64 products wrap: formed in u64)
__device__ __forceinline__ u64 rx_transit(const StreamHot &h, u32 clockRate, u64 ets, i64 t) {
  const i64 since = i64(u64(t) - u64(h.firstTime));
  return u64(i64(u64(since) * u64(i64(clockRate))) / 1000000000LL) - ets;
}
__device__ __forceinline__ void rx_jitter_fold(StreamHot &h, u64 transit, u64 ets) {
  if (h.lastTransit != 0) {
    i64 d = i64(transit - h.lastTransit);
    if (d < 0) d = i64(0 - u64(d));
    h.jitter += (double(d) - h.jitter) / 16;
    if (h.jitter > h.maxJitter) h.maxJitter = h.jitter;
  }
  h.lastTransit = transit;
  h.lastJitterExtTs = ets;
}
__device__ __forceinline__ void rx_jitter(StreamHot &h, u32 clockRate, u64 ets, i64 t) {
  if (h.lastJitterExtTs == ets) return;
  rx_jitter_fold(h, rx_transit(h, clockRate, ets, t), ets);
}

// One datagram through Buffer.calc (buffer.go:407-489): processHeaderExtensions,
// RTPStatsReceiver.Update (rtpstats_receiver.go:76-241), the padding
// RangeMap, the dependency descriptor; its flow, forward flag and DD record.
// (the datagram, its descriptor and the stream come as pointers into the
// batch's arrays and the bucket context from LDS: references to the caller's
// per-lane copies put them on every lane's private stack — 400 B of scratch a
// lane, written by every wave of the stream kernel, r4's tick WRITE_SIZE)
template <int HS>
__device__ __noinline__ lkf_flow ing_step(StreamHot &h, u64 *hs, RangeEntry *ring, const DevStream *sg,
                                         const IngParsed *pg, const lkf_raw_pkt *rg, u32 ic, lkf_flow *flows,
                                         u32 *fwd, IngDD *ingDD, const u8 *raw, DDIngState *dds,
                                         DDStruct *ddStructs, u32 *err, const BktCtx *bkg, bool bkOn, u32 *gap) {
  const DevStream s = *sg;
  const IngParsed p = *pg;
  const lkf_raw_pkt rp = *rg;
  const BktCtx bk = *bkg;
  const i64 arrival = rp.arrival_ns;
  lkf_flow f = {};
  f.pkt = 0xffffffffu;
  u32 forward = 0;
  IngDD dv = {};
  do {
    if (!(p.flags & IP_OK)) {
      f.flags = LKF_FLOW_BAD;
      break;
    }
    // processHeaderExtensions (buffer.go:573-596)
    if (s.levelExt) level_step(h, s, p.flags, p.ts, p.level, arrival);
    // RTPStatsReceiver.Update (rtpstats_receiver.go:76-241)
    const int hdrSize = p.hdrSize, payloadSize = p.payloadLen, paddingSize = p.paddingSize;
    WAResult rsn, rts;
    if (!(h.flags & S_INIT)) {
      if (payloadSize == 0) {
        f.flags = LKF_FLOW_NOT_HANDLED;
        break;
      }
      h.flags |= S_INIT;
      h.firstTime = arrival;  // rtpstats_receiver.go:106-107
      h.highestTime = arrival;
      rsn = wa16_update(h, p.sn);
      rts = wa32_update(h, p.ts);
    } else {
      rsn = wa16_update(h, p.sn);
      if (rsn.unhandled) {
        f.flags = LKF_FLOW_NOT_HANDLED;
        break;
      }
      rts = wa32_update(h, p.ts);
    }
    const u64 pktSize = u64(hdrSize + payloadSize + paddingSize);
    const i64 gapSN = i64(rsn.extVal - rsn.preHighest);
    bool dup = false, ooo = false;
    if (gapSN <= 0) {
      if (gapSN != 0) h.packetsOutOfOrder++;
      const i64 diff = i64(rsn.preHighest - rsn.extVal);
      if (diff >= 0 && diff < i64(kHistWords) * 64) {  // isInRange :427-430
        if (hist_isset<HS>(hs, rsn.extVal)) {
          h.bytesDuplicate += pktSize;
          h.headerBytesDuplicate += u64(hdrSize);
          h.packetsDuplicate++;
          dup = true;
        } else {
          h.packetsLost--;
          hist_set<HS>(hs, rsn.extVal);
        }
      }
      ooo = true;
    } else {
      rx_gap(gap, u64(gapSN));
      hist_clear_range<HS>(hs, rsn.preHighest + 1, rsn.extVal - 1);
      h.packetsLost += u64(gapSN - 1);
      hist_set<HS>(hs, rsn.extVal);
      if (p.ts != u32(rts.preHighest)) h.highestTime = arrival;  // :209-213
      if (gapSN > 1) {
        f.flags |= LKF_FLOW_HAS_LOSS;
        f.loss_start = rsn.preHighest + 1;
        f.loss_end = rsn.extVal;
      }
    }
    f.ext_sn = rsn.extVal;
    f.ext_ts = rts.extVal;
    if (!dup) {
      if (payloadSize == 0) {
        h.packetsPadding++;
        h.bytesPadding += pktSize;
        h.headerBytesPadding += u64(hdrSize);
      } else {
        h.bytes += pktSize;
        h.headerBytes += u64(hdrSize);
        if (p.flags & IP_MARKER) h.frames++;
        rx_jitter(h, s.clockRate, rts.extVal, arrival);
      }
    }
    if (dup) f.flags |= LKF_FLOW_DUPLICATE;
    if (ooo) f.flags |= LKF_FLOW_OUT_OF_ORDER;
    // Buffer.calc (buffer.go:439-489)
    if (payloadSize == 0 && (!ooo || dup)) {
      if (!ooo) irm_exclude(h, ring, rsn.extVal, rsn.extVal + 1);
      f.flags |= LKF_FLOW_PADDING;
      break;
    }
    u64 adj = 0;
    if (!irm_get(h, ring, rsn.extVal, adj)) {
      f.flags |= LKF_FLOW_BAD;
      break;
    }
    f.ext_sn = rsn.extVal - adj;
    if (dup) break;  // the RTX bucket already holds it (ErrRTXPacket)
    // AddPacketWithSequenceNumber under the adjusted SN (buffer.go:471-481):
    // too old, too large or already held -> no ExtPacket (before getExtPacket)
    if (bkOn && bkt_add_one(bk, u16(f.ext_sn), rp.len, ic) < 0) break;
    f.flags |= LKF_FLOW_BUCKET;
    // getExtPacket (buffer.go:599-671): the dependency descriptor first
    if (payloadSize > 0 && s.ddIdx != 0xffffffffu && p.ddLen) {
      bool limit = false;
      if (!dd_ingest(*dds, ddStructs + size_t(s.ddIdx) * 2, raw + rp.off + p.ddOff, p.ddLen,
                     u16(f.ext_sn), dv, limit)) {
        if (limit) atomicOr(err, 4u);
        f.flags |= LKF_FLOW_BAD;
        break;
      }
      dv.ddOff = p.ddOff;
      dv.ddLen = p.ddLen;
    }
    // VP8 unmarshal failed, or VP9 without a descriptor that failed
    if ((p.flags & IP_VP8_BAD) && !(s.codec == LKF_CODEC_VP9 && dv.present)) {
      f.flags |= LKF_FLOW_BAD;
      break;
    }
    forward = 1;
    f.flags |= LKF_FLOW_FORWARD;
  } while (false);
  flows[ic] = f;
  fwd[ic] = forward;
  if (ingDD) ingDD[ic] = dv;
  return f;
}

// The datagrams of a closed stream (lkf_remove_track): not handled, no state
// change, no ExtPacket (lanes first, first + step, ...)
__device__ void closed_flows(const DevStream &s, u32 sid, u32 pb, u32 pe, const lkf_raw_pkt *raws, lkf_flow *flows,
                             u32 *fwd, IngDD *ingDD, const u32 *list, const u32 *cnt, u32 stride, u32 first,
                             u32 step, NackIn *nackIn) {
  const bool useList = s.layer < 3;
  const u32 nIdx = useList ? cnt[s.track * 3 + s.layer] : pe - pb;
  const u32 *lst = list + size_t(useList ? s.layer : 0) * stride + pb;
  for (u32 k = first; k < nIdx; k += step) {
    const u32 ic = useList ? lst[k] : pb + k;
    if (raws[ic].stream != sid) continue;
    lkf_flow f = {};
    f.pkt = 0xffffffffu;
    f.flags = LKF_FLOW_NOT_HANDLED;
    flows[ic] = f;
    fwd[ic] = 0;
    if (ingDD) ingDD[ic] = IngDD{};
    if (nackIn && useList) nackIn[size_t(lst - list) + k] = NackIn{raws[ic].arrival_ns, sid, 0u, 0u, 0u};
  }
}

// ---------------------------------------------------------------------------
// k_ing_stream_wave: one wave per stream, lanes over its datagrams.  The
// receiver recurrence is serial, but a run of in-order datagrams (SN gap 1 to
// 2^15, TS gap up to 2^31, a payload, no audio level or DD to observe, the
// padding RangeMap's open range covering them) only accumulates: the extended
// SN and TS are prefix sums of the gaps, the counters are sums, the history
// is one range clear plus one bit per datagram.  A chunk's leading run is
// taken in one step; the datagram that ends it (reorder, duplicate, padding,
// DD, first packet, audio) goes through ing_step on lane 0, as the
// lane-per-stream kernel does for every datagram.
// ---------------------------------------------------------------------------
// a 64-bit value of lane x (readlane returns int: the low word must not sign-extend)
__device__ __forceinline__ u64 rl_u64(u64 v, u32 x) {
  return (u64(u32(__builtin_amdgcn_readlane(int(u32(v >> 32)), x))) << 32) |
         u64(u32(__builtin_amdgcn_readlane(int(u32(v)), x)));
}
__device__ __forceinline__ u64 wave_incl_scan_u64(u64 v, u32 lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u64 o = __shfl_up(v, d, 64);
    if (lane >= u32(d)) v += o;
  }
  return v;
}
__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// a datagram's NackIn word: its SN, whether updateStreamState ran, whether it
// pushes a loss range
__device__ __forceinline__ u32 nk_snfl(const IngParsed &p, const lkf_flow &f) {
  const bool ok = (p.flags & IP_OK) != 0;
  return u32(p.sn) | ((ok ? 2u : 0u) | (ok && (f.flags & LKF_FLOW_HAS_LOSS) ? 4u : 0u)) << 16;
}

// Two instantiations: <false> for the streams without a dependency-descriptor
// parser, <true> (launched only when DD streams exist) for those with one,
// whose DependencyDescriptorParser + FrameIntegrityChecker state (3.3 KB) is
// staged in LDS for the batch — lane 0's fold of the descriptors then updates
// it there (the plain streams keep the smaller LDS footprint and occupancy).
// Occupancy floor of the stream wave (waves per SIMD).  3 (round 6) over 4:
// the registers it frees take the spills out of the serial step, and a batch's
// 4,000 streams still fit the GPU in one round (configs[1] 0.745 -> 0.727 ms,
// 10-ms tick 0.575 -> 0.553 ms, configs[4] 13.46 -> 13.21 ms; 2: the tick alike,
// configs[4] 14.7 ms; profiles/r6_ab_runs.txt)
#ifndef LKF_ING_PER_WAVE  // (A/B) streams per stream-wave workgroup; 0: from the ingest's length
#define LKF_ING_PER_WAVE 0
#endif
#ifndef LKF_ING_WAVES
#define LKF_ING_WAVES 3
#endif
template <bool DDK>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LKF_ING_WAVES))) k_ing_stream_wave(
    const lkf_raw_pkt *__restrict__ raws, const IngParsed *__restrict__ q, const DevStream *__restrict__ streams,
    StreamHot *__restrict__ hot, u64 *__restrict__ hist, RangeEntry *__restrict__ rings,
    const u32 *__restrict__ tBegin, const u32 *__restrict__ tEnd, lkf_flow *__restrict__ flows,
    u32 *__restrict__ fwd, const u8 *__restrict__ raw, DDIngState *ddStates, DDStruct *ddStructs,
    IngDD *__restrict__ ingDD, u32 *err, const u32 *__restrict__ list, const u32 *__restrict__ cnt, u32 stride,
    BktArgs bka, u32 *__restrict__ rxGap, NackIn *__restrict__ nackIn, u32 nstreams, u32 perWave) {
  static_assert(kHistWords == 64, "one history word per lane");
  static_assert(sizeof(StreamHot) == 64 * sizeof(u32), "one StreamHot dword per lane");
  __shared__ u64 sHist[kHistWords];
  __shared__ StreamHot sh;
  __shared__ BucketState sB;
  __shared__ u32 sOwn[kBktLds];  // (LDS is otherwise small: 4 waves per SIMD either way)
  __shared__ __attribute__((aligned(16))) u8 sDDIRaw[DDK ? sizeof(DDIngState) : 16];
  __shared__ BktCtx sBk;  // (ing_step's copy of bk)
  // A wave serves perWave consecutive streams, one after the other: a short
  // ingest (10-ms ticks: one or two datagrams per stream) with one workgroup
  // per stream is bound by the workgroup dispatch rate (≈240 per µs).
  const u32 lane = threadIdx.x;
  for (u32 jw = 0; jw < perWave; jw++) {
  const u32 sid = blockIdx.x * perWave + jw;
  if (sid >= nstreams) break;
  if (jw) __syncthreads();  // (the previous stream's LDS is read out)
  const DevStream s = streams[sid];
  if ((s.ddIdx != 0xffffffffu) != DDK) continue;  // the other instantiation's stream
  const u32 pb = tBegin[s.track], pe = tEnd[s.track];
  if (pb >= pe) continue;
  if (s.closed) {  // Buffer.Close: Write returns io.EOF, nothing is processed
    closed_flows(s, sid, pb, pe, raws, flows, fwd, ingDD, list, cnt, stride, lane, 64, nackIn);
    continue;
  }
  u64 *const hg = hist + size_t(sid) * kHistWords;
  u32 *const gap = rxGap + size_t(sid) * kGapWords;
  // (the loaded words are kept: only the ones the batch changes go back)
  const u64 hist0 = hg[lane];
  const u32 hot0 = reinterpret_cast<const u32 *>(hot + sid)[lane];
  sHist[lane] = hist0;
  reinterpret_cast<u32 *>(&sh)[lane] = hot0;
  // the stream's RTX bucket (bka.state nullptr: no buckets)
  const bool bkOn = bka.state != nullptr;
  BktCtx bk = {};
  int M = 1;
  if (bkOn) {
    if (lane < 4) reinterpret_cast<u32 *>(&sB)[lane] = reinterpret_cast<const u32 *>(bka.state + sid)[lane];
    __syncthreads();
    M = int(sB.maxSteps);
    bk.b = &sB;
    bk.tag = bka.tag + sB.base;
    bk.owner = bka.owner + sB.base;
    bk.store = bka.store;
    bk.sOwn = sOwn;
    bk.ep = u64(bka.epoch) << 32;
    bk.lds = M <= kBktLds;
    if (bk.lds)
      for (int i = int(lane); i < M; i += 64) sOwn[i] = kNoOwner;
  }
  if (lane == 0) sBk = bk;
  DDIngState *dds = nullptr;
  if (DDK) {
    dds = reinterpret_cast<DDIngState *>(sDDIRaw);
    const uint4 *g = reinterpret_cast<const uint4 *>(ddStates + s.ddIdx);
    uint4 *l = reinterpret_cast<uint4 *>(sDDIRaw);
    for (u32 i = lane; i < sizeof(DDIngState) / 16; i += 64) l[i] = g[i];
  }
  __syncthreads();
  RangeEntry *ring = rings + size_t(sid) * kRangeCap;
  const bool useList = s.layer < 3;
  const u32 nIdx = useList ? cnt[s.track * 3 + s.layer] : pe - pb;
  const u32 *lst = list + size_t(useList ? s.layer : 0) * stride + pb;
  // datagrams a run may take without looking at them twice (the state part
  // is checked per chunk)
  // (audio streams run too: the audio level's own recurrence is folded over
  // each run's datagrams in order, below)
  const bool runStream = true;
  const bool hasDD = s.ddIdx != 0xffffffffu;
  for (u32 j = 0; runStream && j < nIdx; j += 64) {
    // a chunk of 64 datagrams stays in registers while runs and serial steps
    // take its lanes in order from `pos`
    const u32 k = j + lane;
    const bool in = k < nIdx;
    u32 ic = 0;
    IngParsed p = {};
    lkf_raw_pkt rp = {};
    if (in) {
      ic = useList ? lst[k] : pb + k;
      p = q[ic];
      rp = raws[ic];
    }
    const u32 m = min(64u, nIdx - j);
    u32 nkSnFl = 0, nkS0 = 0, nkLen = 0;  // this lane's NackIn (its datagram's flow)
    for (u32 pos = 0; pos < m;) {
    const u32 need = S_INIT | S_SN_INIT | S_TS_INIT;
    const bool stateOk = runStream && (sh.flags & need) == need && sh.rmOpenStart <= sh.snExtHighest + 1;
    const u16 prevSn = u16(__shfl_up(u32(p.sn), 1, 64));
    const u32 prevTs = u32(__shfl_up(p.ts, 1, 64));
    const u16 gs = u16(p.sn - (lane == pos ? sh.snHighest : prevSn));
    const u32 gt = p.ts - (lane == pos ? sh.tsHighest : prevTs);
    // (a descriptor that attaches a structure changes what the later ones are
    // read against: it takes the serial step)
    const bool ddLane = hasDD && p.ddLen;
    const bool ok = lane >= pos && stateOk && in && rp.stream == sid && (p.flags & IP_OK) && p.payloadLen > 0 &&
                    !(p.flags & IP_VP8_BAD) && !(ddLane && dd_attaches(raw + rp.off + p.ddOff, p.ddLen)) &&
                    gs >= 1 && gs <= 0x8000u && gt <= 0x80000000u && (!bkOn || rp.len <= 1498u);
    const u64 snScan = wave_incl_scan_u64(ok ? u64(gs) : 0, lane);  // only read below the run end
    u64 bad = ~__ballot(ok) & ~((1ull << pos) - 1);
    // the history update below is exact while the run spans < 4096 SNs
    bad |= __ballot(lane >= pos && snScan >= u64(kHistWords) * 64);
    // the bucket: every datagram of the run is a push; the first one's step
    // from the bucket head d0 (its adjusted SN against the head), the others'
    // their SN gaps; S = the run's pushes so far, slots distinct while S <= M
    u64 bS = 0;
    u32 d0 = 0;
    if (bkOn) {
      const u32 gs0 = __builtin_amdgcn_readlane(u32(gs), pos);
      d0 = u32(u16(u16(sh.snExtHighest + gs0 - sh.rmOpenValue) - sB.head));
      if (!sB.init || d0 < 1 || d0 > 0x8000u) bad |= 1ull << pos;
      bS = snScan - gs0 + d0;
      bad |= __ballot(lane >= pos && bS > u64(M));
    }
    const u32 end = bad ? u32(__ffsll(static_cast<long long>(bad)) - 1) : 64u;  // the run is [pos, end)
    if (end == pos) {  // the datagram at pos through the serial Buffer.calc step
      if (lane == pos && rp.stream == sid) {
        const lkf_flow fo = ing_step<1>(sh, sHist, ring, streams + sid, q + ic, raws + ic, ic, flows, fwd, ingDD, raw,
                                        dds, ddStructs, err, &sBk, bkOn, gap);
        nkSnFl = nk_snfl(p, fo);
        nkS0 = u32(u16(fo.loss_start));
        nkLen = u32(min<u64>(fo.loss_end - fo.loss_start, 0xffffffffull));
      }
      __syncthreads();
      pos++;
      continue;
    }
    const u32 L = end - pos;
    const bool run = lane >= pos && lane < end;
    const u64 tsScan = wave_incl_scan_u64(run ? u64(gt) : 0, lane);
    const u64 ext = sh.snExtHighest + snScan, extTs = sh.tsExtHighest + tsScan;
    const u64 pktSize = u64(p.hdrSize + p.payloadLen + p.paddingSize);
    const u64 bytesRun = wave_sum_u64(run ? pktSize : 0), hdrRun = wave_sum_u64(run ? u64(p.hdrSize) : 0);
    const u32 framesRun = u32(__popcll(__ballot(run && (p.flags & IP_MARKER))));
    const u64 extLast = __shfl(ext, int(end - 1), 64), extTsLast = __shfl(extTs, int(end - 1), 64);
    const u16 snLast = u16(__shfl(u32(p.sn), int(end - 1), 64));
    const u32 tsLast = u32(__shfl(p.ts, int(end - 1), 64));
    const u64 bSLast = __shfl(bS, int(end - 1), 64);
    // RTPStatsReceiver timing: highestTime from the run's last lane that
    // starts a timestamp (the TS never decreases inside a run); the jitter
    // filter over the run's new timestamps, in order (a float64 recurrence:
    // transits in parallel, the fold serial and wave-uniform)
    const u64 newTs = __ballot(run && p.ts != (lane == pos ? sh.tsHighest : prevTs));
    const u64 prevExtTs = __shfl_up(extTs, 1, 64);
    const u64 newJ = __ballot(run && extTs != (lane == pos ? sh.lastJitterExtTs : prevExtTs));
    const u64 transit = rx_transit(sh, s.clockRate, extTs, rp.arrival_ns);
    if (run) rx_gap(gap, u64(gs));
    // getExtPacket's dependency descriptor for the run's datagrams that carry
    // one (buffer.go:599-620, after the bucket as Buffer.calc orders them):
    // each lane reads its descriptor against the structure in force (none of
    // them attaches one), then lane 0 folds them into the parser state in
    // order; a descriptor the parser refuses leaves its datagram without an
    // ExtPacket (failMask).
    u64 ddFail = 0;
    const u64 ddM = __ballot(run && ddLane);
    if (ddM) {
      DDIngState &dst = *dds;
      const u32 dfl = dst.flags;
      const DDStruct *curS = (dfl & DI_HAS_STRUCT) ? ddStructs + size_t(s.ddIdx) * 2 + ((dfl & DI_CUR) ? 1 : 0) : nullptr;
      DDLite dl = {};
      if (run && ddLane) dl = dd_parse_lite(raw + rp.off + p.ddOff, p.ddLen, curS);
      const int de = dl.err;
      const u32 dlw0 = u32(dl.frameNumber) | (u32(dl.flags) << 16) | (u32(dl.sid & 15) << 24) | (u32(dl.tid & 15) << 28);
      const u16 snL = u16(ext - sh.rmOpenValue);
      // (the loop and its readlanes run on the whole wave, so every lane's
      // operands exist; only lane 0 folds and stores)
      for (u64 w = ddM; w; w &= w - 1) {
        const u32 x = u32(__ffsll(static_cast<long long>(w)) - 1);
        const int ex = __builtin_amdgcn_readlane(de, x);
        const u32 icx = u32(__builtin_amdgcn_readlane(int(ic), x));
        const u32 w0 = u32(__builtin_amdgcn_readlane(int(dlw0), x));
        const u32 amx = u32(__builtin_amdgcn_readlane(int(dl.activeMask), x));
        const u16 snx = u16(__builtin_amdgcn_readlane(int(snL), x));
        const u32 offx = u32(__builtin_amdgcn_readlane(int(p.ddOff), x));
        const u32 lenx = u32(__builtin_amdgcn_readlane(int(p.ddLen), x));
        if (lane == 0) {
          IngDD dv = {};
          bool okx = false;
          if (ex) {
            if (ex == dd::LIMIT) atomicOr(err, 4u);
          } else {
            DDLite o;
            o.frameNumber = u16(w0);
            o.flags = u8(w0 >> 16);
            o.sid = u8((w0 >> 24) & 15);
            o.tid = u8(w0 >> 28);
            o.activeMask = amx;
            okx = dd_fold(dst, snx, o, false, dv);
            if (okx) {
              dv.ddOff = u16(offx);
              dv.ddLen = u8(lenx);
            }
          }
          if (ingDD) ingDD[icx] = dv;
          if (!okx) ddFail |= 1ull << x;
        }
      }
      ddFail = rl_u64(ddFail, 0);
    }
    if (run) {
      lkf_flow f = {};
      f.pkt = 0xffffffffu;
      f.ext_sn = ext - sh.rmOpenValue;
      f.ext_ts = extTs;
      f.flags = LKF_FLOW_FORWARD | LKF_FLOW_BUCKET;
      if (gs > 1) {
        f.flags |= LKF_FLOW_HAS_LOSS;
        f.loss_start = ext - gs + 1;
        f.loss_end = ext;
      }
      const bool failed = (ddFail >> lane) & 1;
      if (failed) f.flags = u8((f.flags & ~LKF_FLOW_FORWARD) | LKF_FLOW_BAD);
      flows[ic] = f;
      nkSnFl = nk_snfl(p, f);
      nkS0 = u32(u16(f.loss_start));
      nkLen = u32(min<u64>(f.loss_end - f.loss_start, 0xffffffffull));
      fwd[ic] = failed ? 0u : 1u;
      if (ingDD && !ddLane) ingDD[ic] = IngDD{};
      if (bkOn) {  // the run's pushes: this lane's skipped slots invalidated, then its own
        const u32 dk = lane == pos ? d0 : u32(gs);
        const int step0 = int(sB.step);
        const int first = int(bS - dk);  // pushes before this lane's gap
        for (u32 i = 0; i + 1 < dk; i++) {
          const int sl = bkt_wrap(step0 + first + int(i), M);
          bk.tag[sl] = 0xFFFF0000u;
          bkt_supersede(bk, sl, kNoOwner);
        }
        const int slot = bkt_wrap(step0 + int(bS) - 1, M);
        const u16 sn = u16(f.ext_sn);
        bk.tag[slot] = (rp.len << 16) | sn;
        bkt_supersede(bk, slot, ic);
        bk.store[ic] = (1ull << 63) | (u64(sn) << 32) | u64(sB.base + u32(slot));
      }
    }
    const u64 pre0 = sh.snExtHighest;
    const u64 adjLast = extLast - sh.rmOpenValue;
    if (s.levelExt) {  // AudioLevel.Observe over the run's datagrams, in order (wave-uniform; lane 0 stores it)
      StreamHot lh;
      lh.flags = sh.flags;
      lh.latestTSForAudioLevel = sh.latestTSForAudioLevel;
      lh.lastObservedNs = sh.lastObservedNs;
      lh.observedDuration = sh.observedDuration;
      lh.activeDuration = sh.activeDuration;
      lh.loudest = sh.loudest;
      lh.smoothedLevel = sh.smoothedLevel;
      for (u32 x = pos; x < end; x++)
        level_step(lh, s, __builtin_amdgcn_readlane(u32(p.flags), x), __builtin_amdgcn_readlane(p.ts, x),
                   u8(__builtin_amdgcn_readlane(u32(p.level), x)), i64(rl_u64(u64(rp.arrival_ns), x)));
      __syncthreads();
      if (lane == 0) {
        sh.flags |= lh.flags & S_LVL_TS_INIT;
        sh.latestTSForAudioLevel = lh.latestTSForAudioLevel;
        sh.lastObservedNs = lh.lastObservedNs;
        sh.observedDuration = lh.observedDuration;
        sh.activeDuration = lh.activeDuration;
        sh.loudest = lh.loudest;
        sh.smoothedLevel = lh.smoothedLevel;
      }
    }
    __syncthreads();
    if (lane == 0) {  // the run's gaps cleared, then its SNs set
      hist_clear_range<1>(sHist, pre0 + 1, extLast);
      sh.packetsLost += extLast - pre0 - L;
      sh.bytes += bytesRun;
      sh.headerBytes += hdrRun;
      sh.frames += framesRun;
      sh.snHighest = snLast;
      sh.snExtHighest = extLast;
      sh.snCycles = extLast - snLast;
      sh.tsHighest = tsLast;
      sh.tsExtHighest = extTsLast;
      sh.tsCycles = extTsLast - tsLast;
      if (bkOn) {
        sB.head = u16(adjLast);
        sB.step = u32(bkt_wrap(int(sB.step) + int(bSLast), M));
      }
    }
    if (newTs) {
      const int kl = 63 - __clzll(static_cast<long long>(newTs));
      const i64 tl = i64(rl_u64(u64(rp.arrival_ns), u32(kl)));
      if (lane == 0) sh.highestTime = tl;
    }
    if (newJ) {  // (every lane runs the fold on uniform values; lane 0 stores it)
      StreamHot jh;
      jh.lastTransit = sh.lastTransit;
      jh.jitter = sh.jitter;
      jh.maxJitter = sh.maxJitter;
      jh.lastJitterExtTs = sh.lastJitterExtTs;
      for (u64 w = newJ; w; w &= w - 1) {
        const u32 k = u32(__ffsll(static_cast<long long>(w)) - 1);
        rx_jitter_fold(jh, rl_u64(transit, k), rl_u64(extTs, k));
      }
      if (lane == 0) {
        sh.lastTransit = jh.lastTransit;
        sh.jitter = jh.jitter;
        sh.maxJitter = jh.maxJitter;
        sh.lastJitterExtTs = jh.lastJitterExtTs;
      }
    }
    __syncthreads();
    if (run) atomicOr(reinterpret_cast<unsigned long long *>(&sHist[(ext >> 6) & (kHistWords - 1)]), 1ull << (ext & 63));
    __syncthreads();
    pos = end;
    }
    // (every stream writes its own, NACK queue or not: a list may hold another
    // stream's datagrams, which only that stream's wave writes)
    if (nackIn && useList && in && rp.stream == sid)
      nackIn[size_t(lst - list) + k] = NackIn{rp.arrival_ns, sid, nkSnFl, nkS0, nkLen};
  }
  if (sHist[lane] != hist0) hg[lane] = sHist[lane];
  const u32 hot1 = reinterpret_cast<const u32 *>(&sh)[lane];
  if (hot1 != hot0) reinterpret_cast<u32 *>(hot + sid)[lane] = hot1;
  if (bkOn && lane < 4) reinterpret_cast<u32 *>(bka.state + sid)[lane] = reinterpret_cast<const u32 *>(&sB)[lane];
  if (DDK) {
    __syncthreads();
    uint4 *g = reinterpret_cast<uint4 *>(ddStates + s.ddIdx);
    const uint4 *l = reinterpret_cast<const uint4 *>(sDDIRaw);
    for (u32 i = lane; i < sizeof(DDIngState) / 16; i += 64) g[i] = l[i];
  }
  }  // next stream of this wave
}

// ---------------------------------------------------------------------------
// k_ing_nack: the receive-side NACK queue (mediatransportutil nack.NackQueue,
// NackQueueParamsDefault) of every stream that has one, as buffer.Buffer
// drives it per datagram (buffer.go:417-421, :545-567, :673-710):
//   updateStreamState: Remove(header SN), then Push(uint16(lost)) for every
//                      lost SN of the flow's range  (the RTP header parsed)
//   deferred doNACKs:  Pairs() at now = the arrival time (every datagram)
// One wave per stream, serial over its datagrams (the queue is one
// recurrence); the queue lives in LDS with two entries per lane, so Remove,
// Push and the per-entry getNack decisions are ballots and a shifted copy.
// The pair packing of the sent entries (a chain over the sent SNs) runs on
// lane 0.  A datagram's result: info = n_pairs | num_nacked << 16 (0: no
// RTCP NACK) and the offset of its pairs in the batch's pair buffer.
// ---------------------------------------------------------------------------

// ---- the lane-parallel form (round 6) -----------------------------------
// Pairs() runs at every datagram of the stream, Remove() before it, Push()
// in between; so an entry's life depends only on the stream's arrival times
// and its own SN: it is nacked at the first datagram whose arrival is at
// least its lastNackedAt plus the interval its tries require, again from
// there, and it leaves at the datagram that carries its SN (Remove, before
// that datagram's Pairs) or at the first Pairs after its MaxTries-th nack
// (purge).  Entries interact only through the queue's capacity (the newest
// CacheSize kept on Push), through Remove's "first entry with that SN", and
// through the pair packing of one Pairs call (the entries nacked together, in
// queue order, against the queue's first entry).  When the capacity cannot be
// reached in this ingest (entries at the start plus every SN pushed <=
// CacheSize), the SNs are distinct and the arrivals do not go back in time,
// each entry's life is computed on its own lane (binary searches over the
// arrival times), the nacks of one datagram are gathered by a sort of
// (datagram, entry) events, and each such datagram's pairs are packed on a
// lane of their own.  Otherwise the serial form below runs.
#ifndef LKF_NACK_FAST_MIN  // fewest datagrams of a stream for the lane-parallel form
#define LKF_NACK_FAST_MIN 16
#endif
#ifndef LKF_NACK_N
#define LKF_NACK_N 512
#endif
constexpr u32 kNackFastN = LKF_NACK_N;  // datagrams of a stream the lane-parallel form stages (a 1-s video layer: ~300)
constexpr u32 kNackFastEv = kNackFastPairs;  // nack events: at most MaxTries per entry (the form takes <= 51 entries)
constexpr u32 kNackNone = 0xffffffffu;
constexpr u32 kNackHash = 256;
struct NackFastLds {
  i64 arr[kNackFastN];
  u16 sn[kNackFastN];
  u16 nextMine[kNackFastN + 1];
  u8 fl[kNackFastN];  // 1 mine, 2 updateStreamState ran, 4 a loss range
  // entries (queue order: the queue at the start, then every pushed SN in push order)
  i64 eLast[kNackSlots];
  u32 eRem[kNackSlots];
  u16 eDeath[kNackSlots];  // 0xffff: still queued
  int16_t eBirth[kNackSlots];  // the pushing datagram, -1: queued before the ingest
  u16 eSn[kNackSlots];
  u8 eTries[kNackSlots];
  u16 pushK[kNackCap], pushOff[kNackCap + 1];
  u16 pushS0[kNackCap];
  u16 key[kNackFastEv];  // nack events: datagram << 7 | entry (0xffff: none)
  u8 hash[256];          // entry by SN (kNackHash slots)
  u16 gStart[kNackFastEv + 1];
  u16 gNp[kNackFastEv], gOff[kNackFastEv];
  lkf_nack_pair stage[kNackFastEv];
  u32 nEv;
};
static_assert(kNackSlots <= 128 && kNackFastN <= 512 && kNackFastEv / kNackMaxTries < 127,
              "16-bit event keys: 9 bits of datagram, 7 of entry, below the 0xffff pad");

#ifndef LKF_NACK_DBG  // (diagnosis builds: print why a stream takes the serial form)
#define LKF_NACK_DBG 0
#endif
#define NF_DECLINE(code)                                                                                 \
  do {                                                                                                   \
    if (LKF_NACK_DBG == 1 && lane == 0) printf("nack serial sid=%u why=%d nIdx=%u count0=%u\n", sid, code, nIdx, count0); \
    return false;                                                                                        \
  } while (0)
#if LKF_NACK_DBG == 2  // per-wave phase stamps (wall clock, 100 MHz), read by lkf_debug_nack_stamps
constexpr u32 kNackStampCap = 1u << 16;
__device__ u64 gNackStamp[size_t(kNackStampCap) * 7];
#else
constexpr u32 kNackStampCap = 0;
__device__ u64 *const gNackStamp = nullptr;
#endif
// a wave's stamp record (lane 0; nullptr in production builds), its entry time stored
__device__ __forceinline__ u64 *nack_stamp(u32 lane, u32 sid, u64 tEntry) {
  if (LKF_NACK_DBG != 2 || sid >= kNackStampCap) return nullptr;
  u64 *r = gNackStamp + size_t(sid) * 7;  // (by stream: no shared counter to perturb the timing)
  if (lane == 0) r[1] = tEntry;
  return r;
}
__device__ bool nack_fast(NackFastLds &F, u32 lane, u32 sid, NackState *g, u32 count0, u32 rtt, u32 nIdx,
                          const u32 *lst, bool useList, u32 pb, const NackIn *__restrict__ nk,
                          const lkf_raw_pkt *__restrict__ raws, const IngParsed *__restrict__ q,
                          const lkf_flow *__restrict__ flows, u32 *__restrict__ info,
                          u32 *__restrict__ pairOff, u32 *pairCnt, lkf_nack_pair *__restrict__ pairs, u32 pairCap,
                          u32 *err, u64 *stamp) {
  // (LKF_NACK_DBG 2: the wave's phase stamps, stored as they are taken)
#define NF_STAMP(w)                                                    \
  do {                                                                 \
    if (LKF_NACK_DBG == 2 && lane == 0 && stamp) stamp[w] = wall_clock64(); \
  } while (0)
  // (a stream with a few datagrams: the serial form's per-datagram steps cost
  // less than this form's fixed phases — 10-ms ticks, 1-2 per stream: 92 vs
  // 203 us per ingest)
  if (nIdx < LKF_NACK_FAST_MIN || nIdx > kNackFastN || count0 * kNackMaxTries > kNackFastEv) NF_DECLINE(1);
  // the queue's entries (at most 51: one per lane), loaded beside the datagrams
  static_assert(kNackFastEv / kNackMaxTries <= 64, "one queued entry per lane");
  u32 q0sn = 0, q0tries = 0;
  i64 q0last = 0;
  if (lane < count0) {
    q0sn = g->sn[lane];
    q0tries = g->tries[lane];
    q0last = g->last[lane];
  }
  // ---- the stream's datagrams, and its pushes
  u64 lossTot = 0;
  u32 nPush = 0;
  bool mono = true;
  i64 prevArr = INT64_MIN;
  // every chunk's loads in flight together (a chunk at a time waited a round
  // trip per chunk): the stream kernel's NackIn records, contiguous in list
  // order, or (no records: a stream without a list) the datagram's index, then
  // its raw, parsed and flow entries
  constexpr u32 kCh = kNackFastN / 64;
  u32 stv[kCh], sfv[kCh];  // stream; SN | (2 parsed, 4 loss) << 16
  i64 arv[kCh];
  u64 s0v[kCh], lnv[kCh];
  if (nk) {
#pragma unroll
    for (u32 c = 0; c < kCh; c++) {
      const u32 k = c * 64 + lane;
      stv[c] = 0xffffffffu;
      arv[c] = 0;
      sfv[c] = 0;
      s0v[c] = lnv[c] = 0;
      if (k < nIdx) {
        const NackIn r = nk[k];
        stv[c] = r.stream;
        arv[c] = r.arrival;
        sfv[c] = r.snFl;
        s0v[c] = r.s0;
        lnv[c] = r.len;
      }
    }
  } else {
    u32 icv[kCh], ffv[kCh];
#pragma unroll
    for (u32 c = 0; c < kCh; c++) {
      const u32 k = c * 64 + lane;
      icv[c] = k < nIdx ? (useList ? lst[k] : pb + k) : 0u;
    }
#pragma unroll
    for (u32 c = 0; c < kCh; c++) {
      stv[c] = 0xffffffffu;
      arv[c] = 0;
      sfv[c] = 0;
      ffv[c] = 0;
      if (c * 64 + lane < nIdx) {
        stv[c] = raws[icv[c]].stream;
        arv[c] = raws[icv[c]].arrival_ns;
        const IngParsed &pq = q[icv[c]];
        sfv[c] = u32(pq.sn) | ((pq.flags & IP_OK) ? 2u << 16 : 0u);
        ffv[c] = flows[icv[c]].flags;
      }
    }
#pragma unroll
    for (u32 c = 0; c < kCh; c++) {  // the loss ranges (a loss datagram's flow), all chunks in flight
      s0v[c] = lnv[c] = 0;
      if (c * 64 + lane < nIdx && stv[c] == sid && (sfv[c] & (2u << 16)) && (ffv[c] & LKF_FLOW_HAS_LOSS)) {
        sfv[c] |= 4u << 16;
        const u64 ls = flows[icv[c]].loss_start;
        s0v[c] = u16(ls);
        lnv[c] = flows[icv[c]].loss_end - ls;
      }
    }
  }
#pragma unroll
  for (u32 c = 0; c < kCh; c++) {
    const u32 base = c * 64;
    if (base >= nIdx) break;
    const u32 k = base + lane;
    const bool v = k < nIdx;
    u32 flg = 0;
    u16 sn = 0;
    i64 arr = v ? arv[c] : prevArr;
    u64 L = 0, s0 = 0;
    if (v) {
      if (stv[c] == sid) {
        flg = 1;
        if (sfv[c] & (2u << 16)) {
          flg |= 2;
          sn = u16(sfv[c]);
          if (sfv[c] & (4u << 16)) {
            flg |= 4;
            s0 = s0v[c];
            L = lnv[c];
          }
        }
      }
      F.arr[k] = arr;
      F.sn[k] = sn;
      F.fl[k] = u8(flg);
    }
    const u64 prevLane = u64(__shfl_up(u64(arr), 1, 64));
    if (__ballot(v && arr < (lane ? i64(prevLane) : prevArr))) mono = false;
    prevArr = i64(rl_u64(u64(arr), 63));
    if (__ballot(L > u64(kNackCap) || ((flg & 4) && L == 0))) NF_DECLINE(2);
    const u64 lm = __ballot(flg & 4);
    const u32 before4 = u32(__popcll(lm & ((1ull << lane) - 1)));
    if ((flg & 4) && nPush + before4 < u32(kNackCap)) {
      F.pushK[nPush + before4] = u16(k);
      F.pushS0[nPush + before4] = u16(s0);
    }
    // the loss lengths in push order (a prefix over the chunk's loss datagrams)
    u64 Ls = wave_incl_scan_u64(L, lane);
    if ((flg & 4) && nPush + before4 < u32(kNackCap)) F.pushOff[nPush + before4 + 1] = u16(lossTot + Ls);
    lossTot += rl_u64(Ls, 63);
    nPush += u32(__popcll(lm));
    if (u64(count0) + lossTot > u64(kNackCap)) NF_DECLINE(3);  // the capacity could be reached
  }
  NF_STAMP(2);
  // no queued entry and no loss: the queue stays empty and nothing is nacked
  // (configs[2] has no loss: the rest of this form is fixed cost)
  if (count0 == 0 && lossTot == 0) return true;
  if (!mono) NF_DECLINE(4);
  const u32 M = count0 + u32(lossTot);
  if (M * kNackMaxTries > kNackFastEv) NF_DECLINE(5);  // (more entries than the event list holds nacks of)
  if (lane == 0) F.pushOff[0] = 0;
  __syncthreads();
  // ---- the entries
  if (lane < count0) {
    F.eSn[lane] = u16(q0sn);
    F.eTries[lane] = u8(q0tries);
    F.eLast[lane] = q0last;
    F.eBirth[lane] = -1;
  }
  for (u32 p = 0; p < nPush; p++) {
    const u32 o = F.pushOff[p], L = F.pushOff[p + 1] - o, k = F.pushK[p];
    const u16 s0 = F.pushS0[p];
    for (u32 i = lane; i < L; i += 64) {
      const u32 e = count0 + o + i;
      F.eSn[e] = u16(s0 + i);
      F.eTries[e] = 0;
      F.eLast[e] = F.arr[k];
      F.eBirth[e] = int16_t(k);
    }
  }
  for (u32 e = lane; e < M; e += 64) F.eRem[e] = kNackNone;
  // next datagram of the stream at or after k (Pairs runs there)
  if (lane == 0) F.nextMine[nIdx] = 0xffffu;
  for (i32 base = i32((nIdx - 1) & ~63u); base >= 0; base -= 64) {
    const u32 k = u32(base) + lane;
    const bool mine = k < nIdx && (F.fl[k] & 1);
    const u64 mm = __ballot(mine);
    const u64 ge = mm & ~((1ull << lane) - 1);
    const u32 after = (u32(base) + 64 < nIdx) ? u32(F.nextMine[u32(base) + 64]) : 0xffffu;
    __syncthreads();
    if (k < nIdx) F.nextMine[k] = ge ? u16(u32(base) + u32(__ffsll((long long)ge) - 1)) : u16(after);
    __syncthreads();
  }
  __syncthreads();
  // the entries by SN in an LDS hash (256 slots, linear probing: at most 51
  // entries); an SN already there means equal SNs, which Remove's "first
  // entry with that SN" leaves to the serial form
  for (u32 i = lane; i < kNackHash; i += 64) F.hash[i] = 0xffu;
  __syncthreads();
  bool dup = false;
  if (lane == 0)
    for (u32 e = 0; e < M && !dup; e++) {
      u32 h = (u32(F.eSn[e]) * 0x9E37u >> 8) & (kNackHash - 1);
      while (F.hash[h] != 0xffu && !dup) {
        dup = F.eSn[F.hash[h]] == F.eSn[e];
        h = (h + 1) & (kNackHash - 1);
      }
      F.hash[h] = u8(e);
    }
  if (__ballot(dup)) NF_DECLINE(6);
  __syncthreads();
  // Remove: the first datagram (from the entry's birth on) that carries its SN,
  // a probe of the hash per datagram and an LDS minimum per entry
  for (u32 base = 0; base < nIdx; base += 64) {
    const u32 k = base + lane;
    if (k < nIdx && (F.fl[k] & 2)) {
      const u16 sn = F.sn[k];
      for (u32 h = (u32(sn) * 0x9E37u >> 8) & (kNackHash - 1); F.hash[h] != 0xffu; h = (h + 1) & (kNackHash - 1)) {
        const u32 e = F.hash[h];
        if (F.eSn[e] == sn) {
          if (k >= u32(F.eBirth[e] + 1)) atomicMin(&F.eRem[e], k);
          break;
        }
      }
    }
  }
  __syncthreads();
  NF_STAMP(3);
  if (lane == 0) F.nEv = 0;
  __syncthreads();
  // ---- each entry's life
  auto backoff = [&](u64 num, u64 den) {
    i64 r = i64(num / den) * 1000000;
    if (r > 400000000) r = 400000000;
    return r < 20000000 ? i64(20000000) : r;
  };
  const i64 req0 = 20000000, req1 = backoff(rtt, 1), req2 = backoff(u64(rtt) * 5, 4),
            req3 = backoff(u64(rtt) * 25, 16), req4 = backoff(u64(rtt) * 125, 64);
  for (u32 e = lane; e < M; e += 64) {
    u32 t = F.eTries[e];
    i64 l = F.eLast[e];
    u32 k = u32(F.eBirth[e] + 1);
    const u32 rm = F.eRem[e];
    u32 death = kNackNone;
    for (;;) {
      u32 j;
      if (t >= kNackMaxTries) {
        j = k < nIdx ? u32(F.nextMine[k]) : 0xffffu;
        if (j == 0xffffu) j = kNackNone;
        if (rm != kNackNone && rm <= j) death = rm;
        else if (j != kNackNone) death = j + 1;  // purged by the Pairs there (still the queue's at it)
        break;
      }
      const i64 need = l + (t == 0 ? req0 : t == 1 ? req1 : t == 2 ? req2 : t == 3 ? req3 : req4);
      u32 lo = k, hi = nIdx;  // first datagram at or after k arriving at or after need
      while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (F.arr[mid] >= need) hi = mid;
        else lo = mid + 1;
      }
      j = lo < nIdx ? u32(F.nextMine[lo]) : 0xffffu;
      if (j == 0xffffu) j = kNackNone;
      if (rm != kNackNone && rm <= j) {
        death = rm;
        break;
      }
      if (j == kNackNone) break;
      const u32 slot = atomicAdd(&F.nEv, 1u);
      if (slot < kNackFastEv) F.key[slot] = u16((j << 7) | e);
      t++;
      l = F.arr[j];
      k = j + 1;
    }
    F.eTries[e] = u8(t);
    F.eLast[e] = l;
    F.eDeath[e] = u16(death == kNackNone ? 0xffffu : death);
  }
  __syncthreads();
  const u32 E = F.nEv;
  if (E > kNackFastEv) {  // (cannot happen: at most MaxTries nacks per entry, M * MaxTries <= kNackFastEv)
    if (lane == 0) atomicOr(err, 8u);
    return true;
  }
  // ---- the events in (datagram, queue) order: a bitonic sort in LDS
  u32 P = 1;
  while (P < E) P <<= 1;
  for (u32 i = E + lane; i < P; i += 64) F.key[i] = 0xffffu;
  __syncthreads();
  for (u32 size = 2; size <= P; size <<= 1)
    for (u32 stride = size >> 1; stride > 0; stride >>= 1) {
      for (u32 i = lane; i < P; i += 64) {
        const u32 jx = i ^ stride;
        if (jx > i) {
          const u32 a = F.key[i], b = F.key[jx];
          const bool up = (i & size) == 0;
          if ((a > b) == up) {
            F.key[i] = u16(b);
            F.key[jx] = u16(a);
          }
        }
      }
      __syncthreads();
    }
  NF_STAMP(4);
  // ---- one group per nacking datagram: its pairs (NackQueue.Pairs), packed on a lane
  u32 G = 0;
  for (u32 base = 0; base < E; base += 64) {
    const u32 i = base + lane;
    const bool st = i < E && (i == 0 || (F.key[i] >> 7) != (F.key[i - 1] >> 7));
    const u64 m = __ballot(st);
    if (st) F.gStart[G + u32(__popcll(m & ((1ull << lane) - 1)))] = u16(i);
    G += u32(__popcll(m));
  }
  if (lane == 0) F.gStart[G] = u16(E);
  __syncthreads();
  u64 nacked = 0;
  for (u32 gi = lane; gi < G; gi += 64) {
    const u32 b = F.gStart[gi], en = F.gStart[gi + 1];
    const u32 j = F.key[b] >> 7;
    u32 first = 0;  // the queue's first entry at the Pairs of datagram j
    for (u32 e = 0; e < M; e++)
      if (F.eBirth[e] <= i32(j) && j < u32(F.eDeath[e])) {
        first = F.eSn[e];
        break;
      }
    u32 baseSN = u32(u16(first - 17u));
    bool active = false;
    lkf_nack_pair cur = {0, 0};
    u32 np = 0;
    for (u32 i = b; i < en; i++) {
      const u32 sn16 = F.eSn[F.key[i] & 127u];
      const u32 d = u32(u16(sn16 - baseSN));
      if (d > 16) {
        if (active) F.stage[b + np++] = cur;
        baseSN = sn16;
        cur.packet_id = u16(sn16);
        cur.lost_packets = 0;
        active = true;
      } else {
        const u32 sh = u32(u16(d - 1));
        if (sh < 16) cur.lost_packets = u16(cur.lost_packets | (1u << sh));
      }
    }
    if (active) F.stage[b + np++] = cur;
    F.gNp[gi] = u16(np);
    nacked += np ? u64(en - b) : 0ull;  // (UpdateNack only with a packet)
  }
  nacked = wave_sum_u64(nacked);
  __syncthreads();
  // pair offsets (a prefix over the groups), one reservation for the stream
  u32 tot = 0;
  for (u32 base = 0; base < G; base += 64) {
    const u32 gi = base + lane;
    const u64 np = gi < G ? F.gNp[gi] : 0;
    const u64 inc = wave_incl_scan_u64(np, lane);
    if (gi < G) F.gOff[gi] = u16(tot + u32(inc - np));
    tot += u32(rl_u64(inc, 63));
  }
  __syncthreads();
  // (the stream's own block of kNackFastPairs past the shared buffer: a pair
  // covers at least one event, so tot <= E <= kNackFastEv.  One counter
  // reserved by every stream serialised ~4000 returning atomics on one address)
  if (tot) {
    const u32 off = pairCap + sid * kNackFastPairs;
    for (u32 gi = lane; gi < G; gi += 64) {
      const u32 b = F.gStart[gi], np = F.gNp[gi], o = off + F.gOff[gi];
      for (u32 i = 0; i < np; i++) pairs[o + i] = F.stage[b + i];
      if (np) {
        const u32 kk = F.key[b] >> 7;
        const u32 icx = useList ? lst[kk] : pb + kk;
        info[icx] = np | ((F.gStart[gi + 1] - b) << 16);
        pairOff[icx] = o;
      }
    }
  }
  // ---- the queue after the ingest: the entries still in it, in order
  bool changed = M != count0 || E > 0;
  u32 kept = 0;
  for (u32 base = 0; base < M; base += 64) {
    const u32 e = base + lane;
    const bool live = e < M && F.eDeath[e] == 0xffffu;
    changed = changed || (e < M && !live);
    const u64 m = __ballot(live);
    const u32 at = kept + u32(__popcll(m & ((1ull << lane) - 1)));
    i64 l = 0;
    u16 sn = 0;
    u8 t = 0;
    if (live) {
      l = F.eLast[e];
      sn = F.eSn[e];
      t = F.eTries[e];
    }
    __syncthreads();
    if (live) {  // (entries move only toward the front: e >= at)
      F.eLast[at] = l;
      F.eSn[at] = sn;
      F.eTries[at] = t;
    }
    __syncthreads();
    kept += u32(__popcll(m));
  }
  if (__ballot(changed)) {
    for (u32 i = lane; i < kept; i += 64) {
      g->last[i] = F.eLast[i];
      g->sn[i] = F.eSn[i];
      g->tries[i] = F.eTries[i];
    }
    if (lane == 0) g->count = kept;
  }
  if (lane == 0 && nacked) g->nacks += nacked;
  NF_STAMP(5);
  if (LKF_NACK_DBG == 2 && lane == 0 && stamp) {
    stamp[0] = u64(sid) | (u64(nIdx) << 32);
    stamp[6] = u64(M) | (u64(E) << 32);
  }
  return true;
}

#ifndef LKF_NACK_FAST  // the lane-parallel form where it is exact (1), or always the serial one (0)
#define LKF_NACK_FAST 1
#endif
#ifndef LKF_NACK_LIVE  // stage only the live entries (1), or all slots with the count (0, round 4)
#define LKF_NACK_LIVE 1
#endif
// FAST: the lane-parallel form first (its 13 KB of LDS hold 12 workgroups per
// CU); the serial-only instantiation (5 KB) is launched for short ingests,
// where every stream takes the serial form anyway (LKF_NACK_FAST_MIN) and
// occupancy is what counts (10-ms ticks at 1,000 rooms: 40,000 streams).
template <bool FAST>
__global__ void __launch_bounds__(64) k_ing_nack(const lkf_raw_pkt *__restrict__ raws,
                                                 const IngParsed *__restrict__ q, const lkf_flow *__restrict__ flows,
                                                 const DevStream *__restrict__ streams, NackState *__restrict__ states,
                                                 StreamHot *__restrict__ hot, const u32 *__restrict__ tBegin,
                                                 const u32 *__restrict__ tEnd, const u32 *__restrict__ list,
                                                 const u32 *__restrict__ cnt, u32 stride, u32 *__restrict__ info,
                                                 u32 *__restrict__ pairOff, u32 *pairCnt,
                                                 lkf_nack_pair *__restrict__ pairs, u32 pairCap, u32 *err,
                                                 const NackIn *__restrict__ nackIn) {
  // the stream's RTCP NACKs of this ingest, staged and written in blocks: one
  // reservation in the batch's pair buffer per block instead of one atomic per
  // NACK (every stream's NACKs on one counter serialised the kernel)
  constexpr u32 kPairStage = 512, kRecStage = 64;
  struct Serial {
    i64 last[kNackSlots];
    u32 sn[kNackSlots], tries[kNackSlots], purge[kNackSlots];
    lkf_nack_pair stage[kPairStage];
    u32 recIc[kRecStage], recInfo[kRecStage], recOff[kRecStage];
  };
  // (the lane-parallel form and the serial one share the LDS: the serial form
  // runs only when the other declined, before it wrote anything but LDS)
  union U {
    NackFastLds f;
    Serial s;
  };
  __shared__ __attribute__((aligned(16))) u8 sRaw[FAST ? sizeof(U) : sizeof(Serial)];
  Serial &sS = *reinterpret_cast<Serial *>(sRaw);
  i64 *const sLast = sS.last;
  u32 *const sSn = sS.sn;
  u32 *const sTries = sS.tries;
  u32 *const sPurge = sS.purge;
  lkf_nack_pair *const sStage = sS.stage;
  u32 *const sRecIc = sS.recIc, *const sRecInfo = sS.recInfo, *const sRecOff = sS.recOff;
  const u64 tEntry = LKF_NACK_DBG == 2 ? wall_clock64() : 0;  // (diagnosis builds)
  const u32 sid = blockIdx.x, lane = threadIdx.x;
  const DevStream s = streams[sid];
  if (!s.nack || s.closed) return;
  const u32 pb = tBegin[s.track], pe = tEnd[s.track];
  if (pb >= pe) return;  // no datagram of its track: no calc, no doNACKs
  NackState *const g = states + sid;
  // only the live entries are staged (every read below is of an index < count)
  u32 count = g->count;
  const u32 rtt = g->rtt;
  const bool useList = s.layer < 3;
  const u32 nIdx = useList ? cnt[s.track * 3 + s.layer] : pe - pb;
  const u32 *lst = list + size_t(useList ? s.layer : 0) * stride + pb;
  const NackIn *nk = useList && nackIn ? nackIn + size_t(s.layer) * stride + pb : nullptr;
  if (FAST && LKF_NACK_FAST && nack_fast(*reinterpret_cast<NackFastLds *>(sRaw), lane, sid, g, count, rtt, nIdx, lst, useList, pb, nk, raws, q, flows, info,
                                 pairOff, pairCnt, pairs, pairCap, err, nack_stamp(lane, sid, tEntry)))
    return;
  __syncthreads();
  for (u32 i = lane; i < (LKF_NACK_LIVE ? count : u32(kNackSlots)); i += 64) {
    sLast[i] = g->last[i];
    sSn[i] = g->sn[i];
    sTries[i] = g->tries[i];
  }
  bool dirty = false;  // wave-uniform: an entry moved, was pushed or was nacked
  __syncthreads();
  // getNack's required interval per tries value (tries < MaxTries):
  // tries 0: MinInterval; else min(MaxInterval, floor(rtt * 1.25^(tries-1)) ms),
  // at least MinInterval (rtt * 1.25^k is exact in float64 for k <= 3)
  static_assert(kNackMaxTries == 5, "one required interval per tries value 0..4");
  auto backoff = [&](u64 num, u64 den) {
    i64 r = i64(num / den) * 1000000;
    if (r > 400000000) r = 400000000;
    return r < 20000000 ? i64(20000000) : r;
  };
  const i64 req0 = 20000000, req1 = backoff(rtt, 1), req2 = backoff(u64(rtt) * 5, 4),
            req3 = backoff(u64(rtt) * 25, 16), req4 = backoff(u64(rtt) * 125, 64);
  // entry idx < count moves down one slot from index k on (NackQueue.Remove)
  auto removeAt = [&](u32 k) {
    i64 l[2];
    u32 sn[2], tr[2];
    bool mv[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const u32 idx = lane + 64u * u32(h);
      mv[h] = idx >= k && idx + 1 < count;
      if (mv[h]) {
        l[h] = sLast[idx + 1];
        sn[h] = sSn[idx + 1];
        tr[h] = sTries[idx + 1];
      }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const u32 idx = lane + 64u * u32(h);
      if (mv[h]) {
        sLast[idx] = l[h];
        sSn[idx] = sn[h];
        sTries[idx] = tr[h];
      }
    }
    __syncthreads();
    count--;
    dirty = true;
  };
  auto removeSn = [&](u32 sn16) {  // the first entry with that SN
    const u64 m0 = __ballot(lane < count && sSn[lane] == sn16);
    const u64 m1 = __ballot(lane + 64 < count && sSn[lane + 64] == sn16);
    if (m0 | m1) removeAt(m0 ? u32(__ffsll((long long)m0) - 1) : 64u + u32(__ffsll((long long)m1) - 1));
  };
  u64 nacked = 0;
  // The earliest arrival time at which Pairs() can do anything: min over the
  // entries of lastNackedAt + the interval its tries require (an entry at
  // MaxTries is purged by the next call: -inf).  Before it, Pairs() sends and
  // purges nothing, so a datagram that arrives earlier skips it (exactly the
  // reference's outcome: no entry due, no RTCP NACK).  Pushes lower it; after
  // a Pairs() that changed entries it is recomputed; removals leave a bound
  // that is at most early (a skipped call is then only not skipped).
  auto reqOf = [&](u32 t) { return t == 0 ? req0 : t == 1 ? req1 : t == 2 ? req2 : t == 3 ? req3 : req4; };
  auto dueMin = [&]() -> i64 {
    i64 m = INT64_MAX;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const u32 idx = lane + 64u * u32(h);
      if (idx < count) {
        const u32 t = sTries[idx];
        const i64 d = t >= kNackMaxTries ? INT64_MIN : sLast[idx] + reqOf(t);
        m = d < m ? d : m;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const i64 x = i64((u64(u32(__shfl_xor(int(u32(u64(m) >> 32)), o, 64))) << 32) |
                        u64(u32(__shfl_xor(int(u32(u64(m))), o, 64))));
      m = x < m ? x : m;
    }
    return i64(rl_u64(u64(m), 0));
  };
  i64 nextDue = count ? dueMin() : INT64_MAX;
  u32 stageN = 0, recN = 0;  // wave-uniform
  auto flush = [&]() {
    __syncthreads();  // (lane 0's staged pairs and records)
    if (stageN) {
      u32 off = 0;
      if (lane == 0) off = atomicAdd(pairCnt, stageN);
      off = __builtin_amdgcn_readfirstlane(off);
      if (off + stageN > pairCap) {
        if (lane == 0) atomicOr(err, 8u);  // pair buffer capacity: these RTCP NACKs are not recorded
      } else {
        for (u32 i = lane; i < stageN; i += 64) pairs[off + i] = sStage[i];
        if (lane < recN) {
          info[sRecIc[lane]] = sRecInfo[lane];
          pairOff[sRecIc[lane]] = off + sRecOff[lane];
        }
      }
    }
    __syncthreads();
    stageN = recN = 0;
  };
  for (u32 base = 0; base < nIdx; base += 64) {
    const u32 k = base + lane;
    u32 ic = 0, stm = 0xffffffffu, ipf = 0, sn = 0, ff = 0;
    i64 arr = 0;
    u64 ls = 0, le = 0;
    if (k < nIdx) {
      ic = useList ? lst[k] : pb + k;
      const lkf_raw_pkt rp = raws[ic];
      stm = rp.stream;
      arr = rp.arrival_ns;
      ipf = q[ic].flags;
      sn = q[ic].sn;
      const lkf_flow f = flows[ic];
      ff = f.flags;
      ls = f.loss_start;
      le = f.loss_end;
    }
    // Only some datagrams can act on the queue: one whose SN may be in it
    // (the chunk-start entries, or a range an earlier datagram of the chunk
    // pushes — Remove), one with a loss range (Push), and the first one at or
    // past nextDue (Pairs).  The others are skipped: Remove finds nothing and
    // Pairs sends and purges nothing, as in the reference.
    const bool mine = k < nIdx && stm == sid;
    const bool upd = mine && (ipf & IP_OK);
    const bool lossL = upd && (ff & LKF_FLOW_HAS_LOSS);
    bool hit = false;
    if (upd) {
      for (u32 i = 0; i < count; i++) hit = hit || sSn[i] == u32(u16(sn));
    }
    for (u64 lm = __ballot(lossL); lm; lm &= lm - 1) {  // SNs the chunk's earlier datagrams push
      const u32 a = u32(__ffsll((long long)lm) - 1);
      const u64 s0 = rl_u64(ls, a), e0 = rl_u64(le, a);
      hit = hit || (lane > a && u64(u16(u16(sn) - u16(s0))) < e0 - s0);
    }
    const u64 evM = __ballot(upd && (hit || lossL));
    const u64 mineM = __ballot(mine);
    for (u32 pos = 0; pos < 64;) {
      const u64 after = ~((1ull << pos) - 1);
      const u64 dueM = count ? (__ballot(mine && arr >= nextDue) & mineM) : 0ull;
      const u64 nx = (evM | dueM) & after;
      if (!nx) break;
      const u32 x = u32(__ffsll((long long)nx) - 1);
      pos = x + 1;
      const i64 now = i64(rl_u64(u64(arr), x));
      const u32 icx = __builtin_amdgcn_readlane(ic, x);
      if (__builtin_amdgcn_readlane(ipf, x) & IP_OK) {  // updateStreamState ran
        removeSn(__builtin_amdgcn_readlane(sn, x));
        if (__builtin_amdgcn_readlane(ff, x) & LKF_FLOW_HAS_LOSS) {
          const u64 s0 = rl_u64(ls, x), e0 = rl_u64(le, x);
          // Push each lost SN: the queue keeps the newest CacheSize entries of
          // (queue, lost SNs in order); every new one has tries 0, lastNackedAt now
          const u64 L = e0 - s0;
          const u64 total = u64(count) + L;
          const u32 drop = total > u64(kNackCap) ? u32(min(total - u64(kNackCap), u64(count))) : 0u;
          const u32 newCount = total > u64(kNackCap) ? u32(kNackCap) : u32(total);
          const u64 first = L > u64(kNackCap) ? e0 - u64(kNackCap) : s0;  // first new SN kept
          const u32 keptOld = count - drop;
          i64 l[2];
          u32 sv[2], tv[2];
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const u32 idx = lane + 64u * u32(h);
            if (idx < newCount) {
              if (idx < keptOld) {
                l[h] = sLast[idx + drop];
                sv[h] = sSn[idx + drop];
                tv[h] = sTries[idx + drop];
              } else {
                l[h] = now;
                sv[h] = u32(u16(first + (idx - keptOld)));
                tv[h] = 0;
              }
            }
          }
          __syncthreads();
#pragma unroll
          for (int h = 0; h < 2; h++) {
            const u32 idx = lane + 64u * u32(h);
            if (idx < newCount) {
              sLast[idx] = l[h];
              sSn[idx] = sv[h];
              sTries[idx] = tv[h];
            }
          }
          __syncthreads();
          count = newCount;
          dirty = true;
          nextDue = now + req0 < nextDue ? now + req0 : nextDue;  // the new entries (tries 0, lastNackedAt now)
        }
      }
      if (count == 0 || now < nextDue) continue;
      // ---- Pairs(now): getNack of every entry, in parallel
      bool rem[2], snd[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const u32 idx = lane + 64u * u32(h);
        rem[h] = snd[h] = false;
        if (idx < count) {
          const u32 t = sTries[idx];
          rem[h] = t >= kNackMaxTries;
          const i64 rq = t == 0 ? req0 : t == 1 ? req1 : t == 2 ? req2 : t == 3 ? req3 : req4;
          snd[h] = !rem[h] && now - sLast[idx] >= rq;
        }
      }
      const u64 r0 = __ballot(rem[0]), r1 = __ballot(rem[1]);
      const u64 s0m = __ballot(snd[0]), s1m = __ballot(snd[1]);
      if (!(r0 | r1 | s0m | s1m)) {
        nextDue = dueMin();  // (a removal left the bound early)
        continue;
      }
      const u32 base16 = u32(u16(sSn[0] - 17u));  // set far back to open the first pair
      // purge list (queue order), before any entry moves
      const u32 nr0 = u32(__popcll(r0));
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const u64 mm = h ? r1 : r0;
        if (rem[h]) sPurge[(h ? nr0 : 0u) + u32(__popcll(mm & ((1ull << lane) - 1)))] = sSn[lane + 64u * u32(h)];
      }
#pragma unroll
      for (int h = 0; h < 2; h++)
        if (snd[h]) {
          const u32 idx = lane + 64u * u32(h);
          sTries[idx] = sTries[idx] + 1;
          sLast[idx] = now;
        }
      __syncthreads();
      const u32 numNacked = u32(__popcll(s0m) + __popcll(s1m));
      dirty = true;
      if (numNacked && (stageN + u32(kNackCap) > kPairStage || recN == kRecStage)) flush();
      lkf_nack_pair *const sPairs = sStage + stageN;
      u32 np = 0;
      if (lane == 0 && numNacked) {  // pair packing (NackQueue.Pairs), in queue order
        u32 baseSN = base16;
        bool active = false;
        lkf_nack_pair cur = {0, 0};
        for (int h = 0; h < 2; h++)
          for (u64 mm = h ? s1m : s0m; mm; mm &= mm - 1) {
            const u32 sn16 = sSn[u32(__ffsll((long long)mm) - 1) + 64u * u32(h)];
            const u32 d = u32(u16(sn16 - baseSN));
            if (d > 16) {
              if (active) sPairs[np++] = cur;
              baseSN = sn16;
              cur.packet_id = u16(sn16);
              cur.lost_packets = 0;
              active = true;
            } else {
              const u32 sh = u32(u16(d - 1));
              if (sh < 16) cur.lost_packets = u16(cur.lost_packets | (1u << sh));
            }
          }
        if (active) sPairs[np++] = cur;
        if (np) {
          sRecIc[recN] = icx;
          sRecInfo[recN] = np | (numNacked << 16);
          sRecOff[recN] = stageN;
        }
      }
      np = __builtin_amdgcn_readfirstlane(np);
      if (np) {
        stageN += np;
        recN++;
      }
      if (numNacked && np) nacked += numNacked;  // UpdateNack only with a packet
      // purge (NackQueue.Remove of every entry at MaxTries, in order)
      const u32 nPurge = nr0 + u32(__popcll(r1));
      for (u32 i = 0; i < nPurge; i++) removeSn(sPurge[i]);
      __syncthreads();
      nextDue = count ? dueMin() : INT64_MAX;
    }
  }
  flush();
  if (dirty) {  // (entries past count are never read: only the live ones go back)
    for (u32 i = lane; i < count; i += 64) {
      g->last[i] = sLast[i];
      g->sn[i] = u16(sSn[i]);
      g->tries[i] = u8(sTries[i]);
    }
    if (lane == 0) g->count = count;
  }
  if (lane == 0 && nacked) g->nacks += nacked;
}

// lkf_ingest_nacks: records at their compacted positions, pairs gathered in
// record order
__global__ void k_nack_compact(u32 n, const lkf_raw_pkt *__restrict__ raws, const DevStream *__restrict__ streams,
                               const u32 *__restrict__ info, const u32 *__restrict__ pairOff,
                               const lkf_nack_pair *__restrict__ pairs, const u64 *__restrict__ recPos,
                               const u64 *__restrict__ pairPos, lkf_rtcp_nack *__restrict__ outRecs,
                               lkf_nack_pair *__restrict__ outPairs) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !info[i]) return;
  const u32 np = info[i] & 0xffffu;
  lkf_rtcp_nack r = {};
  r.datagram = i;
  r.stream = raws[i].stream;
  r.media_ssrc = streams[r.stream].ssrc;
  r.pair_off = u32(pairPos[i]);
  r.n_pairs = u16(np);
  r.num_nacked = u16(info[i] >> 16);
  outRecs[recPos[i]] = r;
  for (u32 k = 0; k < np; k++) outPairs[pairPos[i] + k] = pairs[pairOff[i] + k];
}

// ---------------------------------------------------------------------------
// k_ing_out: the ExtPacket of every forwarded datagram at its batch position
// ---------------------------------------------------------------------------
// FwdPrep: the forwarding context's per-batch preparation folded in (one
// dispatch instead of k_batch_init + k_track_ranges on the prep chain).
struct FwdPrep {
  u32 *tBegin, *tEnd, *err, *fwdCnt;
  u64 *stats, *fwdBytes;
  u32 nstats, ndts, ntracks;
  const u32 *rawBegin, *rawEnd;  // the ingest's per-track datagram ranges (grouped by track)
  const u64 *total;              // ExtPackets of the ingest
};
__global__ void k_ing_out(const lkf_raw_pkt *__restrict__ raws, const IngParsed *__restrict__ q,
                          const DevStream *__restrict__ streams, const u32 *__restrict__ fwd,
                          const u64 *__restrict__ pos, u32 n, lkf_flow *__restrict__ flows,
                          lkf_pkt *__restrict__ out, const IngDD *__restrict__ ingDD, lkf_pkt_dd *__restrict__ outDD,
                          FwdPrep fp) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (fp.tBegin) {
    // track t's ExtPackets are [pos[rawBegin], pos[rawEnd]) (the ingest writes
    // them in datagram order, datagrams grouped by track); an empty track
    // [0, 0) as k_track_ranges leaves it.  The counters start at zero.
    const u32 stride = gridDim.x * blockDim.x;
    for (u32 j = i; j < fp.ntracks || j < fp.ndts || j < fp.nstats || j < 4; j += stride) {
      if (j < fp.ntracks) {
        const u32 rb = fp.rawBegin[j], re = fp.rawEnd[j];
        u32 b = 0, e = 0;
        if (re > rb) {
          b = u32(pos[rb]);
          e = re < n ? u32(pos[re]) : u32(*fp.total);
        }
        fp.tBegin[j] = b < e ? b : 0u;
        fp.tEnd[j] = b < e ? e : 0u;
      }
      if (j < fp.ndts) {
        fp.fwdCnt[j] = 0;
        fp.fwdBytes[j] = 0;
      }
      if (j < fp.nstats) fp.stats[j] = 0;
      if (j < 4) fp.err[j] = 0;
    }
  }
  if (i >= n || !fwd[i]) return;
  const u32 k = u32(pos[i]);
  const IngParsed p = q[i];
  const lkf_raw_pkt rp = raws[i];
  const DevStream s = streams[rp.stream];
  flows[i].pkt = k;
  lkf_pkt e = {};
  e.ext_sn = flows[i].ext_sn;
  e.ext_ts = flows[i].ext_ts;
  e.arrival_ns = rp.arrival_ns;
  e.arena_off = rp.off;
  e.track = s.track;
  e.ssrc = p.ssrc;
  e.payload_off = p.hdrSize;
  e.payload_len = p.payloadLen;
  e.hdr0 = p.b0;
  e.hdr1 = p.b1;
  e.spatial = -1;
  e.temporal = p.payloadLen > 0 ? 0 : -1;
  e.layer = int8_t(s.layer);
  if (p.flags & IP_LEVEL) {
    e.flags |= LKF_PKT_HAS_LEVEL;
    e.audio_level = p.level;
  }
  if (p.flags & IP_VP8) {
    e.flags |= LKF_PKT_VP8 | ((p.flags & IP_KF) ? LKF_PKT_KEYFRAME : 0);
    e.temporal = int8_t(p.tid);
    e.vp8_first = p.vfirst;
    e.vp8_bits = p.vbits;
    e.vp8_hdr_size = p.vhs;
    e.vp8_picture_id = p.pid;
    e.vp8_tl0picidx = p.tl0;
    e.vp8_tid = p.tid;
    e.vp8_keyidx = p.keyidx;
  }
  const IngDD dv = ingDD ? ingDD[i] : IngDD{};
  if (dv.present) {  // ExtPacket.DependencyDescriptor + VideoLayer (buffer.go:613-621)
    e.flags |= LKF_PKT_DD;
    e.spatial = int8_t(dv.sid);
    e.temporal = int8_t(dv.tid);
    if (p.flags & IP_VP8) {  // VP8 with DD: TID from the descriptor, no spatial (buffer.go:630-635)
      e.temporal = int8_t(dv.tid);
      e.vp8_tid = dv.tid;
      e.spatial = -1;
    }
  }
  if (p.flags & IP_VP9) {
    if (!dv.present) {  // VideoLayer{SID, TID}, Payload = VP9Packet (buffer.go:645-655)
      e.flags |= LKF_PKT_VP9;
      e.spatial = int8_t(p.sid);
      e.temporal = int8_t(p.tid);
      e.vp9_bits = p.vp9bits;
    }
  }
  if ((s.codec == LKF_CODEC_VP9 || s.codec == LKF_CODEC_H264 || s.codec == LKF_CODEC_AV1) && (p.flags & IP_KF))
    e.flags |= LKF_PKT_KEYFRAME;  // IsVP9KeyFrame / IsH264KeyFrame / IsAV1KeyFrame (buffer.go:656-660)
  if (e.spatial >= 0) e.layer = e.spatial;  // svc packet: forwardRTP dispatches pkt.Spatial (receiver.go:667-672)
  out[k] = e;
  if (outDD) {
    lkf_pkt_dd d = {};
    if (dv.present) {
      d.ext_frame_num = dv.extFN;
      d.ext_key_frame_num = dv.extKFN;
      d.dd_off = dv.ddOff;
      d.dd_len = dv.ddLen;
      d.flags = dv.flags;
    }
    outDD[k] = d;
  }
}

// ---------------------------------------------------------------------------
// k_rtx: the retransmission of one NACKed record (downtrack.go:1640-1698), one
// workgroup per record.  Lane 0 reads the source packet's layout (pion
// Packet.Unmarshal; VP8 descriptor for the re-munge) and the RTX header
// (marker/SN/TS from the sequencer, DownTrack SSRC/PT, source CSRCs, the
// pacer's extension block: abs-send-time placeholder) into LDS; SIZE pass:
// lens[i] (0 = skipped); WRITE pass: all lanes write the bytes at offs[i].
// ---------------------------------------------------------------------------
template <bool WRITE>
__global__ void __launch_bounds__(64) k_rtx(const lkf_rtx *__restrict__ rtx, const lkf_raw_pkt *__restrict__ src,
                                            const u8 *__restrict__ arena, const DevDT *__restrict__ dts,
                                            const DevTrack *__restrict__ tracks, u32 *__restrict__ lens,
                                            const u64 *__restrict__ offs, u8 *__restrict__ out,
                                            const u8 *__restrict__ dd) {
  __shared__ u8 pre[12 + 60 + 4 + 2 + kDDMaxBytes + 5 + 3 + 8 + 4];
  __shared__ u32 sPre, sLen, sPay;
  const u32 i = blockIdx.x, lane = threadIdx.x;
  if (lane == 0) {
    u32 total = 0;
    const lkf_raw_pkt rp = src[i];
    const lkf_rtx x = rtx[i];
    const DevDT dt = dts[x.dt];
    IngParsed q = {};
    int lo = -1;
    const u8 *b = arena + rp.off;
    if (rp.len && rtp_parse(b, int(rp.len), 0, 0, q, lo)) {
      u32 pay = q.hdrSize, payLen = q.payloadLen;
      bool ok = true;
      int n = 0;
      const int cc = q.b0 & 0xf;
      pre[n++] = u8((q.b0 & 0xe0) | ((dt.extAbs || dt.extTcc) ? 0x10 : 0) | cc);
      pre[n++] = u8((x.meta.marker ? 0x80 : 0) | (dt.pt & 0x7f));
      pre[n++] = u8(x.meta.target_sn >> 8);
      pre[n++] = u8(x.meta.target_sn);
      for (int k = 3; k >= 0; k--) pre[n++] = u8(x.meta.timestamp >> (8 * k));
      for (int k = 3; k >= 0; k--) pre[n++] = u8(dt.ssrc >> (8 * k));
      for (int k = 0; k < 4 * cc; k++) pre[n++] = b[12 + k];
      // the pacer's extension block (pacer/base.go:71-100): the sequencer's
      // ddBytes under the DownTrack's DD extension id (downtrack.go:1684; ID 0
      // or no bytes: skipped), then abs-send-time, then the TWCC interceptor's
      // transport-cc element (0 here, stamped in send order by k_twcc_stamp);
      // pion's one-byte profile, or the two-byte profile for a DD above 16 B
      const u32 ddLen = (dd && dt.extDD) ? dd[size_t(i) * kSeqDDBytes] : 0u;
      const u8 *ddB = ddLen ? dd + size_t(i) * kSeqDDBytes + 1 : nullptr;
      if (ddLen > 16) {
        const int eb = 2 + int(ddLen) + (dt.extAbs ? 5 : 0) + (dt.extTcc ? 4 : 0);
        const int words = (eb + 3) >> 2;
        pre[0] |= 0x10;
        pre[n++] = 0x10;
        pre[n++] = 0x00;
        pre[n++] = u8(words >> 8);
        pre[n++] = u8(words);
        pre[n++] = dt.extDD;
        pre[n++] = u8(ddLen);
        for (u32 k = 0; k < ddLen; k++) pre[n++] = ddB[k];
        if (dt.extAbs) {
          pre[n++] = dt.extAbs;
          pre[n++] = 3;
          pre[n++] = 0;
          pre[n++] = 0;
          pre[n++] = 0;
        }
        if (dt.extTcc) {
          pre[n++] = dt.extTcc;
          pre[n++] = 2;
          pre[n++] = 0;
          pre[n++] = 0;
        }
        for (int k = eb; k < 4 * words; k++) pre[n++] = 0;
      } else if (ddLen || dt.extAbs || dt.extTcc) {
        const int eb = (ddLen ? 1 + int(ddLen) : 0) + (dt.extAbs ? 4 : 0) + (dt.extTcc ? 3 : 0);
        const int words = (eb + 3) >> 2;
        pre[0] |= 0x10;
        pre[n++] = 0xBE;
        pre[n++] = 0xDE;
        pre[n++] = u8(words >> 8);
        pre[n++] = u8(words);
        if (ddLen) {
          pre[n++] = u8((dt.extDD << 4) | (ddLen - 1));
          for (u32 k = 0; k < ddLen; k++) pre[n++] = ddB[k];
        }
        if (dt.extAbs) {
          pre[n++] = u8((dt.extAbs << 4) | 2);
          pre[n++] = 0;
          pre[n++] = 0;
          pre[n++] = 0;
        }
        if (dt.extTcc) {
          pre[n++] = u8((dt.extTcc << 4) | 1);
          pre[n++] = 0;
          pre[n++] = 0;
        }
        for (int k = eb; k < 4 * words; k++) pre[n++] = 0;
      }
      if (tracks[dt.track].codec == LKF_CODEC_VP8 && payLen > 0 && x.meta.codec_len) {
        IngParsed v = {};
        if (vp8_parse(b + pay, int(payLen), v)) {  // translateVP8PacketTo downtrack.go:1728-1736
          for (int k = 0; k < x.meta.codec_len; k++) pre[n++] = x.meta.codec[k];
          pay += v.vhs;
          payLen -= v.vhs;
        } else {
          ok = false;  // "could not unmarshal VP8 packet": skipped
        }
      }
      if (ok) {
        total = u32(n) + payLen;
        sPre = u32(n);
        sPay = rp.off + pay;
      }
    }
    sLen = total;
    if (!WRITE) lens[i] = total;
  }
  __syncthreads();
  if (!WRITE || !sLen) return;
  u8 *o = out + offs[i];
  const u32 np = sPre, len = sLen, padded = (len + 15) & ~15u;
  for (u32 k = lane; k < padded; k += 64) o[k] = k < np ? pre[k] : k < len ? arena[sPay + (k - np)] : 0;
}

hipError_t launch_rtx_emit(hipStream_t s, bool write, u32 n, const lkf_rtx *rtx, const lkf_raw_pkt *src,
                           const u8 *arena, const DevDT *dts, const DevTrack *tracks, u32 *lens, const u64 *offs,
                           u8 *out, const u8 *dd) {
  if (!n) return hipSuccess;
  if (write)
    hipLaunchKernelGGL(k_rtx<true>, dim3(n), dim3(64), 0, s, rtx, src, arena, dts, tracks, lens, offs, out, dd);
  else
    hipLaunchKernelGGL(k_rtx<false>, dim3(n), dim3(64), 0, s, rtx, src, arena, dts, tracks, lens, offs, out, dd);
  return hipGetLastError();
}

// k_rtx_dd: epm.ddBytes of each lkf_rtx record (sequencer.go:326: copied
// from its slot at getExtPacketMetas) — the slot k_rtx_lookup returned
// (reserved = slot + 1), if it still holds the record's target SN; one
// thread per record, 256 B staged per record
__global__ void k_rtx_dd(u32 n, const lkf_rtx *__restrict__ rtx, const DevDT *__restrict__ dts,
                         const SeqMeta *__restrict__ seq, u32 seqSize, const u32 *__restrict__ ddIdx,
                         const u8 *__restrict__ seqDD, u8 *__restrict__ dd) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const lkf_rtx x = rtx[i];
  u8 *o = dd + size_t(i) * kSeqDDBytes;
  u32 len = 0;
  const u32 d = u32(x.dt);
  if (x.reserved && x.reserved <= seqSize && ddIdx[d] != 0xffffffffu && dts[d].extDD) {
    const u32 slot = x.reserved - 1;
    if (seq[size_t(d) * seqSize + slot].targetSeqNo == x.meta.target_sn) {
      const u8 *e = seqDD + (size_t(ddIdx[d]) * seqSize + slot) * kSeqDDBytes;
      len = e[0];
      for (u32 k = 0; k < len; k++) o[1 + k] = e[1 + k];
    }
  }
  o[0] = u8(len);
}

hipError_t launch_rtx_dd(hipStream_t s, u32 n, const lkf_rtx *rtx, const DevDT *dts, const SeqMeta *seq, u32 seqSize,
                         const u32 *ddIdx, const u8 *seqDD, u8 *dd) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_rtx_dd, dim3((n + 63) / 64), dim3(64), 0, s, n, rtx, dts, seq, seqSize, ddIdx, seqDD, dd);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_speakers: wave per room, lane per participant (<= 64 per room).
// partMics[partOff[r*64 + j] .. ) lists participant j's microphone streams.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_speakers(const u32 *__restrict__ roomPartOff, const u32 *__restrict__ partId,
                                                 const u32 *__restrict__ partMicOff, const u32 *__restrict__ mics,
                                                 const DevStream *__restrict__ streams, StreamHot *__restrict__ hot,
                                                 i64 nowNs, lkf_speaker *__restrict__ slots, u32 *__restrict__ counts,
                                                 const u32 *__restrict__ roomId) {
  const u32 r = blockIdx.x;
  const u32 lane = threadIdx.x;
  const u32 p0 = roomPartOff[r], p1 = roomPartOff[r + 1];
  const u32 np = p1 - p0;  // host guarantees <= 64
  const bool live = lane < np;
  double level = 0.0;
  bool active = false;
  u32 pid = 0;
  if (live) {
    const u32 pi = p0 + lane;
    pid = partId[pi];
    for (u32 m = partMicOff[pi]; m < partMicOff[pi + 1]; m++) {
      const u32 sid = mics[m];
      const DevStream s = streams[sid];
      StreamHot &h = hot[sid];
      // GetLevel -> resetIfStaleLocked (Milliseconds() truncates toward zero)
      if (!((nowNs - h.lastObservedNs) / 1000000 < i64(2 * s.observeDuration))) {
        h.smoothedLevel = 0.0;
        h.loudest = 127;
        h.activeDuration = 0;
        h.observedDuration = 0;
      }
      const double lv = h.smoothedLevel;
      if (lv >= s.activeThreshold) {
        active = true;
        if (lv > level) level = lv;
      }
    }
  }
  const float lf = float(level);
  // rank among the active participants: level descending, participant ascending
  u32 rank = 0;
  for (u32 j = 0; j < 64; j++) {
    const float lj = __shfl(lf, int(j), 64);
    const int aj = __shfl(int(active), int(j), 64);
    const u32 pj = u32(__shfl(int(pid), int(j), 64));
    if (live && active && aj && j < np && j != lane && (lj > lf || (lj == lf && pj < pid))) rank++;
  }
  const u64 am = __ballot(live && active);
  if (live && active) {
    lkf_speaker o;
    o.room = roomId[r];
    o.participant = pid;
    o.level = float(ceil(double(lf * 8.0f)) * (1.0 / 8));  // room.go:274-276
    o.active = 1;
    slots[size_t(r) * 64 + rank] = o;
  }
  if (lane == 0) counts[r] = u32(__popcll(am));
}

// ---------------------------------------------------------------------------
// k_spk_pack / k_bwe_pack: the summary records the room manager all-gathers every
// UpdateInterval (Room.audioUpdateWorker room.go:1278-1316),
// packed in place from the ranking slots and the DownTracks' sendingPacket
// totals: spk row entries (participant, float bits of the level, active) and
// bwe slots (subscriber, packets, bytes, deficient DownTracks, DownTracks),
// one thread per entry.  A slot's DownTracks are a host-built list (ascending
// subscribers within a room, as rooms.fold_summaries orders them), so the sums
// are plain loops: no atomics, the same bits every tick.
// ---------------------------------------------------------------------------
__global__ void k_spk_pack(RoomPackLaunch a) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.rows * a.k) return;
  const u32 row = i / a.k, j = i % a.k;
  const i32 r = a.rowEng[row];
  i32 v0 = -1, v1 = 0, v2 = 0;
  if (r >= 0 && j < a.counts[r]) {
    const lkf_speaker sp = a.slots[size_t(r) * 64 + j];
    v0 = i32(sp.participant);
    v1 = __float_as_int(sp.level);
    v2 = i32(sp.active);
  }
  a.spk[size_t(i) * 3] = v0;
  a.spk[size_t(i) * 3 + 1] = v1;
  a.spk[size_t(i) * 3 + 2] = v2;
}

__global__ void k_bwe_pack(RoomPackLaunch a) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.rows * a.s) return;
  const u32 b = a.slotOff[i], e = a.slotOff[i + 1];
  u64 pk = 0, by = 0, def = 0;
  for (u32 q = b; q < e; q++) {
    const DTCum c = a.cum[a.slotDts[q]];
    pk += c.packets;
    by += c.bytes;
    def += (c.flags & F_DEFICIENT) ? 1u : 0u;
  }
  i64 *o = a.bwe + size_t(i) * 5;
  o[0] = b == e ? -1 : a.slotSub[i];
  o[1] = i64(pk);
  o[2] = i64(by);
  o[3] = i64(def);
  o[4] = i64(e - b);
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
static u32 nblk(u64 n, u32 t) { return u32((n + t - 1) / t); }

// Zeroes an ingest's per-track ranges, error words, ExtPacket total and (with
// buckets) the per-datagram store list in one launch (they were five to six
// memsets on the ingest's critical path).
__global__ void k_ing_init(u32 ntracks, u32 n, u32 *__restrict__ tBegin, u32 *__restrict__ tEnd,
                           u32 *__restrict__ tRuns, u32 *__restrict__ err, u64 *__restrict__ total,
                           u64 *__restrict__ store) {
  const u32 stride = gridDim.x * blockDim.x;
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < ntracks || i < n || i < 4; i += stride) {
    if (i < ntracks) {
      tBegin[i] = 0;
      tEnd[i] = 0;
      tRuns[i] = 0;
    }
    if (store && i < n) store[i] = 0;
    if (i < 4) err[i] = 0;
    if (i < 2) total[i] = 0;
  }
}

// An ingest's RTCP NACK results start empty (side stream, before k_ing_nack).
__global__ void k_nack_init(u32 n, u32 *__restrict__ info, u32 *__restrict__ pairCnt) {
  const u32 stride = gridDim.x * blockDim.x;
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) info[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) *pairCnt = 0;
}

// The ingest chain on st (the prep stream: the next lkf_run's batch depends on
// it).  The NACK queues (k_ing_nack) need only the flows: they run on `side`
// after the stream kernel, beside the bucket decisions, the ExtPacket scan and
// the run's preparation; `sideDone` is recorded after them (the next ingest
// waits for it: it rewrites the parsed datagrams, flows and lists they read).
hipError_t launch_ingest(hipStream_t st, const IngestLaunch &a, hipStream_t side, hipEvent_t sideFork,
                         hipEvent_t sideDone, bool *sideUsed) {
  *sideUsed = false;
  if (a.n == 0) return hipSuccess;
  {
    const u32 m = a.ntracks > a.n ? a.ntracks : a.n;
    u32 g = nblk(m < 4 ? 4 : m, 256);
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_ing_init, dim3(g), dim3(256), 0, st, a.ntracks, a.n, a.tBegin, a.tEnd, a.tRuns, a.err,
                       a.total, a.bucket ? a.bucket->store : nullptr);
  }
  hipLaunchKernelGGL(k_ing_parse, dim3(nblk(a.n, kParseT)), dim3(kParseT), 0, st, a.raws, a.n, a.raw, a.streams, a.nstreams,
                     a.parsed, a.twcc, a.err, a.ntracks, a.tBegin, a.tEnd, a.tRuns);
  hipLaunchKernelGGL(k_ing_lists, dim3(a.ntracks), dim3(64), 0, st, a.raws, a.streams, a.nstreams, a.tBegin,
                     a.tEnd, a.listStride, a.list, a.listCnt);
  if (a.nstreams) {
    BktArgs bka = {};
    if (a.bucket) {  // the buckets decided in stream order inside the stream kernel
      bka.state = a.bucket->state;
      bka.tag = a.bucket->tag;
      bka.owner = a.bucket->owner;
      bka.store = a.bucket->store;
      bka.epoch = a.bucket->epoch;
    }
    // streams per wave: 4 when the ingest has fewer than 8 datagrams per stream
    const u32 sper = LKF_ING_PER_WAVE ? u32(LKF_ING_PER_WAVE) : u64(a.n) < u64(8) * a.nstreams ? 4u : 1u;
    const u32 sgrid = (a.nstreams + sper - 1) / sper;
    hipLaunchKernelGGL(k_ing_stream_wave<false>, dim3(sgrid), dim3(64), 0, st, a.raws, a.parsed, a.streams,
                       a.hot, a.hist, a.rings, a.tBegin, a.tEnd, a.flows, a.fwd, a.raw, a.ddStates, a.ddStructs,
                       a.ingDD, a.err, a.list, a.listCnt, a.listStride, bka, a.rxGap, a.nack ? a.nackIn : nullptr, a.nstreams, sper);
    if (a.ddStates)  // DD streams exist
      hipLaunchKernelGGL(k_ing_stream_wave<true>, dim3(sgrid), dim3(64), 0, st, a.raws, a.parsed, a.streams,
                         a.hot, a.hist, a.rings, a.tBegin, a.tEnd, a.flows, a.fwd, a.raw, a.ddStates, a.ddStructs,
                         a.ingDD, a.err, a.list, a.listCnt, a.listStride, bka, a.rxGap, a.nack ? a.nackIn : nullptr, a.nstreams, sper);
  }
  if (a.nack && a.nstreams) {  // after the flows: the loss ranges it pushes
    hipError_t r = hipEventRecord(sideFork, st);
    if (r == hipSuccess) r = hipStreamWaitEvent(side, sideFork, 0);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL(k_nack_init, dim3(std::min<u32>(nblk(a.n, 256), 1024)), dim3(256), 0, side, a.n, a.nackInfo,
                       a.nackPairCnt);
    // (the lane-parallel form needs >= LKF_NACK_FAST_MIN datagrams in a stream)
#define NACK_ARGS                                                                                              \
  a.raws, a.parsed, a.flows, a.streams, a.nack, a.hot, a.tBegin, a.tEnd, a.list, a.listCnt, a.listStride, a.nackInfo, \
      a.nackPairOff, a.nackPairCnt, a.nackPairs, a.nackPairCap, a.err, a.nackIn
    if (u64(a.n) >= u64(LKF_NACK_FAST_MIN) * a.nstreams)
      hipLaunchKernelGGL(k_ing_nack<true>, dim3(a.nstreams), dim3(64), 0, side, NACK_ARGS);
    else
      hipLaunchKernelGGL(k_ing_nack<false>, dim3(a.nstreams), dim3(64), 0, side, NACK_ARGS);
#undef NACK_ARGS
    r = hipEventRecord(sideDone, side);
    if (r != hipSuccess) return r;
    *sideUsed = true;
    // (measurement: LKF_NACK_ALONE=1 orders the rest of the ingest after the
    // NACK queues, so a kernel trace times k_ing_nack with the GPU to itself)
    static const bool alone = [] {
      const char *v = getenv("LKF_NACK_ALONE");
      return v && atoi(v) != 0;
    }();
    if (alone && (r = hipStreamWaitEvent(st, sideDone, 0)) != hipSuccess) return r;
  }
  hipError_t r = launch_scan(st, 2, nullptr, nullptr, nullptr, a.fwd, nullptr, a.n, a.partA, a.partB, a.pos, nullptr,
                             a.total, nullptr, nullptr);
  if (r != hipSuccess) return r;
  FwdPrep fp = {};
  if (a.fwdPrep.tBegin) {
    fp.tBegin = a.fwdPrep.tBegin;
    fp.tEnd = a.fwdPrep.tEnd;
    fp.err = a.fwdPrep.err;
    fp.fwdCnt = a.fwdPrep.fwdCnt;
    fp.stats = a.fwdPrep.stats;
    fp.fwdBytes = a.fwdPrep.fwdBytes;
    fp.nstats = a.fwdPrep.nstats;
    fp.ndts = a.fwdPrep.ndts;
    fp.ntracks = a.ntracks;
    fp.rawBegin = a.tBegin;
    fp.rawEnd = a.tEnd;
    fp.total = a.total;
  }
  u32 go = nblk(a.n, 256);
  if (fp.tBegin) {  // (enough threads for the per-track / per-DownTrack part too, grid-stride beyond)
    const u32 m = std::max(std::max(a.ntracks, fp.ndts), fp.nstats);
    go = std::max(go, std::min<u32>(nblk(m, 256), 1024));
  }
  hipLaunchKernelGGL(k_ing_out, dim3(go), dim3(256), 0, st, a.raws, a.parsed, a.streams, a.fwd, a.pos, a.n, a.flows,
                     a.out, a.ingDD, a.outDD, fp);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The RTX bucket (bucket_oracle.h restates it): k_ing_stream_wave decides
// AddPacketWithSequenceNumber per stream in datagram order (bkt_add_one; the
// in-order runs' pushes lane-parallel) on the slot tags and lists what to
// store per datagram; k_bkt_store then copies each stored datagram whose slot
// no later datagram of the batch took, its SN field set to the adjusted SN.
// ---------------------------------------------------------------------------
// One wave per 64 datagrams (grid-stride): lane = datagram for the store word
// and the descriptor (coalesced), then the wave copies the stored ones with
// four datagrams' loads in flight — 16-B copies when the source is 16-B
// aligned (the ring slots are), dword or byte copies otherwise.
#ifndef LKF_BKT_NOREAD  // (measurement builds: the ring copies written without reading the arena)
#define LKF_BKT_NOREAD 0
#endif
constexpr u32 kBktChunks = (kBktSlot - 16) / 16;  // 16-B chunks of the largest stored datagram (95)
__device__ __forceinline__ void bkt_store16(uint4 *p, uint4 v) {
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
  __builtin_nontemporal_store(v.z, &p->z);
  __builtin_nontemporal_store(v.w, &p->w);
}
static_assert(kBktChunks <= 128, "k_bkt_store copies at most two chunks per lane");
__global__ void __launch_bounds__(256) k_bkt_store(BucketLaunch A) {
  const u32 lane = threadIdx.x & 63;
  const u32 w0 = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (u32 base = w0 * 64; base < A.n; base += nw * 64) {
    const u32 ic = base + lane;
    u64 stw = 0;
    lkf_raw_pkt rp = {};
    if (ic < A.n) {
      stw = A.store[ic];
      if (stw >> 63) rp = A.raws[ic];
    }
    const u32 slotL = u32(stw), snL = u32(stw >> 32) & 0xffffu;
    u64 todo = __ballot(stw >> 63);
    while (todo) {
      u32 js[4];
      u32 k = 0;
      for (; k < 4 && todo; k++) {
        js[k] = u32(__ffsll(static_cast<long long>(todo))) - 1;
        todo &= todo - 1;
      }
      uint4 v[4][2];
#pragma unroll
      for (u32 x = 0; x < 4; x++) {  // the aligned datagrams' loads, all in flight
        v[x][0] = v[x][1] = make_uint4(0, 0, 0, 0);
        if (x < k) {
          const u32 off = __builtin_amdgcn_readlane(rp.off, js[x]);
          const u32 nc = (__builtin_amdgcn_readlane(rp.len, js[x]) + 15) / 16;
          if ((off & 15) == 0 && !LKF_BKT_NOREAD) {
            const uint4 *src = reinterpret_cast<const uint4 *>(A.raw + off);
            if (lane < nc) v[x][0] = src[lane];
            if (lane + 64 < nc) v[x][1] = src[lane + 64];
          }
        }
      }
#pragma unroll
      for (u32 x = 0; x < 4; x++) {
        if (x >= k) break;
        const u32 off = __builtin_amdgcn_readlane(rp.off, js[x]);
        const u32 len = __builtin_amdgcn_readlane(rp.len, js[x]);
        const u32 slot = __builtin_amdgcn_readlane(slotL, js[x]);
        const u16 sn = u16(__builtin_amdgcn_readlane(snL, js[x]));
        u8 *dst = A.ring + size_t(slot) * kBktSlot + 16;
        const u8 *src = A.raw + off;
        const u32 snw = (u32(sn >> 8) << 16) | (u32(sn & 255) << 24);  // SN field (bytes 2-3), little-endian word 0
        if ((off & 15) == 0) {
          const u32 nc = (len + 15) / 16;
          if (lane == 0) v[x][0].x = (v[x][0].x & 0x0000FFFFu) | snw;
          // (non-temporal: the ring is read back only for a NACK, long after;
          // the batch's payloads stay in the caches for emit)
          if (lane < nc) bkt_store16(reinterpret_cast<uint4 *>(dst) + lane, v[x][0]);
          if (lane + 64 < nc) bkt_store16(reinterpret_cast<uint4 *>(dst) + lane + 64, v[x][1]);
        } else if ((off & 3) == 0) {
          for (u32 w = lane; w < (len + 3) / 4; w += 64) {
            u32 d = reinterpret_cast<const u32 *>(src)[w];
            if (w == 0) d = (d & 0x0000FFFFu) | snw;
            reinterpret_cast<u32 *>(dst)[w] = d;
          }
        } else {
          for (u32 j = lane; j < len; j += 64) dst[j] = j == 2 ? u8(sn >> 8) : j == 3 ? u8(sn) : src[j];
        }
      }
    }
  }
}

// Bucket.GetPacket per RTX record, one wave each: the lookup on every lane
// (uniform), then the stored bytes gathered into the record's kBktSlot-byte
// slot of the RTX input buffer (the rings are 64-bit addressed; the RTX
// kernels take 32-bit offsets into that buffer).
__global__ void __launch_bounds__(64) k_bkt_read(u32 n, const int32_t *__restrict__ stream,
                                                 const u16 *__restrict__ sns, const BucketState *__restrict__ state,
                                                 const u32 *__restrict__ tag, const u8 *__restrict__ ring,
                                                 u8 *__restrict__ out, lkf_raw_pkt *__restrict__ src) {
  const u32 i = blockIdx.x, lane = threadIdx.x;
  if (i >= n) return;
  u32 len = 0;
  const u8 *p = nullptr;
  const int32_t sid = stream[i];
  if (sid >= 0) {
    const BucketState b = state[sid];
    const u16 sn = sns[i];
    const int diff = int(i16(u16(b.head - sn)));
    const int M = int(b.maxSteps);
    if (b.init && diff >= 0 && diff < M) {  // else ErrPacketTooNew / ErrPacketTooOld
      int sl = (int(b.step) - diff - 1) % M;
      if (sl < 0) sl += M;
      const u32 t = tag[b.base + u32(sl)];
      if ((t >> 16) != 0xFFFFu && u16(t) == sn) {  // else ErrPacketSizeInvalid / ErrPacketMismatch
        p = ring + size_t(b.base + u32(sl)) * kBktSlot + 16;
        len = t >> 16;
      }
    }
  }
  u8 *dst = out + size_t(i) * kBktSlot;
  for (u32 w = lane; w < (len + 3) / 4; w += 64) reinterpret_cast<u32 *>(dst)[w] = reinterpret_cast<const u32 *>(p)[w];
  if (lane == 0) {
    lkf_raw_pkt r = {};
    if (len) {
      u32 h = 12 + 4 * (p[0] & 15);
      if ((p[0] & 0x10) && h + 4 <= len) h += 4 + 4 * ((u32(p[h + 2]) << 8) | p[h + 3]);
      r.off = i * kBktSlot;
      r.len = len;
      r.reserved = h;
    }
    src[i] = r;
  }
}

hipError_t launch_bucket_store(hipStream_t st, const BucketLaunch &a) {
  if (a.n == 0 || a.nstreams == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bkt_store, dim3(std::min<u32>(nblk(a.n, 4), 4096)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_bucket_read(hipStream_t st, u32 n, const int32_t *stream, const u16 *sn, const BucketState *state,
                              const u32 *tag, const u8 *ring, u8 *out, lkf_raw_pkt *src) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_bkt_read, dim3(n), dim3(64), 0, st, n, stream, sn, state, tag, ring, out, src);
  return hipGetLastError();
}

hipError_t launch_nack_compact(hipStream_t st, u32 n, const lkf_raw_pkt *raws, const DevStream *streams,
                               const u32 *info, const u32 *pairOff, const lkf_nack_pair *pairs, u64 *partA,
                               u64 *partB, u64 *recPos, u64 *pairPos, u64 *totals, lkf_rtcp_nack *outRecs,
                               lkf_nack_pair *outPairs) {
  if (n == 0) return hipSuccess;
  hipError_t r = launch_scan(st, 3, nullptr, nullptr, nullptr, info, nullptr, n, partA, partB, recPos, pairPos,
                             totals, totals + 1, nullptr);
  if (r != hipSuccess) return r;
  hipLaunchKernelGGL(k_nack_compact, dim3(nblk(n, 256)), dim3(256), 0, st, n, raws, streams, info, pairOff, pairs,
                     recPos, pairPos, outRecs, outPairs);
  return hipGetLastError();
}

hipError_t launch_room_pack(hipStream_t spkStream, hipStream_t bweStream, const RoomPackLaunch &a) {
  if (a.rows * a.k) hipLaunchKernelGGL(k_spk_pack, dim3(nblk(u64(a.rows) * a.k, 256)), dim3(256), 0, spkStream, a);
  if (a.rows * a.s) hipLaunchKernelGGL(k_bwe_pack, dim3(nblk(u64(a.rows) * a.s, 256)), dim3(256), 0, bweStream, a);
  return hipGetLastError();
}

hipError_t launch_speakers(hipStream_t st, const SpeakersLaunch &a) {
  if (a.nrooms == 0) return hipSuccess;
  hipLaunchKernelGGL(k_speakers, dim3(a.nrooms), dim3(64), 0, st, a.roomPartOff, a.partId, a.partMicOff, a.mics,
                     a.streams, a.hot, a.nowNs, a.slots, a.counts, a.roomId);
  return hipGetLastError();
}

}  // namespace lkf

// (diagnosis builds, LKF_NACK_DBG=2) the NACK kernel's per-wave phase stamps
// since the last call: 7 words per wave; returns the count (then reset)
extern "C" int lkf_debug_nack_stamps(unsigned long long *out, unsigned int cap) {
#if LKF_NACK_DBG == 2
  static std::vector<unsigned long long> all;
  all.assign(size_t(lkf::kNackStampCap) * 7, 0);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(all.data(), HIP_SYMBOL(lkf::gNackStamp), all.size() * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  unsigned int n = 0;
  for (size_t i = 0; i < lkf::kNackStampCap && n < cap; i++)
    if (all[i * 7 + 5]) {  // (a wave that finished the lane-parallel form)
      for (int w = 0; w < 7; w++) out[size_t(n) * 7 + w] = all[i * 7 + w];
      n++;
    }
  std::fill(all.begin(), all.end(), 0ull);
  if (hipMemcpyToSymbol(HIP_SYMBOL(lkf::gNackStamp), all.data(), all.size() * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  return int(n);
#else
  (void)out;
  (void)cap;
  return -1;
#endif
}
