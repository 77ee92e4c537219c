// sender_kernels.hip — DownTrack.rtpStats on the GPU: buffer.RTPStatsSender
// .Update (rtpstats_sender.go:229-432) for every packet DownTrack.sendingPacket
// accounts (downtrack.go:1930-1959), SURVEY.md §8(f) 2.
//
//   k_sender_stats    the forwarded tuples of a batch: one wave per DownTrack
//                     with tuples, lane = tuple.  Update is a serial recurrence
//                     (extHighestSN, the snInfo ring's lost/duplicate test, the
//                     jitter filter), but a run of in-order packets only
//                     accumulates: it is decided lane-parallel (see below) and
//                     only the packets that end a run (out of order,
//                     duplicate, a large gap) step through the scalar Update.
//                     It runs on the emit stream after k_emit, beside the next
//                     batch's decide.
//   k_sender_updates  host-listed packets (padding, blank frames, RTX): one
//                     thread per DownTrack, its packets in call order.
//
// The snInfo ring (4096 x u32 per DownTrack) stays in HBM: a forwarded packet
// writes its slot, a loss gap clears the skipped slots, and only an
// out-of-order or duplicate packet reads one.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace lkf {
namespace {
using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

constexpr u64 kSnMask = kSnInfoSize - 1;
constexpr u32 kFlagMarker = 1, kFlagPadding = 2, kFlagOOO = 4;  // snInfoFlag rtpstats_sender.go:36-40

// rtpStatsBase.updateGapHistogram rtpstats_base.go:871-882
__device__ void ss_gap(u32 *gap, i64 g) {
  if (g < 2) return;
  const i64 missing = g - 1;
  gap[missing > kGapBins ? kGapBins - 1 : missing - 1]++;
}

// rtpStatsBase.updateJitter rtpstats_base.go:775-813 (Go's int64 arithmetic
// wraps: the products are formed in u64)
__device__ void ss_jitter(SenderStats &S, u64 ets, i64 t) {
  if (S.lastJitterExtTimestamp == ets) return;
  const i64 since = i64(u64(t) - u64(S.firstTime));
  const u64 rtp = u64(i64(u64(since) * u64(i64(S.clockRate))) / 1000000000LL);
  const u64 transit = rtp - ets;
  if (S.lastTransit != 0) {
    i64 d = i64(transit - S.lastTransit);
    if (d < 0) d = i64(0 - u64(d));
    S.jitter += (double(d) - S.jitter) / 16;
    if (S.jitter > S.maxJitter) S.maxJitter = S.jitter;
  }
  S.lastTransit = transit;
  S.lastJitterExtTimestamp = ets;
}

// getSnInfoOutOfOrderSlot rtpstats_sender.go:889-897
__device__ __forceinline__ int ss_ooo_slot(u64 esn, u64 ehsn) {
  const i64 off = i64(ehsn - esn);
  return (off >= kSnInfoSize || off < 0) ? -1 : int(esn & kSnMask);
}

// Update rtpstats_sender.go:229-432 (one thread; S in LDS or registers, the
// ring and histogram in HBM)
__device__ void ss_update(SenderStats &S, u32 *ring, u32 *gap, i64 t, u64 esn, u64 ets, bool marker, u32 hdr,
                          u32 pay, u32 pad) {
  if (!S.initialized) {
    if (pay == 0) return;  // do not start on a padding only packet
    S.initialized = 1;
    S.firstTime = t;
    S.highestTime = t;
    S.extStartSN = esn;
    S.extHighestSN = esn - 1;
    S.extStartTS = ets;
    S.extHighestTS = ets;
  }
  const u64 pkt = u64(hdr + pay + pad);
  const u32 info = u32(u16(pkt)) | (u32(u8(hdr)) << 16) |
                   ((marker ? kFlagMarker : 0u) | (pay == 0 ? kFlagPadding : 0u)) << 24;
  bool dup = false;
  const i64 g = i64(esn - S.extHighestSN);
  if (g <= 0) {  // duplicate OR out-of-order
    if (pay == 0 && esn < S.extStartSN) return;
    if (esn < S.extStartSN) {
      S.packetsLost += S.extStartSN - esn;
      S.extStartSN = esn;
    }
    if (g != 0) S.packetsOutOfOrder++;
    const int slot = ss_ooo_slot(esn, S.extHighestSN);
    if (!(slot >= 0 && (ring[slot] & 0xffffu) == 0)) {  // !isSnInfoLost
      S.bytesDuplicate += pkt;
      S.headerBytesDuplicate += hdr;
      S.packetsDuplicate++;
      dup = true;
    } else {
      S.packetsLost--;
      ring[slot] = info | (kFlagOOO << 24);  // setSnInfo with isOutOfOrder
    }
  } else {  // in-order
    ss_gap(gap, g);
    // clearSnInfos(extHighestSN+1, esn): a gap of 4096 or more clears the ring
    const u64 nclr = u64(g - 1) < u64(kSnInfoSize) ? u64(g - 1) : u64(kSnInfoSize);
    for (u64 i = 0; i < nclr; i++) ring[(S.extHighestSN + 1 + i) & kSnMask] = 0;
    S.packetsLost += u64(g - 1);
    ring[esn & kSnMask] = info;
    S.extHighestSN = esn;
  }
  if (ets < S.extStartTS) S.extStartTS = ets;
  if (ets > S.extHighestTS) {
    if (pay > 0) S.highestTime = t;
    S.extHighestTS = ets;
  }
  if (!dup) {
    if (pay == 0) {
      S.packetsPadding++;
      S.bytesPadding += pkt;
      S.headerBytesPadding += hdr;
    } else {
      S.bytes += pkt;
      S.headerBytes += hdr;
      if (marker) S.frames++;
      ss_jitter(S, ets, t);
    }
  }
}

__device__ __forceinline__ u64 shfl_up64(u64 v, u32 d) {
  const u32 lane = threadIdx.x;
  const int src = lane >= d ? int(lane - d) : int(lane);
  const u32 lo = u32(__shfl(int(u32(v)), src, 64)), hi = u32(__shfl(int(u32(v >> 32)), src, 64));
  return lane >= d ? ((u64(hi) << 32) | lo) : 0;
}
__device__ __forceinline__ u64 shfl_idx64(u64 v, u32 src) {
  const u32 lo = u32(__shfl(int(u32(v)), int(src), 64)), hi = u32(__shfl(int(u32(v >> 32)), int(src), 64));
  return (u64(hi) << 32) | lo;
}
// inclusive prefix max over the lanes (u64)
__device__ __forceinline__ u64 scan_max64(u64 v) {
  for (u32 d = 1; d < 64; d <<= 1) {
    const u64 o = shfl_up64(v, d);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ u32 wave_sum32(u32 v) {
  for (int d = 32; d >= 1; d >>= 1) v += u32(__shfl_xor(int(v), d, 64));
  return v;
}
__device__ __forceinline__ u64 wave_sum64(u64 v) {
  for (int d = 32; d >= 1; d >>= 1) {
    const u32 lo = u32(__shfl_xor(int(u32(v)), d, 64)), hi = u32(__shfl_xor(int(u32(v >> 32)), d, 64));
    v += (u64(hi) << 32) | lo;
  }
  return v;
}

// One wave per DownTrack with forwarded tuples, 64 tuples at a time (lane =
// tuple, in send order).  A segment of in-order packets — each above every
// SN before it, a gap of at most 64, a payload, a timestamp not below the
// start — is decided in parallel: gap histogram / clears / snInfo writes per
// lane (distinct ring slots: the segment spans < 4096 SNs), counters as wave
// sums, the highest timestamp as a prefix max; only the jitter filter (a
// float64 recurrence over the new frames) steps serially.  The packet that
// ends a segment (out of order, duplicate, a larger gap, the first packet)
// takes the scalar Update on lane 0.  State S lives in LDS.
__global__ void __launch_bounds__(64) k_sender_stats(SenderLaunch A) {
  __shared__ __attribute__((aligned(16))) SenderStats sS;
  // the chunk's tuples (lane 0 reads them by index: the scalar steps, the
  // segment's last values) and the segment's per-frame jitter inputs
  __shared__ u64 sEsn[64], sEts[64], sTr[64];
  __shared__ i64 sT[64];
  __shared__ double sD[64];
  __shared__ u32 sHP[64];  // hdr | pay << 16
  __shared__ u8 sFl[64], sPT[64];
  const u32 d = blockIdx.x, lane = threadIdx.x;
  if (d >= A.ndts) return;
  const u32 n = A.fwdCnt[d];
  if (n == 0) return;
  constexpr u32 kW = sizeof(SenderStats) / 16;
  if (lane < kW) reinterpret_cast<uint4 *>(&sS)[lane] = reinterpret_cast<const uint4 *>(A.ss + d)[lane];
  u32 *ring = A.ring + size_t(d) * kSnInfoSize;
  u32 *gap = A.gap + size_t(d) * kGapWords;
  const Tuple *tp = A.tuples + A.slotBase[d];
  for (u32 c0 = 0; c0 < n; c0 += 64) {
    const u32 m = min(64u, n - c0);
    const bool valid = lane < m;
    u64 esn = 0, ets = 0;
    i64 t = 0;
    u32 hdr = 0, pay = 0;
    u8 fl = 0;
    if (valid) {
      const Tuple tu = tp[c0 + lane];
      const lkf_pkt &p = A.pkts[tu.pkt];
      esn = tu.extSN;
      ets = tu.extTS;
      t = p.arrival_ns;
      // sendingPacket: hdr.MarshalSize() of the translated header (the incoming
      // header's size: getTranslatedRTPHeader keeps its extensions), len(payload)
      hdr = p.payload_off;
      pay = u32(tu.outLen - tu.hdrLen);
      fl = tu.flags;
      sEsn[lane] = esn;
      sEts[lane] = ets;
      sT[lane] = t;
      sHP[lane] = hdr | (pay << 16);
      sFl[lane] = fl;
    }
    __syncthreads();
    const bool marker = fl & LKF_OUT_MARKER, kf = fl & LKF_OUT_KEYFRAME;
    u32 pos = 0;
    while (pos < m) {
      // ---- the in-order segment starting at pos
      const bool inSeg = valid && lane >= pos;
      const u64 high0 = sS.extHighestSN;
      // in a run where every SN exceeds the one before it, the highest SN
      // before a lane is its predecessor's; the first lane breaking that ends the run
      const u64 prevLane = shfl_up64(esn, 1);
      const u64 prev = lane > pos ? prevLane : high0;
      const u64 g = esn - prev;
      const bool ok = inSeg && sS.initialized && pay > 0 && i64(esn - prev) > 0 && g <= 64 && ets >= sS.extStartTS;
      const u64 badM = __ballot(inSeg && !ok);
      const u32 end = badM ? u32(__ffsll((long long)badM) - 1) : m;
      if (end > pos) {
        const bool act = lane >= pos && lane < end;
        // gap histogram, clearSnInfos(prev + 1, esn), setSnInfo (in order)
        if (act && g >= 2) {
          atomicAdd(&gap[g - 1 > u64(kGapBins) ? kGapBins - 1 : u32(g - 2)], 1u);
          for (u64 k = prev + 1; k != esn; k++) ring[k & kSnMask] = 0;
        }
        if (act) {
          const u64 pk = u64(hdr + pay);
          ring[esn & kSnMask] = u32(u16(pk)) | (u32(u8(hdr)) << 16) | ((marker ? kFlagMarker : 0u) << 24);
        }
        // highest timestamp: the lanes whose ets exceeds every earlier one (a
        // prefix max, unless the run's timestamps never decrease)
        const u64 h0 = sS.extHighestTS;
        const u64 prevEts = shfl_up64(ets, 1);
        u64 before = lane > pos ? prevEts : h0;
        if (__ballot(act && lane > pos && ets < prevEts)) {
          const u64 tm = scan_max64(act ? ets : 0ull);
          const u64 tmEx = shfl_up64(tm, 1);
          before = (lane > pos && tmEx > h0) ? tmEx : h0;
        } else if (lane > pos && h0 > before) {
          before = h0;
        }
        const u64 upM = __ballot(act && ets > before);
        // jitter over the segment's new frames (ets differs from the previous packet's)
        const bool isNew = act && ets != (lane > pos ? prevEts : sS.lastJitterExtTimestamp);
        const u64 newM = __ballot(isNew);
        const i64 since = i64(u64(t) - u64(sS.firstTime));
        const u64 rtp = u64(i64(u64(since) * u64(i64(sS.clockRate))) / 1000000000LL);
        const u64 transit = rtp - ets;
        // each new frame's previous transit: the previous new lane's, or the state's
        const u64 below = newM & ((1ull << lane) - 1);
        const int pl = below ? 63 - __clzll((long long)below) : -1;
        const u64 ptShfl = shfl_idx64(transit, pl >= 0 ? u32(pl) : lane);
        const u64 prevTransit = pl >= 0 ? ptShfl : sS.lastTransit;
        i64 dj = i64(transit - prevTransit);
        if (dj < 0) dj = i64(0 - u64(dj));
        if (isNew) {
          sD[lane] = double(dj);
          sPT[lane] = prevTransit != 0;
          sTr[lane] = transit;
        }
        // (a run of <= 64 packets: the byte, header and loss sums fit 32 bits)
        const u64 sumB = wave_sum32(act ? hdr + pay : 0u), sumH = wave_sum32(act ? hdr : 0u);
        const u32 frames = u32(__popcll(__ballot(act && marker))), kfs = u32(__popcll(__ballot(act && kf)));
        const u64 lost = wave_sum32((act && g >= 2) ? u32(g - 1) : 0u);
        __threadfence_block();
        __syncthreads();
        if (lane == 0) {  // the serial jitter filter over the new frames, then the segment's totals
          SenderStats &S = sS;
          double j = S.jitter, mj = S.maxJitter;
          int kl = -1;
          for (u64 w = newM; w; w &= w - 1) {
            const int k = __ffsll((long long)w) - 1;
            if (sPT[k]) {
              j += (sD[k] - j) / 16;
              if (j > mj) mj = j;
            }
            kl = k;
          }
          S.jitter = j;
          S.maxJitter = mj;
          if (kl >= 0) {
            S.lastTransit = sTr[kl];
            S.lastJitterExtTimestamp = sEts[kl];
          }
          if (upM) {
            const int ku = 63 - __clzll((long long)upM);
            S.highestTime = sT[ku];
            S.extHighestTS = sEts[ku];
          }
          S.extHighestSN = sEsn[end - 1];
          S.packetsLost += lost;
          S.bytes += sumB;
          S.headerBytes += sumH;
          S.frames += frames;
          S.keyFrames += kfs;
        }
        __syncthreads();
      }
      pos = end;
      if (pos < m) {  // the packet that ends the segment: the scalar Update on lane 0
        if (lane == 0) {
          const u32 hp = sHP[pos];
          ss_update(sS, ring, gap, sT[pos], sEsn[pos], sEts[pos], (sFl[pos] & LKF_OUT_MARKER) != 0, hp & 0xffffu,
                    hp >> 16, 0);
          if (sFl[pos] & LKF_OUT_KEYFRAME) sS.keyFrames++;  // UpdateKeyFrame(1) rtpstats_base.go:429-439
        }
        __threadfence_block();
        __syncthreads();
        pos++;
      }
    }
  }
  if (lane < kW) reinterpret_cast<uint4 *>(A.ss + d)[lane] = reinterpret_cast<const uint4 *>(&sS)[lane];
}

// Short batches (a 10-ms tick: one or two tuples per DownTrack): one thread
// per DownTrack, the scalar Update per tuple in send order — a wave per
// DownTrack would spend its time loading and storing the state.
__global__ void __launch_bounds__(64) k_sender_stats_thread(SenderLaunch A) {
  const u32 d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= A.ndts) return;
  const u32 n = A.fwdCnt[d];
  if (n == 0) return;
  SenderStats S = A.ss[d];
  u32 *ring = A.ring + size_t(d) * kSnInfoSize;
  u32 *gap = A.gap + size_t(d) * kGapWords;
  const Tuple *tp = A.tuples + A.slotBase[d];
  for (u32 k = 0; k < n; k++) {
    const Tuple tu = tp[k];
    const lkf_pkt &p = A.pkts[tu.pkt];
    ss_update(S, ring, gap, p.arrival_ns, tu.extSN, tu.extTS, (tu.flags & LKF_OUT_MARKER) != 0, p.payload_off,
              u32(tu.outLen - tu.hdrLen), 0);
    if (tu.flags & LKF_OUT_KEYFRAME) S.keyFrames++;  // UpdateKeyFrame(1) rtpstats_base.go:429-439
  }
  A.ss[d] = S;
}

__global__ void k_sender_updates(SenderListLaunch A) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.ngroups) return;
  const u32 b = A.gBegin[g], e = A.gBegin[g + 1];
  if (b >= e) return;
  const u32 d = A.list[b].dt;
  SenderStats S = A.ss[d];
  u32 *ring = A.ring + size_t(d) * kSnInfoSize;
  u32 *gap = A.gap + size_t(d) * kGapWords;
  for (u32 i = b; i < e; i++) {
    const SenderUpd &u = A.list[i];
    ss_update(S, ring, gap, u.t, u.esn, u.ets, u.marker != 0, u.hdr, u.pay, u.pad);
  }
  A.ss[d] = S;
}
}  // namespace

hipError_t launch_sender_stats(hipStream_t s, const SenderLaunch &a) {
  if (!a.ndts) return hipSuccess;
  if (a.perThread)
    hipLaunchKernelGGL(k_sender_stats_thread, dim3((a.ndts + 63) / 64), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_sender_stats, dim3(a.ndts), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sender_updates(hipStream_t s, const SenderListLaunch &a) {
  if (!a.ngroups) return hipSuccess;
  hipLaunchKernelGGL(k_sender_updates, dim3((a.ngroups + 63) / 64), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace lkf
