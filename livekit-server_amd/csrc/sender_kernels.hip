// sender_kernels.hip — DownTrack.rtpStats on the GPU: buffer.RTPStatsSender
// .Update (rtpstats_sender.go:229-432) for every packet DownTrack.sendingPacket
// accounts (downtrack.go:1930-1959), SURVEY.md §8(f) 2.
//
//   k_sender_stats    the forwarded tuples of a batch: one wave per DownTrack
//                     with tuples.  Update is a serial recurrence (extHighestSN,
//                     the snInfo ring's lost/duplicate test, the jitter filter),
//                     so the wave stages 64 tuples at a time in LDS (one
//                     coalesced load of the Tuple records and the packets'
//                     arrival times / header sizes) and lane 0 steps through
//                     them with the DownTrack's statistics in LDS.  Parallelism
//                     is across DownTracks (thousands of waves per batch); the
//                     kernel runs on the emit stream after k_emit, so it
//                     overlaps the next batch's decide.
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

__global__ void __launch_bounds__(64) k_sender_stats(SenderLaunch A) {
  __shared__ __attribute__((aligned(16))) SenderStats sS;
  __shared__ u64 sEsn[64], sEts[64];
  __shared__ i64 sT[64];
  __shared__ u32 sHP[64];  // hdr | pay << 16
  __shared__ u8 sFl[64];
  const u32 d = blockIdx.x, lane = threadIdx.x;
  if (d >= A.ndts) return;
  const u32 n = A.fwdCnt[d];
  if (n == 0) return;
  constexpr u32 kW = sizeof(SenderStats) / 16;
  if (lane < kW) reinterpret_cast<uint4 *>(&sS)[lane] = reinterpret_cast<const uint4 *>(A.ss + d)[lane];
  __syncthreads();
  u32 *ring = A.ring + size_t(d) * kSnInfoSize;
  u32 *gap = A.gap + size_t(d) * kGapWords;
  const Tuple *tp = A.tuples + A.slotBase[d];
  for (u32 c0 = 0; c0 < n; c0 += 64) {
    const u32 m = min(64u, n - c0);
    if (lane < m) {
      const Tuple t = tp[c0 + lane];
      const lkf_pkt &p = A.pkts[t.pkt];
      sEsn[lane] = t.extSN;
      sEts[lane] = t.extTS;
      sT[lane] = p.arrival_ns;
      // sendingPacket: hdr.MarshalSize() of the translated header (the incoming
      // header's size: getTranslatedRTPHeader keeps its extensions), len(payload)
      sHP[lane] = u32(p.payload_off) | (u32(t.outLen - t.hdrLen) << 16);
      sFl[lane] = t.flags;
    }
    __syncthreads();
    if (lane == 0) {
      for (u32 k = 0; k < m; k++) {
        const u32 hp = sHP[k];
        ss_update(sS, ring, gap, sT[k], sEsn[k], sEts[k], (sFl[k] & LKF_OUT_MARKER) != 0, hp & 0xffffu, hp >> 16, 0);
        if (sFl[k] & LKF_OUT_KEYFRAME) sS.keyFrames++;  // UpdateKeyFrame(1) rtpstats_base.go:429-439
      }
    }
    __syncthreads();
  }
  if (lane < kW) reinterpret_cast<uint4 *>(A.ss + d)[lane] = reinterpret_cast<const uint4 *>(&sS)[lane];
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
  hipLaunchKernelGGL(k_sender_stats, dim3(a.ndts), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sender_updates(hipStream_t s, const SenderListLaunch &a) {
  if (!a.ngroups) return hipSuccess;
  hipLaunchKernelGGL(k_sender_updates, dim3((a.ngroups + 63) / 64), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace lkf
