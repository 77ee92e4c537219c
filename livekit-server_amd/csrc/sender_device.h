// sender_device.h — buffer.RTPStatsSender.Update (rtpstats_sender.go:229-432)
// as device code: the scalar recurrence (one thread, or every lane of a wave
// with the same arguments) shared by k_decide_dt (the forwarded packets of a
// batch, folded into the DownTrack's decide wave) and k_sender_updates
// (host-listed padding, blank frames and RTX).  The snInfo ring (4096 x u32
// per DownTrack) and the gap histogram stay in HBM.
#pragma once
#include <hip/hip_runtime.h>

#include "fwd_state.h"

namespace lkf {
namespace ss {
using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

constexpr u64 kSnMask = kSnInfoSize - 1;
constexpr u32 kFlagMarker = 1, kFlagPadding = 2, kFlagOOO = 4;  // snInfoFlag rtpstats_sender.go:36-40

// rtpStatsBase.updateGapHistogram rtpstats_base.go:871-882
__device__ inline void ss_gap(u32 *gap, i64 g) {
  if (g < 2) return;
  const i64 missing = g - 1;
  gap[missing > kGapBins ? kGapBins - 1 : missing - 1]++;
}

// rtpStatsBase.updateJitter rtpstats_base.go:775-813 (Go's int64 arithmetic
// wraps: the products are formed in u64)
__device__ inline void ss_jitter(SenderStats &S, u64 ets, i64 t) {
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
__device__ inline void ss_update(SenderStats &S, u32 *ring, u32 *gap, i64 t, u64 esn, u64 ets, bool marker, u32 hdr,
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

}  // namespace ss
}  // namespace lkf
