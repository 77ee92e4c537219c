// =============================================================================
//  sender_oracle.h — TEST INFRASTRUCTURE ONLY (checker + CPU baseline).
//
//  Scalar restatement of buffer.RTPStatsSender.Update, the per-forwarded-packet
//  sender statistics every DownTrack keeps (pkg/sfu/buffer/rtpstats_sender.go
//  :229-432, with rtpStatsBase.updateJitter / updateGapHistogram /
//  UpdateKeyFrame rtpstats_base.go:429-439, :775-813, :871-882), driven from
//  DownTrack.sendingPacket (downtrack.go:1930-1959) for forwarded packets
//  (:737), padding (:835), blank frames (:1377) and RTX (:1671).
//
//  Not restated (wall clock or report machinery, outside the per-packet path):
//  startTime (time.Now() at init), endTime (Stop), the receiver- and
//  sender-report snapshots (their start adjustments and maxJitterFeed) and
//  lastKeyFrame (time.Now()).  No reference test covers the sender side:
//  parity of this restatement is unpinned beyond the shared rtpStatsBase code
//  (its gap histogram / jitter formulas) and is checked engine-vs-oracle only.
// =============================================================================
#pragma once
#include <cstdint>
#include <cstring>

namespace orc_ss {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;

constexpr int kSnInfoSize = 4096;  // cSnInfoSize rtpstats_sender.go:30
constexpr u64 kSnInfoMask = kSnInfoSize - 1;
constexpr int kGapBins = 101;      // cGapHistogramNumBins rtpstats_base.go:31
constexpr u8 kFlagMarker = 1, kFlagPadding = 2, kFlagOutOfOrder = 4;  // snInfoFlag rtpstats_sender.go:36-40

struct SnInfo {  // rtpstats_sender.go:42-46
  u16 pktSize;
  u8 hdrSize;
  u8 flags;
};

struct RTPStatsSender {
  u32 clockRate = 0;
  bool initialized = false;
  i64 firstTime = 0, highestTime = 0;  // ns (virtual clock: the packet times passed in)
  u64 extStartSN = 0, extHighestSN = 0, extStartTS = 0, extHighestTS = 0;
  u64 lastTransit = 0, lastJitterExtTimestamp = 0;
  u64 bytes = 0, headerBytes = 0, bytesDuplicate = 0, headerBytesDuplicate = 0, bytesPadding = 0,
      headerBytesPadding = 0;
  u64 packetsDuplicate = 0, packetsPadding = 0, packetsOutOfOrder = 0, packetsLost = 0;
  u32 frames = 0, keyFrames = 0;
  double jitter = 0, maxJitter = 0;
  u32 gapHistogram[kGapBins] = {};
  SnInfo snInfos[kSnInfoSize] = {};

  // rtpstats_base.go:871-882
  void updateGapHistogram(i64 gap) {
    if (gap < 2) return;
    const i64 missing = gap - 1;
    if (missing > kGapBins)
      gapHistogram[kGapBins - 1]++;
    else
      gapHistogram[missing - 1]++;
  }
  // rtpstats_base.go:775-813 (Go int64 arithmetic wraps: done in u64)
  void updateJitter(u64 ets, i64 packetTime) {
    if (lastJitterExtTimestamp != ets) {
      const i64 timeSinceFirst = i64(u64(packetTime) - u64(firstTime));
      const u64 packetTimeRTP = u64(i64(u64(timeSinceFirst) * u64(i64(clockRate))) / 1000000000LL);
      const u64 transit = packetTimeRTP - ets;
      if (lastTransit != 0) {
        i64 d = i64(transit - lastTransit);
        if (d < 0) d = i64(0 - u64(d));
        jitter += (double(d) - jitter) / 16;
        if (jitter > maxJitter) maxJitter = jitter;
      }
      lastTransit = transit;
      lastJitterExtTimestamp = ets;
    }
  }
  // rtpstats_sender.go:889-897
  int getSnInfoOutOfOrderSlot(u64 esn, u64 ehsn) const {
    const i64 offset = i64(ehsn - esn);
    if (offset >= kSnInfoSize || offset < 0) return -1;
    return int(esn & kSnInfoMask);
  }
  // rtpstats_sender.go:899-923
  void setSnInfo(u64 esn, u64 ehsn, u16 pktSize, u8 hdrSize, u16 payloadSize, bool marker, bool ooo) {
    int slot;
    if (i64(esn - ehsn) < 0) {
      slot = getSnInfoOutOfOrderSlot(esn, ehsn);
      if (slot < 0) return;
    } else {
      slot = int(esn & kSnInfoMask);
    }
    SnInfo &s = snInfos[slot];
    s.pktSize = pktSize;
    s.hdrSize = hdrSize;
    s.flags = u8((marker ? kFlagMarker : 0) | (payloadSize == 0 ? kFlagPadding : 0) | (ooo ? kFlagOutOfOrder : 0));
  }
  // rtpstats_sender.go:925-936
  void clearSnInfos(u64 from, u64 toExcl) {
    if (toExcl <= from) return;
    for (u64 esn = from; esn != toExcl; esn++) snInfos[esn & kSnInfoMask] = SnInfo{0, 0, 0};
  }
  // rtpstats_sender.go:938-945
  bool isSnInfoLost(u64 esn, u64 ehsn) const {
    const int slot = getSnInfoOutOfOrderSlot(esn, ehsn);
    if (slot < 0) return false;
    return snInfos[slot].pktSize == 0;
  }

  // Update rtpstats_sender.go:229-432
  void Update(i64 packetTime, u64 esn, u64 ets, bool marker, int hdrSize, int payloadSize, int paddingSize) {
    if (!initialized) {
      if (payloadSize == 0) return;  // do not start on a padding only packet
      initialized = true;
      firstTime = packetTime;
      highestTime = packetTime;
      extStartSN = esn;
      extHighestSN = esn - 1;
      extStartTS = ets;
      extHighestTS = ets;
    }
    const u64 pktSize = u64(hdrSize + payloadSize + paddingSize);
    bool isDuplicate = false;
    const i64 gapSN = i64(esn - extHighestSN);
    if (gapSN <= 0) {  // duplicate OR out-of-order
      if (payloadSize == 0 && esn < extStartSN) return;
      if (esn < extStartSN) {
        packetsLost += extStartSN - esn;
        extStartSN = esn;
      }
      if (gapSN != 0) packetsOutOfOrder++;
      if (!isSnInfoLost(esn, extHighestSN)) {
        bytesDuplicate += pktSize;
        headerBytesDuplicate += u64(hdrSize);
        packetsDuplicate++;
        isDuplicate = true;
      } else {
        packetsLost--;
        setSnInfo(esn, extHighestSN, u16(pktSize), u8(hdrSize), u16(payloadSize), marker, true);
      }
    } else {  // in-order
      updateGapHistogram(gapSN);
      clearSnInfos(extHighestSN + 1, esn);
      packetsLost += u64(gapSN - 1);
      setSnInfo(esn, extHighestSN, u16(pktSize), u8(hdrSize), u16(payloadSize), marker, false);
      extHighestSN = esn;
    }
    if (ets < extStartTS) extStartTS = ets;
    if (ets > extHighestTS) {
      if (payloadSize > 0) highestTime = packetTime;
      extHighestTS = ets;
    }
    if (!isDuplicate) {
      if (payloadSize == 0) {
        packetsPadding++;
        bytesPadding += pktSize;
        headerBytesPadding += u64(hdrSize);
      } else {
        bytes += pktSize;
        headerBytes += u64(hdrSize);
        if (marker) frames++;
        updateJitter(ets, packetTime);
      }
    }
  }
  void UpdateKeyFrame(u32 n) { keyFrames += n; }  // rtpstats_base.go:429-439 (lastKeyFrame: wall clock)
};

}  // namespace orc_ss
