// =============================================================================
//  tracker_oracle.h — TEST INFRASTRUCTURE ONLY (checker of the GPU stream
//  trackers).  CPU restatement of livekit-server v1.5.2's packet stream
//  tracker (the StreamTracker Observe of receiver.go:686-695):
//    StreamTracker        pkg/sfu/streamtracker/streamtracker.go:57-320
//    StreamTrackerPacket  pkg/sfu/streamtracker/streamtracker_packet.go:29-97
//  The worker goroutine's tickers (CheckStatus every CycleDuration, the
//  bitrate report every BitrateReportInterval) become calls made by the host
//  at those times: Tick(check, elapsedNs).  A worker runs from the Observe
//  that activates the tracker until Reset / SetPaused / Stop bump the
//  generation (streamtracker.go:155-185, 249-271): ticks without a live
//  worker do nothing.  Pinned by streamtracker_packet_test.go (kat_tracker.inc).
// =============================================================================
#pragma once
#include <cstdint>

namespace orc_st {
using i64 = int64_t;
using u32 = uint32_t;

enum Status : int { Stopped = 0, Active = 1 };
enum Change : int { ChangeNone = 0, ChangeStopped, ChangeActive };

struct PacketTracker {  // StreamTrackerPacket
  u32 samplesRequired, cyclesRequired;
  u32 countSinceLast = 0;
  bool initialized = false;
  u32 cycleCount = 0;
  void Reset() {
    countSinceLast = 0;
    cycleCount = 0;
    initialized = false;
  }
  Change Observe() {
    if (!initialized) {
      initialized = true;
      countSinceLast = 1;
      return ChangeActive;
    }
    countSinceLast++;
    return ChangeNone;
  }
  Change CheckStatus() {
    if (!initialized) return ChangeNone;
    if (countSinceLast >= samplesRequired)
      cycleCount++;
    else
      cycleCount = 0;
    Change c = ChangeNone;
    if (cycleCount == 0)
      c = ChangeStopped;
    else if (cycleCount >= cyclesRequired)
      c = ChangeActive;
    countSinceLast = 0;
    return c;
  }
};

struct Tracker {  // StreamTracker over a PacketTracker
  PacketTracker impl;
  bool paused = false, stopped = false, workerLive = false;
  Status status = Stopped, lastNotified = Stopped;
  int notifications = 0;         // onStatusChanged calls
  bool bitrateChanged = false;   // onBitrateAvailable fired by the last report
  i64 bytesForBitrate[4] = {0, 0, 0, 0};
  i64 bitrate[4] = {0, 0, 0, 0};

  Tracker(u32 samples, u32 cycles) { impl.samplesRequired = samples, impl.cyclesRequired = cycles; }
  void maybeNotify() {
    if (status != lastNotified) {
      lastNotified = status;
      notifications++;
    }
  }
  void resetLocked() {
    workerLive = false;  // generation bump
    status = Stopped;
    for (int i = 0; i < 4; i++) bytesForBitrate[i] = bitrate[i] = 0;
    impl.Reset();
  }
  void Reset() {
    if (stopped) return;
    resetLocked();
    maybeNotify();
  }
  void SetPaused(bool p) {
    paused = p;
    if (!p) {
      resetLocked();
    } else {
      workerLive = false;
      status = Stopped;
    }
    maybeNotify();
  }
  void Stop() {
    if (stopped) return;
    stopped = true;
    workerLive = false;
  }
  // Observe streamtracker.go:187-219
  void Observe(int temporalLayer, int pktSize, int payloadSize) {
    if (stopped || paused || payloadSize == 0) return;
    const Change c = impl.Observe();
    if (c == ChangeActive) {
      status = Active;
      workerLive = true;  // go s.worker(generation)
    }
    if (temporalLayer >= 0) bytesForBitrate[temporalLayer] += pktSize;
    if (c != ChangeNone) maybeNotify();
  }
  // updateStatus streamtracker.go:273-284
  void updateStatus() {
    switch (impl.CheckStatus()) {
      case ChangeStopped:
        status = Stopped;
        break;
      case ChangeActive:
        status = Active;
        break;
      default:
        break;
    }
    maybeNotify();
  }
  // bitrateReport streamtracker.go:286-310 (diff = the elapsed report interval)
  void bitrateReport(i64 elapsedNs) {
    const double secs = double(elapsedNs) / 1e9;  // time.Duration.Seconds
    bitrateChanged = false;
    for (int i = 0; i < 4; i++) {
      const i64 br = i64(double(bytesForBitrate[i] * 8) / secs);
      if ((bitrate[i] == 0 && br > 0) || (bitrate[i] > 0 && br == 0)) bitrateChanged = true;
      bitrate[i] = br;
      bytesForBitrate[i] = 0;
    }
  }
  // the worker's tick(s): check = the status ticker, elapsedNs > 0 = the bitrate ticker
  void Tick(bool check, i64 elapsedNs) {
    bitrateChanged = false;
    if (!workerLive) return;
    if (check) updateStatus();
    if (elapsedNs > 0) bitrateReport(elapsedNs);
  }
  // BitrateTemporalCumulative streamtracker.go:221-247
  void Cumulative(i64 out[4]) const {
    for (int i = 0; i < 4; i++) out[i] = bitrate[i];
    for (int i = 3; i >= 1; i--)
      if (out[i] != 0)
        for (int j = i - 1; j >= 0; j--) out[i] += out[j];
    for (int i = 0; i < 4; i++)
      if (out[i] == 0)
        for (int j = i + 1; j < 4; j++) out[j] = 0;
  }
};

}  // namespace orc_st
