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
#include <cmath>
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

// StreamTrackerFrame streamtracker_frame.go:39-211
struct FrameTracker {
  u32 clockRate = 0;
  double minFPS = 0;
  bool initialized = false, tsInitialized = false;
  u32 oldestTS = 0, newestTS = 0;
  int numFrames = 0;
  double estimatedFrameRate = 0;
  i64 evalIntervalNs = 0;
  bool lastCheckSet = false;  // !lastStatusCheckAt.IsZero()
  i64 lastCheckNs = 0;
  static double roundFrameRate(double fr) { return std::round(fr / 0.01) * 0.01; }
  void updateEvalInterval() {
    evalIntervalNs = 500000000;  // checkInterval
    if (estimatedFrameRate > 0.0) {
      const i64 iv = i64(1e9 / estimatedFrameRate);
      if (iv > evalIntervalNs) evalIntervalNs = iv;
    }
    if (minFPS > 0.0) {
      const i64 iv = i64(1e9 / minFPS);
      if (iv > evalIntervalNs) evalIntervalNs = iv;
    }
  }
  void resetFPSCalculator() {
    tsInitialized = false;
    oldestTS = newestTS = 0;
    numFrames = 0;
    estimatedFrameRate = 0.0;
    updateEvalInterval();
  }
  void Reset() {
    initialized = false;
    resetFPSCalculator();
    lastCheckSet = false;
    lastCheckNs = 0;
  }
  Change Observe(bool hasMarker, u32 ts, i64 nowNs) {
    if (hasMarker) {
      if (!tsInitialized) {
        tsInitialized = true;
        oldestTS = newestTS = ts;
        numFrames = 1;
      } else {
        if (u32(ts - oldestTS) > (1u << 31)) oldestTS = ts;
        if (u32(ts - newestTS) < (1u << 31)) newestTS = ts;
        numFrames++;
      }
    }
    if (!initialized) {
      initialized = true;
      lastCheckSet = true;
      lastCheckNs = nowNs;
      return ChangeActive;
    }
    return ChangeNone;
  }
  double updateEstimatedFrameRate() {
    const u32 diff = newestTS - oldestTS;
    if (diff == 0 || numFrames < 2) return 0.0;
    const double frameRate = roundFrameRate(double(clockRate) / double(diff) * double(numFrames - 1));
    oldestTS = newestTS;
    numFrames = 1;
    double factor = 1.0;
    if (estimatedFrameRate < frameRate)
      factor = 0.6;  // frameRateIncreaseFactor
    else if (estimatedFrameRate > frameRate)
      factor = 0.9;  // frameRateDecreaseFactor
    const double est = roundFrameRate(frameRate * factor + estimatedFrameRate * (1.0 - factor));
    if (estimatedFrameRate != est) {
      estimatedFrameRate = est;
      updateEvalInterval();
    }
    return frameRate;
  }
  Change CheckStatus(i64 nowNs) {
    if (!initialized) return ChangeNone;
    if (!lastCheckSet) {
      lastCheckSet = true;
      lastCheckNs = nowNs;
    }
    if (nowNs - lastCheckNs < i64(0.98 * double(evalIntervalNs))) return ChangeNone;  // statusCheckTolerance
    lastCheckNs = nowNs;
    if (updateEstimatedFrameRate() == 0.0) {
      resetFPSCalculator();
      return ChangeStopped;
    }
    return ChangeActive;
  }
};

struct Tracker {  // StreamTracker over a PacketTracker (or a FrameTracker when frame)
  PacketTracker impl;
  bool frame = false;
  FrameTracker fimpl;
  bool paused = false, stopped = false, workerLive = false;
  Status status = Stopped, lastNotified = Stopped;
  int notifications = 0;         // onStatusChanged calls
  bool bitrateChanged = false;   // onBitrateAvailable fired by the last report
  i64 bytesForBitrate[4] = {0, 0, 0, 0};
  i64 bitrate[4] = {0, 0, 0, 0};

  Tracker(u32 samples, u32 cycles) { impl.samplesRequired = samples, impl.cyclesRequired = cycles; }
  static Tracker Frame(u32 clockRate, double minFPS) {
    Tracker t(0, 0);
    t.frame = true;
    t.fimpl.clockRate = clockRate;
    t.fimpl.minFPS = minFPS;
    t.fimpl.Reset();
    return t;
  }
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
    if (frame) fimpl.Reset();
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
  void Observe(int temporalLayer, int pktSize, int payloadSize, bool hasMarker = false, u32 ts = 0, i64 nowNs = 0) {
    if (stopped || paused || payloadSize == 0) return;
    const Change c = frame ? fimpl.Observe(hasMarker, ts, nowNs) : impl.Observe();
    if (c == ChangeActive) {
      status = Active;
      workerLive = true;  // go s.worker(generation)
    }
    if (temporalLayer >= 0) bytesForBitrate[temporalLayer] += pktSize;
    if (c != ChangeNone) maybeNotify();
  }
  // updateStatus streamtracker.go:273-284
  void updateStatus(i64 nowNs = 0) {
    switch (frame ? fimpl.CheckStatus(nowNs) : impl.CheckStatus()) {
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
  void Tick(bool check, i64 elapsedNs, i64 nowNs = 0) {
    bitrateChanged = false;
    if (!workerLive) return;
    if (check) updateStatus(nowNs);
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

// StreamTrackerDependencyDescriptor streamtracker_dd.go:27-289 — one per SVC
// track with the dependency-descriptor extension, shared by its spatial
// layers (LayeredTracker).  Observe takes the packet's ExtDependencyDescriptor
// (nullptr-equivalent: hasDD false): the active-decode-target mask when
// updated, the parser's decode targets and the frame's DTIs.  The worker runs
// from the first mask (maxSpatial leaving -1) or a SetPaused(true) until
// Stop / SetPaused(false); host ticks report bitrates over `elapsedNs`.
// Pinned by streamtracker_dd_test.go (kat_tracker.inc).
struct DDTracker {
  struct DT {
    int target;
    int s, t;
  };
  bool paused = false, stopped = false, workerLive = false;
  int maxS = -1, maxT = -1;  // InvalidLayerSpatial / InvalidLayerTemporal
  i64 bytes[3][4] = {}, bitrate[3][4] = {};
  int notifications[3] = {0, 0, 0};  // onStatusChanged calls per layer
  int lastNotified[3] = {-1, -1, -1};  // the status of the last call per layer (-1: none)
  u32 bitrateChangedMask = 0;          // onBitrateAvailable per layer by the last report
  void notify(int from, int to, int st) {
    for (int i = from; i <= to; i++) {
      notifications[i]++;
      lastNotified[i] = st;
    }
  }
  // Observe :133-212
  void Observe(int pktSize, int payloadSize, bool hasDD, bool activeUpdated, bool hasMask, u32 mask,
               const DT *targets, int ntargets, const uint8_t *dtis, int ndtis) {
    if (stopped || paused || payloadSize == 0 || !hasDD) return;
    if (hasMask && activeUpdated) {
      int ms = 0, mt = 0;
      for (int k = 0; k < ntargets; k++)
        if ((mask & (1u << targets[k].target)) != 0) {  // != DecodeTargetNotPresent (0)
          if (ms < targets[k].s) ms = targets[k].s;
          if (mt < targets[k].t) mt = targets[k].t;
        }
      if (ms > 2) ms = 2;
      if (mt > 3) mt = 3;
      const int old = maxS;
      maxS = ms, maxT = mt;
      if (old == -1) workerLive = true;  // go s.worker(s.generation.Inc())
      if (old > maxS)
        notify(maxS + 1, old, Stopped);
      else if (old < maxS)
        notify(old + 1, maxS, Active);
    }
    for (int k = 0; k < ntargets; k++) {
      if (ndtis <= targets[k].target) continue;
      if (dtis[targets[k].target] == 0) continue;  // DecodeTargetNotPresent
      bytes[targets[k].s][targets[k].t] += pktSize;
    }
  }
  // resetLocked :108-121
  void resetLocked() {
    workerLive = false;
    for (int s = 0; s < 3; s++)
      for (int t = 0; t < 4; t++) bytes[s][t] = bitrate[s][t] = 0;
  }
  // SetPaused :123-137
  void SetPaused(bool p) {
    if (paused == p) return;
    paused = p;
    if (!p)
      resetLocked();
    else
      workerLive = true;
  }
  // Stop :57-68
  void Stop() {
    if (stopped) return;
    stopped = true;
    workerLive = false;
  }
  int Status(int layer) const { return layer > maxS ? Stopped : Active; }  // :84-93
  void Cumulative(int layer, i64 out[4]) const {                            // :95-106 (not cumulative)
    for (int t = 0; t < 4; t++) out[t] = layer > maxS ? 0 : bitrate[layer][t];
  }
  // bitrateReport :226-259, diff = the elapsed report interval (Duration.Seconds)
  void bitrateReport(i64 elapsedNs) {
    const double secs = double(elapsedNs / 1000000000LL) + double(elapsedNs % 1000000000LL) / 1e9;
    bitrateChangedMask = 0;
    for (int s = 0; s < 3; s++) {
      bool changed = false;
      for (int t = 0; t < 4; t++) {
        const i64 br = i64(double(bytes[s][t] * 8) / secs);
        if ((bitrate[s][t] == 0 && br > 0) || (bitrate[s][t] > 0 && br == 0)) changed = true;
        bitrate[s][t] = br;
        bytes[s][t] = 0;
      }
      if (changed) bitrateChangedMask |= 1u << s;
    }
  }
  void Tick(i64 elapsedNs) {
    bitrateChangedMask = 0;
    if (workerLive && elapsedNs > 0) bitrateReport(elapsedNs);
  }
};

}  // namespace orc_st
