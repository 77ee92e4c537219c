// tracker_kernels.hip — the packet stream tracker of every (track, spatial
// layer) on the GPU (StreamTracker.Observe from
// WebRTCReceiver.forwardRTP receiver.go:686-695; streamtracker.go:57-320,
// streamtracker_packet.go:29-97).
//   k_tracker_observe  per batch: one wave per tracker counts its layer's
//                      packets (payload > 0) and bytes per temporal layer —
//                      order-free sums, except the first packet after a reset,
//                      which activates the tracker (and starts its worker)
//   k_tracker_tick     the worker's tickers, driven by the host: CheckStatus
//                      (cycle counting) and the bitrate report, one thread each
// A frame tracker (streamtracker_frame.go:39-211) observes its layer's marker
// packets in batch order (oldest / newest timestamp, frame count: lane-uniform
// updates over the ballot of markers) and estimates the frame rate at
// CheckStatus on the virtual clock.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace lkf {
namespace {
using u32 = uint32_t;
using i64 = int64_t;
using u64 = uint64_t;

__device__ __forceinline__ u64 wsum(u64 v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ void notify(TrackerState &s) {  // maybeNotifyStatus streamtracker.go:104-118
  if (s.status != s.lastNotified) {
    s.lastNotified = s.status;
    s.notifications++;
  }
}

__global__ void __launch_bounds__(64) k_tracker_observe(TrackerState *st, u32 n, const RunDesc *__restrict__ desc,
                                                        const u32 *__restrict__ tBegin, const u32 *__restrict__ tEnd) {
  const lkf_pkt *__restrict__ pkts = reinterpret_cast<const lkf_pkt *>(desc->pkts);
  const u32 k = blockIdx.x;
  if (k >= n) return;
  TrackerState s = st[k];  // (wave-uniform)
  if (s.stopped || s.paused) return;
  const u32 b = tBegin[s.track], e = tEnd[s.track];
  u64 cnt = 0, bytes[4] = {0, 0, 0, 0};
  bool gotFirst = false;
  i64 firstArrival = 0;
  for (u32 base = b; base < e; base += 64) {  // (uniform trip count)
    const u32 i = base + threadIdx.x;
    bool q = false, mk = false;
    u32 ts = 0;
    i64 arr = 0;
    if (i < e) {
      const lkf_pkt &p = pkts[i];
      q = p.layer == s.layer && p.payload_len > 0;
      if (q) {
        cnt++;
        // len(pkt.RawPacket): header + payload (the padding of a padded packet is not in lkf_pkt)
        const int t = p.temporal;
        if (t >= 0 && t < 4) bytes[t] += u64(p.payload_off) + p.payload_len;
        mk = (p.hdr1 & 0x80) != 0;
        ts = u32(p.ext_ts);
        arr = p.arrival_ns;
      }
    }
    if (!s.frame) continue;
    const u64 qm = __ballot(q);
    if (!gotFirst && qm) {
      gotFirst = true;
      firstArrival = __shfl(arr, __ffsll(static_cast<long long>(qm)) - 1, 64);
    }
    for (u64 mm = __ballot(mk); mm; mm &= mm - 1) {  // StreamTrackerFrame.Observe, marker packets in order
      const u32 t = u32(__shfl(int(ts), __ffsll(static_cast<long long>(mm)) - 1, 64));
      if (!s.tsInit) {
        s.tsInit = 1;
        s.oldestTS = s.newestTS = t;
        s.numFrames = 1;
      } else {
        if (u32(t - s.oldestTS) > (1u << 31)) s.oldestTS = t;
        if (u32(t - s.newestTS) < (1u << 31)) s.newestTS = t;
        s.numFrames++;
      }
    }
  }
  cnt = wsum(cnt);
  for (int t = 0; t < 4; t++) bytes[t] = wsum(bytes[t]);
  if (threadIdx.x != 0 || cnt == 0) return;
  if (!s.initialized) {  // StreamTrackerPacket / Frame.Observe: the first packet activates
    s.initialized = 1;
    if (s.frame) {  // lastStatusCheckAt = time.Now()
      s.lastCheckSet = 1;
      s.lastCheckNs = firstArrival;
    }
    s.countSinceLast = u32(cnt);
    s.status = 1;
    s.workerLive = 1;  // go s.worker(generation)
    notify(s);
  } else {
    s.countSinceLast += u32(cnt);
  }
  for (int t = 0; t < 4; t++) s.bytes[t] += i64(bytes[t]);
  st[k] = s;
}

__device__ __forceinline__ double round_fps(double fr) { return round(fr / 0.01) * 0.01; }  // roundFrameRate

// StreamTrackerFrame.CheckStatus streamtracker_frame.go:124-186: 0 none, 1 stopped, 2 active
__device__ int frame_check(TrackerState &s, i64 nowNs) {
  if (!s.lastCheckSet) {
    s.lastCheckSet = 1;
    s.lastCheckNs = nowNs;
  }
  if (nowNs - s.lastCheckNs < i64(0.98 * double(s.evalIntervalNs))) return 0;
  s.lastCheckNs = nowNs;
  const u32 diff = s.newestTS - s.oldestTS;
  double frameRate = 0.0;
  if (diff != 0 && s.numFrames >= 2) {  // updateEstimatedFrameRate
    frameRate = round_fps(double(s.clockRate) / double(diff) * double(s.numFrames - 1));
    s.oldestTS = s.newestTS;
    s.numFrames = 1;
    double factor = 1.0;
    if (s.estFps < frameRate)
      factor = 0.6;
    else if (s.estFps > frameRate)
      factor = 0.9;
    // unfused, as the reference computes it
    const double est = round_fps(__dadd_rn(__dmul_rn(frameRate, factor), __dmul_rn(s.estFps, __dadd_rn(1.0, -factor))));
    if (s.estFps != est) {
      s.estFps = est;
      tracker_frame_eval_interval(s);
    }
  }
  if (frameRate == 0.0) {
    tracker_frame_reset_fps(s);
    return 1;
  }
  return 2;
}

__global__ void k_tracker_tick(TrackerState *st, const int32_t *__restrict__ ids, u32 n, int check, i64 elapsedNs,
                               i64 nowNs, lkf_tracker_status *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  TrackerState s = st[ids[i]];
  s.bitrateChanged = 0;
  if (s.workerLive) {
    if (check && s.initialized && s.frame) {
      const int c = frame_check(s, nowNs);
      if (c == 1)
        s.status = 0;
      else if (c == 2)
        s.status = 1;
    } else if (check && s.initialized) {  // updateStatus -> StreamTrackerPacket.CheckStatus
      if (s.countSinceLast >= s.samples)
        s.cycleCount++;
      else
        s.cycleCount = 0;
      if (s.cycleCount == 0)
        s.status = 0;
      else if (s.cycleCount >= s.cycles)
        s.status = 1;
      s.countSinceLast = 0;
    }
    if (check) notify(s);
    if (elapsedNs > 0) {  // bitrateReport
      const double secs = double(elapsedNs) / 1e9;
      for (int t = 0; t < 4; t++) {
        const i64 br = i64(double(s.bytes[t] * 8) / secs);
        if ((s.bitrate[t] == 0 && br > 0) || (s.bitrate[t] > 0 && br == 0)) s.bitrateChanged = 1;
        s.bitrate[t] = br;
        s.bytes[t] = 0;
      }
    }
  }
  st[ids[i]] = s;
  lkf_tracker_status o = {};
  o.tracker = ids[i];
  o.status = s.status;
  o.bitrate_changed = s.bitrateChanged;
  o.notifications = s.notifications;
  i64 c[4];
  for (int t = 0; t < 4; t++) o.bitrate[t] = c[t] = s.bitrate[t];
  for (int t = 3; t >= 1; t--)  // BitrateTemporalCumulative streamtracker.go:221-247
    if (c[t] != 0)
      for (int j = t - 1; j >= 0; j--) c[t] += c[j];
  for (int t = 0; t < 4; t++)
    if (c[t] == 0)
      for (int j = t + 1; j < 4; j++) c[j] = 0;
  for (int t = 0; t < 4; t++) o.cumulative[t] = c[t];
  out[i] = o;
}

// the DD stream tracker's worker tick: bitrateReport (streamtracker_dd.go:226-259)
// over the elapsed interval (time.Duration.Seconds), then the status
__global__ void k_dd_tracker_tick(DDTrkState *st, const int32_t *__restrict__ ids, u32 n, i64 elapsedNs,
                                  lkf_dd_tracker_status *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DDTrkState s = st[ids[i]];
  s.changedMask = 0;
  if ((s.flags & DT_WORKER) && elapsedNs > 0) {
    const double secs = double(elapsedNs / 1000000000LL) + double(elapsedNs % 1000000000LL) / 1e9;
    for (int l = 0; l < 3; l++) {
      bool changed = false;
      for (int t = 0; t < 4; t++) {
        const i64 br = i64(double(s.bytes[l][t] * 8) / secs);
        if ((s.bitrate[l][t] == 0 && br > 0) || (s.bitrate[l][t] > 0 && br == 0)) changed = true;
        s.bitrate[l][t] = br;
        s.bytes[l][t] = 0;
      }
      if (changed) s.changedMask |= 1u << l;
    }
  }
  st[ids[i]] = s;
  lkf_dd_tracker_status o = {};
  o.tracker = ids[i];
  o.max_spatial = s.maxS;
  o.max_temporal = s.maxT;
  o.bitrate_changed = s.changedMask;
  for (int l = 0; l < 3; l++) {
    o.notifications[l] = s.notif[l];
    o.last_notified[l] = s.lastNotified[l];
    o.status[l] = l > s.maxS ? 0 : 1;  // Status(layer) :84-93
    for (int t = 0; t < 4; t++) o.bitrate[l][t] = l > s.maxS ? 0 : s.bitrate[l][t];  // BitrateTemporalCumulative
  }
  o.worker = (s.flags & DT_WORKER) ? 1 : 0;
  out[i] = o;
}
}  // namespace

hipError_t launch_dd_tracker_tick(hipStream_t s, DDTrkState *st, const int32_t *ids, uint32_t n, int64_t elapsedNs,
                                  lkf_dd_tracker_status *out) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_dd_tracker_tick, dim3((n + 63) / 64), dim3(64), 0, s, st, ids, n, elapsedNs, out);
  return hipGetLastError();
}

hipError_t launch_tracker_observe(hipStream_t s, TrackerState *st, uint32_t n, const RunDesc *desc,
                                  const uint32_t *tBegin, const uint32_t *tEnd) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_tracker_observe, dim3(n), dim3(64), 0, s, st, n, desc, tBegin, tEnd);
  return hipGetLastError();
}
hipError_t launch_tracker_tick(hipStream_t s, TrackerState *st, const int32_t *ids, uint32_t n, int check,
                               int64_t elapsedNs, int64_t nowNs, lkf_tracker_status *out) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_tracker_tick, dim3((n + 63) / 64), dim3(64), 0, s, st, ids, n, check, elapsedNs, nowNs, out);
  return hipGetLastError();
}

}  // namespace lkf
