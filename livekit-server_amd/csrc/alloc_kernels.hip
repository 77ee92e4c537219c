// alloc_kernels.hip — Forwarder.AllocateOptimal (forwarder.go:591-725) +
// updateAllocation (:1353-1373) for many DownTracks at once (SURVEY.md §8(f)
// 4: "Forwarder allocation ... as a batched control kernel driven by
// streamallocator estimates").  One thread per request: the allocation is a
// few dozen scalar decisions over the DownTrack's layer state and a 3x4
// bitrate table; the bytes are the 256-B DTHot read and written once.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace lkf {
namespace {
using i32 = int32_t;
using u32 = uint32_t;
using i64 = int64_t;
constexpr i32 INV = -1;  // buffer.InvalidLayerSpatial / InvalidLayerTemporal

struct Layer {
  i32 s, t;
  __device__ bool valid() const { return s != INV && t != INV; }
};

// getOptimalBandwidthNeeded forwarder.go:1857-1878
__device__ i64 optimal_bw(bool muted, bool pubMuted, i32 maxPub, const int64_t (*brs)[4], Layer max) {
  if (muted || pubMuted || maxPub == INV) return 0;
  for (i32 i = max.s; i >= 0; i--)
    for (i32 j = max.t; j >= 0; j--)
      if (brs[i][j] != 0) return brs[i][j];
  return 0;
}
// getBandwidthNeeded forwarder.go:1880-1886
__device__ i64 bw_needed(const int64_t (*brs)[4], Layer l, i64 fallback) {
  if (l.valid() && brs[l.s][l.t] > 0) return brs[l.s][l.t];
  return fallback;
}
// getDistanceToDesired forwarder.go:1888-1973 (availableLayers as a bit set:
// only its maximum matters)
__device__ double distance(bool muted, bool pubMuted, Layer seen, u32 avail, const int64_t (*brs)[4], Layer target,
                           Layer max) {
  if (muted || pubMuted || !seen.valid() || !max.valid()) return 0.0;
  Layer adj = max;
  i32 mas = INV, mat = INV;
  for (i32 s = 2; s >= 0 && mas == INV; s--)
    for (i32 t = 3; t >= 0; t--)
      if (brs[s][t] != 0) {
        mas = s;
        break;
      }
  if (avail) {
    const i32 hi = 31 - __clz(avail);
    if (hi > mas) {
      mas = hi;
      mat = seen.t;
    }
  }
  if (mas < adj.s) adj.s = mas;
  if (seen.s < adj.s) adj.s = seen.s;
  if (adj.s != INV)
    for (i32 t = 3; t >= 0; t--)
      if (brs[adj.s][t] != 0) {
        mat = t;
        break;
      }
  if (mat < adj.t) adj.t = mat;
  if (seen.t < adj.t) adj.t = seen.t;
  if (!adj.valid()) adj = Layer{0, 0};
  const Layer at = target.valid() ? target : Layer{0, 0};
  i32 d = ((adj.s - at.s) * (seen.t + 1)) + (adj.t - at.t);
  if (!target.valid()) d += seen.t + 1;
  return double(d) / double(seen.t + 1);
}

__global__ void k_allocate_optimal(const lkf_alloc_req *__restrict__ reqs, u32 n, DTHot *hot, const DevDT *dts,
                                   const DevTrack *tracks, int64_t *lastBw, lkf_allocation *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const lkf_alloc_req q = reqs[i];
  const u32 d = u32(q.dt);
  DTHot h = hot[d];
  lkf_allocation a = {};
  a.dt = q.dt;
  const bool muted = h.flags & F_MUTED, pubMuted = h.flags & F_PUBMUTED;
  if (!(h.flags & F_VIDEO)) {  // audio: lastAllocation, never updated (VideoAllocationDefault forwarder.go:111)
    a.pause_reason = 3;
    a.target_spatial = a.target_temporal = a.request_spatial = a.max_spatial = a.max_temporal = INV;
    out[i] = a;
    return;
  }
  const int64_t(*brs)[4] = q.bitrates;
  const Layer max{h.maxS, h.maxT}, seen{h.seenS, h.seenT}, cur{h.curS, h.curT}, oldTarget{h.tgtS, h.tgtT};
  const i32 reqSpatial = h.reqS;
  const bool overshoot = q.allow_overshoot && (h.flags & F_SIMULCAST);  // IsOvershootOkay: Simulcast only
  const u32 avail = q.available_layers;
  Layer target{INV, INV};
  i32 req = reqSpatial;
  i32 pause = 0;
  const i64 optimal = optimal_bw(muted, pubMuted, seen.s, brs, max);
  if (optimal == 0) pause = 3;  // VideoPauseReasonFeedDry
  const i32 maxT = (seen.t != INV && seen.t < max.t) ? seen.t : max.t;  // getMaxTemporal
  if (!max.valid() || seen.s == INV) {
  } else if (muted) {
    pause = 1;
  } else if (pubMuted) {
    pause = 2;
  } else {
    const i32 limit = min(max.s, seen.s);
    i32 highest = INV, request = INV;
    for (i32 l = 0; l < 32; l++)
      if (avail & (1u << l)) {
        if (l > request && l <= limit) request = l;
        if (l > highest) highest = l;
      }
    if (request == INV && highest != INV && overshoot) request = highest;
    if (cur.valid()) {
      if ((request == reqSpatial && cur.s == reqSpatial) || request == INV)
        target = Layer{cur.s, maxT};
      else
        target = Layer{request, maxT};
      req = target.s;
    } else {  // opportunistic
      i32 maxS = max.s;
      if (overshoot && seen.s > maxS) maxS = seen.s;
      target = Layer{min(seen.s, maxS), maxT};
      req = request == INV ? limit : request;
    }
  }
  if (!target.valid()) {
    target = Layer{INV, INV};
    req = INV;
  }
  const i64 bwr = target.valid() ? optimal : 0;
  a.pause_reason = pause;
  a.bandwidth_needed = optimal;
  a.bandwidth_requested = bwr;
  a.bandwidth_delta = bwr - bw_needed(brs, oldTarget, lastBw[d]);
  a.distance_to_desired = distance(muted, pubMuted, seen, avail, brs, target, max);
  // updateAllocation: H.264 has no temporal layers; setTargetLayer; resync if paused
  if (target.valid() && tracks[dts[d].track].codec == LKF_CODEC_H264) target.t = 0;
  a.target_spatial = target.s;
  a.target_temporal = target.t;
  a.request_spatial = req;
  a.max_spatial = max.s;
  a.max_temporal = max.t;
  a.is_deficient = 0;
  h.flags &= ~F_DEFICIENT;
  h.ptgtS = h.tgtS = target.s;
  h.ptgtT = h.tgtT = target.t;
  h.reqS = target.valid() ? req : INV;
  if (!target.valid()) {  // resyncLocked forwarder.go:1391-1397
    h.curS = h.curT = INV;
    h.lastSSRC = 0;
    if (h.flags & F_PUBMUTED) h.flags |= F_RESUME_BEHIND;
  }
  hot[d] = h;
  lastBw[d] = bwr;
  out[i] = a;
}
}  // namespace

hipError_t launch_allocate_optimal(hipStream_t s, const lkf_alloc_req *reqs, uint32_t n, DTHot *hot, const DevDT *dts,
                                   const DevTrack *tracks, int64_t *lastBw, lkf_allocation *out) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_allocate_optimal, dim3((n + 63) / 64), dim3(64), 0, s, reqs, n, hot, dts, tracks, lastBw, out);
  return hipGetLastError();
}

}  // namespace lkf
