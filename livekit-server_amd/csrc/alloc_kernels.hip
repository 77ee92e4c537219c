// alloc_kernels.hip — Forwarder.AllocateOptimal (forwarder.go:591-725),
// AllocateNextHigher (:1107-1217), GetNextHigherTransition (:1219-1306) and
// Pause (:1308-1351) + updateAllocation (:1353-1373) for many DownTracks at once (SURVEY.md §8(f)
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

// lastAllocation as the reference returns it: the stored VideoAllocation with
// IsDeficient as LKF_CTL_SET_ALLOCATION / the last allocation left F_DEFICIENT
__device__ lkf_allocation last_allocation(const lkf_allocation *last, u32 d, const DTHot &h) {
  lkf_allocation a = last[d];
  a.dt = i32(d);
  a.is_deficient = (h.flags & F_DEFICIENT) ? 1 : 0;
  a.boosted = 0;
  return a;
}

// updateAllocation forwarder.go:1353-1373 + setTargetLayer :1375-1382 +
// resyncLocked :1391-1397 when the target is invalid
__device__ void update_allocation(lkf_allocation &a, DTHot &h, bool h264, lkf_allocation *last, u32 d) {
  if (a.target_spatial != INV && a.target_temporal != INV && h264) a.target_temporal = 0;
  const bool valid = a.target_spatial != INV && a.target_temporal != INV;
  if (a.is_deficient)
    h.flags |= F_DEFICIENT;
  else
    h.flags &= ~F_DEFICIENT;
  h.ptgtS = h.tgtS = a.target_spatial;
  h.ptgtT = h.tgtT = a.target_temporal;
  h.reqS = valid ? a.request_spatial : INV;
  if (!valid) {
    h.curS = h.curT = INV;
    h.lastSSRC = 0;
    if (h.flags & F_PUBMUTED) h.flags |= F_RESUME_BEHIND;
  }
  last[d] = a;
}

__device__ bool is_h264(const DevDT *dts, const DevTrack *tracks, u32 d) {
  return tracks[dts[d].track].codec == LKF_CODEC_H264;
}

__global__ void k_allocate_optimal(const lkf_alloc_req *__restrict__ reqs, u32 n, DTHot *hot, const DevDT *dts,
                                   const DevTrack *tracks, lkf_allocation *last, lkf_allocation *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const lkf_alloc_req q = reqs[i];
  const u32 d = u32(q.dt);
  DTHot h = hot[d];
  if (!(h.flags & F_VIDEO)) {  // audio: lastAllocation, never updated (VideoAllocationDefault forwarder.go:111)
    out[i] = last_allocation(last, d, h);
    return;
  }
  lkf_allocation a = {};
  a.dt = q.dt;
  const bool muted = h.flags & F_MUTED, pubMuted = h.flags & F_PUBMUTED;
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
  a.bandwidth_delta = bwr - bw_needed(brs, oldTarget, last[d].bandwidth_requested);
  a.distance_to_desired = distance(muted, pubMuted, seen, avail, brs, target, max);
  a.target_spatial = target.s;
  a.target_temporal = target.t;
  a.request_spatial = req;
  a.max_spatial = max.s;
  a.max_temporal = max.t;
  a.is_deficient = 0;
  update_allocation(a, h, is_h264(dts, tracks, d), last, d);
  hot[d] = h;
  out[i] = a;
}

// AllocateNextHigher forwarder.go:1107-1217: temporal up in the target's
// spatial layer, then spatial up to the max layer, then (overshoot) above it;
// the first non-zero layer either fits the capacity and becomes the
// allocation, or ends the search unchanged.
__global__ void k_allocate_next_higher(const lkf_alloc_req *__restrict__ reqs, const int64_t *__restrict__ capacity,
                                       u32 n, DTHot *hot, const DevDT *dts, const DevTrack *tracks,
                                       lkf_allocation *last, lkf_allocation *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const lkf_alloc_req q = reqs[i];
  const u32 d = u32(q.dt);
  DTHot h = hot[d];
  out[i] = last_allocation(last, d, h);
  if (!(h.flags & F_VIDEO) || !(h.flags & F_DEFICIENT)) return;
  const Layer target{h.tgtS, h.tgtT}, cur{h.curS, h.curT};
  if (target.valid() && (target.s != cur.s || target.t != cur.t)) return;  // targets still pending
  const int64_t(*brs)[4] = q.bitrates;
  const bool muted = h.flags & F_MUTED, pubMuted = h.flags & F_PUBMUTED;
  const Layer max{h.maxS, h.maxT}, seen{h.seenS, h.seenT};
  const i64 optimal = optimal_bw(muted, pubMuted, seen.s, brs, max);
  const i64 already = target.valid() ? brs[target.s][target.t] : 0;
  const bool overshoot = q.allow_overshoot && (h.flags & F_SIMULCAST);
  const i64 cap = capacity[i];
  // the three searches of :1186-1214 as (minS, maxS, minT, maxT) ranges
  i32 rg[3][4];
  i32 nr = 0;
  if (target.valid()) {
    rg[nr][0] = target.s, rg[nr][1] = target.s, rg[nr][2] = target.t + 1, rg[nr][3] = max.t;
    nr++;
  }
  rg[nr][0] = target.s + 1, rg[nr][1] = max.s, rg[nr][2] = 0, rg[nr][3] = max.t;
  nr++;
  if (overshoot && max.valid()) {
    rg[nr][0] = max.s + 1, rg[nr][1] = 2, rg[nr][2] = 0, rg[nr][3] = 3;
    nr++;
  }
  for (i32 r = 0; r < nr; r++)
    for (i32 s = rg[r][0]; s <= rg[r][1]; s++)
      for (i32 t = rg[r][2]; t <= rg[r][3]; t++) {
        const i64 bwr = brs[s][t];
        if (bwr == 0) continue;
        if (!overshoot && bwr - already > cap) return;  // next higher layer does not fit
        lkf_allocation a = {};
        a.dt = q.dt;
        a.is_deficient = 1;
        a.bandwidth_requested = bwr;
        a.bandwidth_delta = bwr - already;
        a.bandwidth_needed = optimal;
        a.target_spatial = s;
        a.target_temporal = t;
        a.request_spatial = s;
        a.max_spatial = max.s;
        a.max_temporal = max.t;
        a.distance_to_desired = distance(muted, pubMuted, seen, q.available_layers, brs, Layer{s, t}, max);
        const bool greater = s > max.s || (s == max.s && t > max.t);  // VideoLayer.GreaterThan
        if (greater || bwr >= optimal) a.is_deficient = 0;
        update_allocation(a, h, is_h264(dts, tracks, d), last, d);
        hot[d] = h;
        a.boosted = 1;
        out[i] = a;
        return;
      }
}

// GetNextHigherTransition forwarder.go:1219-1306 (reads the state only)
__global__ void k_next_higher_transition(const lkf_alloc_req *__restrict__ reqs, u32 n, const DTHot *hot,
                                         lkf_video_transition *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const lkf_alloc_req q = reqs[i];
  const DTHot h = hot[u32(q.dt)];
  lkf_video_transition tr = {};
  tr.dt = q.dt;
  out[i] = tr;
  if (!(h.flags & F_VIDEO) || !(h.flags & F_DEFICIENT)) return;
  const Layer target{h.tgtS, h.tgtT}, cur{h.curS, h.curT}, max{h.maxS, h.maxT};
  if (target.valid() && (target.s != cur.s || target.t != cur.t)) return;
  const int64_t(*brs)[4] = q.bitrates;
  const i64 already = target.valid() ? brs[target.s][target.t] : 0;
  const bool overshoot = q.allow_overshoot && (h.flags & F_SIMULCAST);
  i32 rg[3][4];
  i32 nr = 0;
  if (target.valid()) {
    rg[nr][0] = target.s, rg[nr][1] = target.s, rg[nr][2] = target.t + 1, rg[nr][3] = max.t;
    nr++;
  }
  rg[nr][0] = target.s + 1, rg[nr][1] = max.s, rg[nr][2] = 0, rg[nr][3] = max.t;
  nr++;
  if (overshoot && max.valid()) {
    rg[nr][0] = max.s + 1, rg[nr][1] = 2, rg[nr][2] = 0, rg[nr][3] = 3;
    nr++;
  }
  for (i32 r = 0; r < nr; r++)
    for (i32 s = rg[r][0]; s <= rg[r][1]; s++)
      for (i32 t = rg[r][2]; t <= rg[r][3]; t++) {
        const i64 bwr = brs[s][t];
        if (bwr == 0 || bwr < already) continue;
        tr.from_spatial = target.s;
        tr.from_temporal = target.t;
        tr.to_spatial = s;
        tr.to_temporal = t;
        tr.bandwidth_delta = bwr - already;
        tr.available = 1;
        out[i] = tr;
        return;
      }
}

// Pause forwarder.go:1308-1351
__global__ void k_pause(const lkf_alloc_req *__restrict__ reqs, u32 n, DTHot *hot, const DevDT *dts,
                        const DevTrack *tracks, lkf_allocation *last, lkf_allocation *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const lkf_alloc_req q = reqs[i];
  const u32 d = u32(q.dt);
  DTHot h = hot[d];
  if (!(h.flags & F_VIDEO)) {  // audio: lastAllocation, no state change (as AllocateOptimal; the
    out[i] = last_allocation(last, d, h);  // reference's Pause needs the video layer selector)
    return;
  }
  const int64_t(*brs)[4] = q.bitrates;
  const bool muted = h.flags & F_MUTED, pubMuted = h.flags & F_PUBMUTED;
  const Layer max{h.maxS, h.maxT}, seen{h.seenS, h.seenT}, target{h.tgtS, h.tgtT};
  const i64 optimal = optimal_bw(muted, pubMuted, seen.s, brs, max);
  lkf_allocation a = {};
  a.dt = q.dt;
  a.bandwidth_delta = 0 - bw_needed(brs, target, last[d].bandwidth_requested);
  a.bandwidth_needed = optimal;
  a.target_spatial = a.target_temporal = a.request_spatial = INV;
  a.max_spatial = max.s;
  a.max_temporal = max.t;
  a.distance_to_desired = distance(muted, pubMuted, seen, q.available_layers, brs, Layer{INV, INV}, max);
  if (muted)
    a.pause_reason = 1;
  else if (pubMuted)
    a.pause_reason = 2;
  else if (optimal == 0)
    a.pause_reason = 3;
  else {
    a.is_deficient = 1;
    a.pause_reason = 4;
  }
  update_allocation(a, h, is_h264(dts, tracks, d), last, d);
  hot[d] = h;
  out[i] = a;
}
}  // namespace

hipError_t launch_allocate(hipStream_t s, int mode, const lkf_alloc_req *reqs, const int64_t *capacity, uint32_t n,
                           DTHot *hot, const DevDT *dts, const DevTrack *tracks, lkf_allocation *last, void *out) {
  if (!n) return hipSuccess;
  const dim3 g((n + 63) / 64), b(64);
  switch (mode) {
    case ALLOC_OPTIMAL:
      hipLaunchKernelGGL(k_allocate_optimal, g, b, 0, s, reqs, n, hot, dts, tracks, last,
                         static_cast<lkf_allocation *>(out));
      break;
    case ALLOC_NEXT_HIGHER:
      hipLaunchKernelGGL(k_allocate_next_higher, g, b, 0, s, reqs, capacity, n, hot, dts, tracks, last,
                         static_cast<lkf_allocation *>(out));
      break;
    case ALLOC_TRANSITION:
      hipLaunchKernelGGL(k_next_higher_transition, g, b, 0, s, reqs, n, hot, static_cast<lkf_video_transition *>(out));
      break;
    case ALLOC_PAUSE:
      hipLaunchKernelGGL(k_pause, g, b, 0, s, reqs, n, hot, dts, tracks, last, static_cast<lkf_allocation *>(out));
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lkf
