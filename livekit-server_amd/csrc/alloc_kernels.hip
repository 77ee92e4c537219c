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

// ---- the stream allocator's cooperative pass (forwarder.go:727-1105) --------
__device__ __forceinline__ bool greater(Layer a, Layer b) {  // VideoLayer.GreaterThan
  return a.s > b.s || (a.s == b.s && a.t > b.t);
}
// ProvisionalAllocatePrepare :727-743
__device__ void prov_prepare(const DTHot &h, ProvState &p, const lkf_alloc_req &q) {
  for (int s = 0; s < 3; s++)
    for (int t = 0; t < 4; t++) p.brs[s][t] = q.bitrates[s][t];
  p.allocS = p.allocT = INV;
  p.muted = ((h.flags & F_MUTED) ? 1u : 0u) | ((h.flags & F_PUBMUTED) ? 2u : 0u);
  p.seenS = h.seenS, p.seenT = h.seenT;
  p.maxS = h.maxS, p.maxT = h.maxT;
  p.curS = h.curS, p.curT = h.curT;
  p.avail = q.available_layers;
}
// ProvisionalAllocate :752-794
__device__ bool prov_allocate(const DTHot &h, ProvState &p, i64 cap, Layer layer, bool allowPause, bool allowOvershoot,
                              i64 &used) {
  used = 0;
  const Layer max{p.maxS, p.maxT}, al{p.allocS, p.allocT};
  const bool ovOk = allowOvershoot && (h.flags & F_SIMULCAST);  // IsOvershootOkay: Simulcast only
  if (p.muted || p.seenS == INV || !max.valid() || (!ovOk && greater(layer, max))) return false;
  const i64 required = p.brs[layer.s][layer.t];
  if (required == 0) return false;
  const i64 already = al.valid() ? p.brs[al.s][al.t] : 0;
  if (!greater(layer, max) && required <= cap + already) {
    p.allocS = layer.s, p.allocT = layer.t;
    used = required - already;
    return true;
  }
  if (!allowPause && (!al.valid() || !greater(layer, al))) {
    p.allocS = layer.s, p.allocT = layer.t;
    used = required - already;
    return true;
  }
  return false;
}
__device__ lkf_video_transition transition(i32 dt, Layer from, Layer to, i64 delta) {
  lkf_video_transition tr = {};
  tr.dt = dt;
  tr.from_spatial = from.s, tr.from_temporal = from.t;
  tr.to_spatial = to.s, tr.to_temporal = to.t;
  tr.bandwidth_delta = delta;
  tr.available = 1;
  return tr;
}
// ProvisionalAllocateGetCooperativeTransition :796-929
__device__ lkf_video_transition prov_cooperative(i32 dt, const DTHot &h, ProvState &p, i64 lastReq, bool allowOvershoot) {
  const Layer existing{h.tgtS, h.tgtT}, max{p.maxS, p.maxT}, cur{p.curS, p.curT};
  if (p.muted) {
    p.allocS = p.allocT = INV;
    return transition(dt, existing, Layer{INV, INV}, -bw_needed(p.brs, existing, lastReq));
  }
  if (existing.valid()) {
    Layer maximal{INV, INV};
    i64 maximalBw = 0;
    for (i32 s = max.s; s >= 0 && maximalBw == 0; s--)
      for (i32 t = max.t; t >= 0; t--)
        if (p.brs[s][t] != 0) {
          maximal = Layer{s, t};
          maximalBw = p.brs[s][t];
          break;
        }
    if (maximal.valid()) {
      if (!greater(existing, maximal) && p.brs[existing.s][existing.t] != 0) {
        p.allocS = existing.s, p.allocT = existing.t;
        return transition(dt, existing, existing, 0);
      }
      if (greater(existing, maximal)) {
        p.allocS = maximal.s, p.allocT = maximal.t;
        return transition(dt, existing, maximal, maximalBw - bw_needed(p.brs, existing, lastReq));
      }
    }
  }
  Layer target{INV, INV};
  i64 required = 0;
  auto next = [&](i32 minS, i32 maxS, i32 minT, i32 maxT) {
    for (i32 s = minS; s <= maxS && required == 0; s++)
      for (i32 t = minT; t <= maxT; t++)
        if (p.brs[s][t] != 0) {
          target = Layer{s, t};
          required = p.brs[s][t];
          break;
        }
  };
  if (!existing.valid()) {
    next(0, max.s, 0, max.t);
    if (required == 0 && max.valid() && allowOvershoot && (h.flags & F_SIMULCAST)) {
      target = Layer{INV, INV};
      next(max.s + 1, 2, 0, 3);
    }
  }
  if (!target.valid()) {
    target = cur;
    if (target.valid()) required = p.brs[target.s][target.t];
  }
  p.allocS = target.s, p.allocT = target.t;
  return transition(dt, existing, target, required - bw_needed(p.brs, existing, lastReq));
}
// ProvisionalAllocateGetBestWeightedTransition :931-1025
__device__ lkf_video_transition prov_best_weighted(i32 dt, const DTHot &h, ProvState &p, i64 lastReq) {
  const Layer target{h.tgtS, h.tgtT}, max{p.maxS, p.maxT};
  if (p.muted) {
    p.allocS = p.allocT = INV;
    return transition(dt, target, Layer{INV, INV}, 0 - bw_needed(p.brs, target, lastReq));
  }
  i32 reachT = INV;
  for (i32 t = max.t; t >= 0 && reachT == INV; t--)
    for (i32 s = max.s; s >= 0; s--)
      if (p.brs[s][t] != 0) {
        reachT = t;
        break;
      }
  if (reachT == INV) {
    p.allocS = p.curS, p.allocT = p.curT;
    return transition(dt, target, Layer{p.curS, p.curT}, 0 - bw_needed(p.brs, target, lastReq));
  }
  const i64 existingBw = bw_needed(p.brs, target, lastReq);
  Layer best{INV, INV};
  i64 bestDelta = 0;
  float bestValue = 0.0f;
  for (i32 s = 0; s <= target.s; s++)
    for (i32 t = 0; t <= target.t; t++) {
      if (s == target.s && t == target.t) break;
      const i64 delta = i64(fmax(0.0, double(existingBw - p.brs[s][t])));
      const i32 transitionCost = target.s != s ? 10 : 0;  // TransitionCostSpatial forwarder.go:43
      const i32 qualityCost = (reachT + 1) * (target.s - s) + (target.t - t);
      float value = 0.0f;
      if (transitionCost + qualityCost != 0) value = float(delta) / float(transitionCost + qualityCost);
      if (value > bestValue || (value == bestValue && delta > bestDelta)) {
        bestValue = value;
        bestDelta = delta;
        best = Layer{s, t};
      }
    }
  p.allocS = best.s, p.allocT = best.t;
  return transition(dt, target, best, -bestDelta);
}
// ProvisionalAllocateCommit :1027-1105 (+ updateAllocation)
__device__ lkf_allocation prov_commit(i32 dt, DTHot &h, ProvState &p, bool h264, lkf_allocation *last, u32 d) {
  const bool muted = p.muted & 1, pubMuted = p.muted & 2;
  const Layer max{p.maxS, p.maxT}, seen{p.seenS, p.seenT}, cur{p.curS, p.curT}, target{h.tgtS, h.tgtT};
  const i64 lastReq = last[d].bandwidth_requested;
  const i64 optimal = optimal_bw(muted, pubMuted, seen.s, p.brs, max);
  lkf_allocation a = {};
  a.dt = dt;
  a.bandwidth_requested = 0;
  a.bandwidth_delta = 0 - bw_needed(p.brs, target, lastReq);
  a.bandwidth_needed = optimal;
  Layer al{p.allocS, p.allocT};
  a.target_spatial = al.s, a.target_temporal = al.t;
  a.request_spatial = al.s;
  a.max_spatial = max.s, a.max_temporal = max.t;
  a.distance_to_desired = distance(muted, pubMuted, seen, p.avail, p.brs, al, max);
  if (muted) {
    a.pause_reason = 1;
  } else if (pubMuted) {
    a.pause_reason = 2;
  } else if (optimal == 0) {
    if (al.valid()) {  // overshoot
      a.bandwidth_requested = p.brs[al.s][al.t];
      a.bandwidth_delta = a.bandwidth_requested - bw_needed(p.brs, target, lastReq);
    } else {
      a.pause_reason = 3;
      if (cur.valid() && cur.s <= max.s) {  // leave target at current for opportunistic forwarding
        p.allocS = cur.s, p.allocT = cur.t;
        a.target_spatial = cur.s, a.target_temporal = cur.t;
        a.request_spatial = cur.s;
      }
    }
  } else {
    if (al.valid()) a.bandwidth_requested = p.brs[al.s][al.t];
    a.bandwidth_delta = a.bandwidth_requested - bw_needed(p.brs, target, lastReq);
    if (greater(al, max) || a.bandwidth_requested >= optimal) {
      a.is_deficient = 0;
    } else {
      a.is_deficient = 1;
      if (!al.valid()) a.pause_reason = 4;
    }
  }
  update_allocation(a, h, h264, last, d);
  return a;
}

__global__ void k_prov(ProvLaunch A) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n) return;
  const i32 dt = A.mode == PROV_PREPARE ? A.alloc[i].dt : A.reqs[i].dt;
  const u32 d = u32(dt);
  DTHot h = A.hot[d];
  ProvState p = A.prov[d];
  switch (A.mode) {
    case PROV_PREPARE:
      prov_prepare(h, p, A.alloc[i]);
      break;
    case PROV_RESET:
      p.allocS = p.allocT = INV;
      break;
    case PROV_ALLOCATE: {
      const lkf_prov_req q = A.reqs[i];
      lkf_prov_result r = {};
      r.dt = dt;
      const bool ok = q.spatial >= 0 && q.spatial <= 2 && q.temporal >= 0 && q.temporal <= 3;
      r.is_candidate = ok && prov_allocate(h, p, q.capacity, Layer{q.spatial, q.temporal}, q.allow_pause != 0,
                                           q.allow_overshoot != 0, r.used);
      static_cast<lkf_prov_result *>(A.out)[i] = r;
      break;
    }
    case PROV_COOPERATIVE:
      static_cast<lkf_video_transition *>(A.out)[i] =
          prov_cooperative(dt, h, p, A.last[d].bandwidth_requested, A.reqs[i].allow_overshoot != 0);
      break;
    case PROV_BEST_WEIGHTED:
      static_cast<lkf_video_transition *>(A.out)[i] = prov_best_weighted(dt, h, p, A.last[d].bandwidth_requested);
      break;
    case PROV_COMMIT:
      static_cast<lkf_allocation *>(A.out)[i] = prov_commit(dt, h, p, is_h264(A.dts, A.tracks, d), A.last, d);
      A.hot[d] = h;
      break;
  }
  A.prov[d] = p;
}

// allocateAllTracks' managed pass (streamallocator.go:1147-1172): one thread
// per subscriber group, serial over its layers and DownTracks
__global__ void k_allocate_all(const lkf_alloc_group *__restrict__ groups, u32 ngroups,
                               const lkf_alloc_req *__restrict__ reqs, DTHot *hot, const DevDT *dts,
                               const DevTrack *tracks, lkf_allocation *last, ProvState *prov, lkf_allocation *out) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  const lkf_alloc_group G = groups[g];
  for (u32 k = 0; k < G.count; k++) {
    const u32 d = u32(reqs[G.first + k].dt);
    ProvState p;
    prov_prepare(hot[d], p, reqs[G.first + k]);
    prov[d] = p;
  }
  i64 cap = G.capacity;
  for (i32 s = 0; s <= 2; s++)
    for (i32 t = 0; t <= 3; t++)
      for (u32 k = 0; k < G.count; k++) {
        const u32 d = u32(reqs[G.first + k].dt);
        i64 used = 0;
        prov_allocate(hot[d], prov[d], cap, Layer{s, t}, G.allow_pause != 0, G.allow_overshoot != 0, used);
        cap -= used;
        if (cap < 0) cap = 0;
      }
  for (u32 k = 0; k < G.count; k++) {
    const u32 d = u32(reqs[G.first + k].dt);
    DTHot h = hot[d];
    ProvState p = prov[d];
    out[G.first + k] = prov_commit(i32(d), h, p, is_h264(dts, tracks, d), last, d);
    hot[d] = h;
    prov[d] = p;
  }
}
}  // namespace

hipError_t launch_prov(hipStream_t s, const ProvLaunch &a) {
  if (!a.n) return hipSuccess;
  hipLaunchKernelGGL(k_prov, dim3((a.n + 63) / 64), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_allocate_all(hipStream_t s, const lkf_alloc_group *groups, uint32_t ngroups, const lkf_alloc_req *reqs,
                               DTHot *hot, const DevDT *dts, const DevTrack *tracks, lkf_allocation *last,
                               ProvState *prov, lkf_allocation *out) {
  if (!ngroups) return hipSuccess;
  hipLaunchKernelGGL(k_allocate_all, dim3((ngroups + 63) / 64), dim3(64), 0, s, groups, ngroups, reqs, hot, dts, tracks,
                     last, prov, out);
  return hipGetLastError();
}

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
