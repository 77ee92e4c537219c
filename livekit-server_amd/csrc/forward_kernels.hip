// forward_kernels.hip — gfx950 kernels of the batched RTP forwarding engine.
//
// Per batch (lkf_run):
//   k_track_ranges  packets grouped by track -> [begin,end) per track
//   scan (slots)    per DownTrack tuple-slot base = sum of its track's packets
//   k_decide_dt     one wave per DownTrack, lanes = its track's packets:
//                   the per-packet recurrence of DownTrack.WriteRTP
//                   (downtrack.go:680-760) = Forwarder.GetTranslationParams
//                   (forwarder.go:1436-1765) + RTPMunger (rtpmunger.go) +
//                   Simulcast/VP8-temporal selectors + VP8 munger
//                   (codecmunger/vp8.go) + sequencer.push (sequencer.go:123)
//                   -> compact per-DownTrack FwdRec records (24 B), with
//                   RTPStatsSender.Update folded in (ss_flush)
//   scan (output)   per DownTrack record base + byte base (16-B aligned wire
//                   packets; order: track, then DownTrack, then packet)
//   k_emit          flat 16-B chunk sweep over the output arena: RTP header +
//                   extension block + munged VP8 descriptor from LDS, payload
//                   copied byte-shifted from the input arena (coalesced
//                   dwordx4 loads/stores); one lkf_out record per tuple.
//
// No MFMA: nothing here is a contraction.  The emit kernel is HBM-bound
// (writes ~ out bytes, input payload re-reads served from L2/MALL).
#include <hip/hip_runtime.h>

#include "../../include/lkfwd.h"
#ifndef LKF_SVC_STATS
#define LKF_SVC_STATS 0
#endif
#if LKF_SVC_STATS  // (diagnostic builds: the counters, below at svc_run)
__device__ unsigned long long g_svc[64 * 48];  // 64 copies (by workgroup) of 48 counters
#define SVC_ADD(k, v) atomicAdd(&g_svc[(blockIdx.x & 63) * 48 + (k)], (unsigned long long)(v))
#endif
#include "dd_device.h"
#include "fwd_state.h"
#include "kernels.h"
#include "sender_device.h"

namespace lkf {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i32 = int32_t;
using i64 = int64_t;

constexpr u64 HALF64 = 1ull << 63;
constexpr i32 INVALID = -1;


// ---------------------------------------------------------------------------
// Checked builds (-DLKF_CHECKED=1, liblkfwd_checked.so): every global access
// whose index is computed on the device is tested against the capacity of
// its allocation; the first violation (site, index, capacity) and the count
// go to g_chk (lkf_debug_check).  The access itself still happens, so a
// checked run behaves like the product build, but an out-of-bounds index is
// reported even when it lands in mapped memory (the usual case, which a
// product run never notices).
// ---------------------------------------------------------------------------
#ifndef LKF_CHECKED
#define LKF_CHECKED 0
#endif
#if LKF_CHECKED
__device__ unsigned long long g_chk[4];
__device__ __noinline__ void chk_fail(u32 site, u64 idx, u64 cap) {
  if (atomicAdd(&g_chk[0], 1ull) == 0) {
    g_chk[1] = site;
    g_chk[2] = idx;
    g_chk[3] = cap;
  }
}
#define CHK(cond, site, idx, cap)                   \
  do {                                              \
    if (!(cond)) chk_fail(site, u64(idx), u64(cap)); \
  } while (0)
#else
#define CHK(cond, site, idx, cap) \
  do {                            \
  } while (0)
#endif
enum ChkSite : u32 {
  CK_DEC_DT = 1,      // decide: DownTrack handle < max_downtracks
  CK_DEC_TRACK,       // decide: track < max_tracks
  CK_DEC_PKT,         // decide: packet index < batch packets
  CK_DEC_TUPLE,       // decide: tuple slot < max_batch_tuples
  CK_DEC_SEQ,         // decide: sequencer slot < seq_size
  CK_DEC_LAYER,       // decide: layer-list index < 3 * max_batch_pkts
  CK_DEC_EVENT,       // decide: control-op index < ops of the batch
  CK_EMIT_POS,        // emit: output position < DownTracks
  CK_EMIT_DT,         // emit: DownTrack handle < max_downtracks
  CK_EMIT_TUPLE,      // emit: tuple slot < max_batch_tuples
  CK_EMIT_PKT,        // emit: packet index < batch packets
  CK_EMIT_ARENA,      // emit: payload read end <= arena length + 64
  CK_EMIT_OUT,        // emit: record < max_out_pkts
  CK_EMIT_BYTES,      // emit: wire byte end <= max_out_bytes + 64
  CK_EMIT_DD,         // emit: DD arena read end <= its capacity
  CK_EMIT_GROUP,      // emit: group index entry < its capacity
  CK_PAD_DT,          // padding: DownTrack handle < max_downtracks
  CK_PAD_SEQ,         // padding: sequencer slot < seq_size
};

// ---------------------------------------------------------------------------
// Packet view (lkf_pkt, 64 B) loaded with 4 x 16-B loads.
// ---------------------------------------------------------------------------
struct PktV {
  u64 esn, ets;
  i64 arr;
  u32 arenaOff, ssrc;
  u16 poff, plen;
  u8 hdr0, hdr1, flags, vfirst, vbits, vhs, tl0, tid, keyidx, vp9;
  int8_t spatial, temporal, layer;
  u16 pid;
};

__device__ __forceinline__ PktV decode_pkt(uint4 a, uint4 b, uint4 c, uint4 d) {
  PktV v;
  v.esn = (u64(a.y) << 32) | a.x;
  v.ets = (u64(a.w) << 32) | a.z;
  v.arr = i64((u64(b.y) << 32) | b.x);
  v.arenaOff = b.z;
  // b.w = track
  v.ssrc = c.x;
  v.poff = u16(c.y & 0xffff);
  v.plen = u16(c.y >> 16);
  v.hdr0 = u8(c.z);
  v.hdr1 = u8(c.z >> 8);
  v.spatial = int8_t(c.z >> 16);
  v.temporal = int8_t(c.z >> 24);
  v.flags = u8(c.w);
  v.vfirst = u8(c.w >> 8);
  v.vbits = u8(c.w >> 16);
  v.vhs = u8(c.w >> 24);
  v.pid = u16(d.x & 0xffff);
  v.tl0 = u8(d.x >> 16);
  v.tid = u8(d.x >> 24);
  v.keyidx = u8(d.y);
  v.layer = int8_t(d.y >> 8);
  v.vp9 = u8(d.y >> 24);
  return v;
}

__device__ __forceinline__ PktV load_pkt(const lkf_pkt *p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  return decode_pkt(q[0], q[1], q[2], q[3]);
}

__device__ __forceinline__ uint4 rfl(uint4 v) {  // wave-uniform copy (SGPRs)
  v.x = __builtin_amdgcn_readfirstlane(v.x);
  v.y = __builtin_amdgcn_readfirstlane(v.y);
  v.z = __builtin_amdgcn_readfirstlane(v.z);
  v.w = __builtin_amdgcn_readfirstlane(v.w);
  return v;
}

// ---------------------------------------------------------------------------
// Wave primitives.  k_decide_dt runs one wave per DownTrack: the DownTrack
// state is wave-uniform, so the rare-path helpers below spread their loops
// over the 64 lanes (every lane calls them with the same arguments).
// ---------------------------------------------------------------------------
__device__ __forceinline__ u32 lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ u32 rl32(u32 v, u32 l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ u64 rl64(u64 v, u32 l) {
  return (u64(rl32(u32(v >> 32), l)) << 32) | u64(rl32(u32(v), l));
}
__device__ __forceinline__ u32 sh32(u32 v, int src) { return u32(__shfl(int(v), src, 64)); }
__device__ __forceinline__ u64 sh64(u64 v, int src) {
  return (u64(sh32(u32(v >> 32), src)) << 32) | u64(sh32(u32(v), src));
}
__device__ __forceinline__ int prev_in(u64 m, u64 lt) {  // highest set lane below this one, or -1
  const u64 pm = m & lt;
  return pm ? 63 - __clzll(pm) : -1;
}
__device__ __forceinline__ u32 excl_scan_u32(u32 v, u32 lane) {
  u32 x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    u32 y = u32(__shfl_up(int(x), o, 64));
    if (lane >= u32(o)) x += y;
  }
  return x - v;
}
__device__ __forceinline__ u32 wave_sum_u32(u32 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += u32(__shfl_xor(int(v), o, 64));
  return v;
}
__device__ __forceinline__ u64 wave_max_u64(u64 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    u64 y = sh64(v, int(threadIdx.x) ^ o);
    v = y > v ? y : v;
  }
  return v;
}

__device__ __forceinline__ u64 wave_or_u64(u64 v) {  // -> wave-uniform (SGPR) result
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= sh64(v, int(threadIdx.x) ^ o);
  return rl64(v, 0);
}
// LDS written by some lanes is read by others below: order the accesses
// (the workgroup is one wave, so the barrier costs no waiting).
__device__ __forceinline__ void wave_lds_sync() { __syncthreads(); }

// ---------------------------------------------------------------------------
// Lane context: hot state in registers + cold-state pointers.
// ---------------------------------------------------------------------------
struct Lane {
  DTHot &h;  // the wave's DownTrack state, staged in LDS (no SGPR pressure / spill traffic)
  RangeEntry *rm;  // the closed-range ring (decide: in LDS, filled on first lookup; padding: HBM)
  RangeEntry *rmG; // the ring in HBM
  u32 rmNew;       // closed ranges appended since the ring was staged (the newest ones; written back)
  bool rmLoaded;   // the older live ranges are in L.rm (rm_load)
  bool vcDirty;    // a VP8 munger map changed (write the maps back)
  VP8Cold *vc;
  i32 *dropKey;  // LDS copy of vc->dropKey
  i32 *exKey;    // LDS copy of vc->exKey
  i32 *missKey;  // LDS copy of vc->missKey
  i32 *missVal;
  SeqMeta *seq;
  u32 seqSize;
  SeqRM *srm;  // the sequencer's RangeMap region (read only with F_SEQ_RM)
  u32 srmCap;
  // track
  u32 kind, codec, hasRefTS, clockRate;
  u32 *offs;  // the DownTrack's reference-layer offsets row (HBM; read on a source switch)
  // static DT
  u8 extPlayout, extAbs, extDD, extTcc;
  // dependency-descriptor selector (F_DD): state staged in LDS, the track's
  // structure ring, this batch's decoded descriptors, the marshal buffer
  DDState *dd;
  const DDStruct *ddRing;
  DDStruct *ddS;  // LDS copy of ring slot ddSSlot (the structure in force: staged again when it changes)
  u32 ddSSlot;
  const DDPkt *ddPkts;
  const u16 *ddSpill;
  u8 *ddBuf;
  DDPkt *ddPktL;  // LDS: the full step's descriptor (dd_select reads it there, not from HBM)
  u32 *err;
};

__device__ __forceinline__ bool hasf(const Lane &L, u32 f) { return (L.h.flags & f) != 0; }
__device__ __forceinline__ void setf(Lane &L, u32 f, bool v) {
  if (v)
    L.h.flags |= f;
  else
    L.h.flags &= ~f;
}

// ---- utils.RangeMap<u64,u64>(100): open range in registers, closed ring --
__device__ __forceinline__ RangeEntry rm_at(const Lane &L, int i) {  // i-th closed range (oldest = 0)
  int idx = (int(L.h.rmHead) + i) % kRangeCap;
  return L.rm[idx];
}
// The decide wave stages the ring lazily: the common path only appends
// (rm_exclude) and never reads it, so the live ranges older than this batch's
// appends come from HBM only when a lookup first needs them (wave-uniform).
__device__ __forceinline__ void rm_load(Lane &L) {
  if (L.rmLoaded) return;
  L.rmLoaded = true;
  const u32 nc = L.h.rmCount, old = nc - min(L.rmNew, nc);
  if (!old) return;
  wave_lds_sync();
  for (u32 i = lane_id(); i < old; i += 64) {
    const u32 idx = (u32(L.h.rmHead) + i) % kRangeCap;
    L.rm[idx] = L.rmG[idx];
  }
  wave_lds_sync();
}
// ClearAndResetValue rangemap.go:66
__device__ __forceinline__ void rm_reset(Lane &L, u64 start, u64 val) {
  L.h.rmHead = 0;
  L.h.rmCount = 0;
  L.rmNew = 0;  // (no live range left to stage or write back)
  L.h.rmOpenStart = start;
  L.h.rmOpenValue = val;
}
// ExcludeRange rangemap.go:100-132
__device__ __forceinline__ bool rm_exclude(Lane &L, u64 s, u64 e) {
  if (e == s || (e - s) > HALF64) return false;
  if (L.h.rmOpenStart > s) return false;
  u64 nv = L.h.rmOpenValue + (e - s);
  if (L.h.rmOpenStart == s) {
    L.h.rmOpenStart = e;
    L.h.rmOpenValue = nv;
    return true;
  }
  RangeEntry c;
  c.start = L.h.rmOpenStart;
  c.end = s - 1;
  c.value = L.h.rmOpenValue;
  if (L.h.rmCount < kRangeCap) {
    int idx = (int(L.h.rmHead) + int(L.h.rmCount)) % kRangeCap;
    L.rm[idx] = c;
    L.h.rmCount++;
  } else {  // prune rangemap.go:171: keep the newest size+1 (100 closed + open)
    L.rm[L.h.rmHead] = c;
    L.h.rmHead = u16((L.h.rmHead + 1) % kRangeCap);
  }
  L.rmNew++;
  L.h.rmOpenStart = e;
  L.h.rmOpenValue = nv;
  return true;
}
// GetValue rangemap.go:134-169 -> true on success.  The reference walks the
// closed ranges from the newest down; at index i it first tests "key inside
// range i", then "key strictly between range i-1 and range i" (-> miss).  The
// first hit of that walk is the hit with the largest index (inside before
// between at equal index), so each lane tests one index and a ballot picks it.
__device__ __forceinline__ bool rm_get(Lane &L, u64 key, u64 &out) {
  out = 0;
  if (key >= L.h.rmOpenStart) {
    out = L.h.rmOpenValue;
    return true;
  }
  const int nc = L.h.rmCount;
  if (nc == 0) return false;  // key < open start = first start
  rm_load(L);
  if (key < rm_at(L, 0).start) return false;
  const u32 l = lane_id();
  int best = -1;
  bool bestIn = false;
  u64 bestVal = 0;
  for (int base = 0; base <= nc; base += 64) {
    const int i = base + int(l);
    bool in = false, between = false;
    u64 val = 0;
    if (i <= nc) {
      u64 nextStart = L.h.rmOpenStart;
      if (i < nc) {
        const RangeEntry rv = rm_at(L, i);
        in = (key - rv.start) < HALF64 && (rv.end - key) < HALF64;
        val = rv.value;
        nextStart = rv.start;
      }
      if (i > 0) {
        const u64 before = key - rm_at(L, i - 1).end;
        const u64 after = nextStart - key;
        between = before > 0 && before < HALF64 && after > 0 && after < HALF64;
      }
    }
    const u64 m = __ballot(in || between);
    if (m) {
      const u32 j = 63 - __clzll(m);
      best = base + int(j);
      bestIn = rl32(u32(in), j) != 0;
      bestVal = rl64(val, j);
    }
  }
  if (best < 0 || !bestIn) return false;
  out = bestVal;
  return true;
}

// ---- RTPMunger (rtpmunger.go) ---------------------------------------------
__device__ __forceinline__ void mg_updateSnOffset(Lane &L) {  // :352-358
  u64 v = 0;
  rm_get(L, L.h.extHighestIncomingSN + 1, v);
  L.h.snOffset = v;
}
__device__ __forceinline__ void mg_setLastSnTs(Lane &L, u64 esn, u64 ets) {  // :135-145
  L.h.extHighestIncomingSN = esn - 1;
  L.h.extLastSN = esn;
  L.h.extSecondLastSN = esn - 1;
  rm_reset(L, esn, 0);
  mg_updateSnOffset(L);
  L.h.extLastTS = ets;
  L.h.extSecondLastTS = ets;
}
__device__ __forceinline__ void mg_updateSnTsOffsets(Lane &L, u64 esn, u64 ets, u64 snAdj, u64 tsAdj) {  // :147
  L.h.extHighestIncomingSN = esn - 1;
  rm_reset(L, esn, esn - L.h.extLastSN - snAdj);
  mg_updateSnOffset(L);
  L.h.tsOffset = ets - L.h.extLastTS - tsAdj;
}
__device__ __forceinline__ void mg_packetDropped(Lane &L, u64 esn) {  // :156-181
  if (L.h.extHighestIncomingSN != esn) return;
  rm_exclude(L, L.h.extHighestIncomingSN, L.h.extHighestIncomingSN + 1);
  L.h.extLastSN = L.h.extSecondLastSN;
  mg_updateSnOffset(L);
  L.h.extLastTS = L.h.extSecondLastTS;
  setf(L, F_LAST_MARKER, hasf(L, F_SECOND_LAST_MARKER));
}
enum { ORD_CONTIG = 0, ORD_OOO = 1, ORD_GAP = 2, ORD_DUP = 3 };
enum { MG_OK = 0, MG_PADDING, MG_DUP, MG_OOO_MISS };
// UpdateAndGetSnTs :183-271
// in-order branch of UpdateAndGetSnTs (rtpmunger.go:186-217), diff >= 1
__device__ __forceinline__ void mg_inorder(Lane &L, const PktV &p, bool marker, u64 &osn, u64 &ots) {
  L.h.extHighestIncomingSN = p.esn;
  u64 msn = p.esn - L.h.snOffset;
  u64 mts = p.ets - L.h.tsOffset;
  L.h.extSecondLastSN = L.h.extLastSN;
  L.h.extLastSN = msn;
  L.h.extSecondLastTS = L.h.extLastTS;
  L.h.extLastTS = mts;
  setf(L, F_SECOND_LAST_MARKER, hasf(L, F_LAST_MARKER));
  setf(L, F_LAST_MARKER, marker);
  if (p.flags & LKF_PKT_KEYFRAME) {
    L.h.extRtxGateSn = msn;
    setf(L, F_RTX_GATE, true);
  }
  if (hasf(L, F_RTX_GATE) && (msn - L.h.extRtxGateSn) > 2000) setf(L, F_RTX_GATE, false);
  osn = msn;
  ots = mts;
}

__device__ int mg_update(Lane &L, const PktV &p, bool marker, int &ord, u64 &osn, u64 &ots) {
  i64 diff = i64(p.esn - L.h.extHighestIncomingSN);
  if ((diff == 1 && p.plen != 0) || diff > 1) {
    L.h.extHighestIncomingSN = p.esn;
    ord = diff > 1 ? ORD_GAP : ORD_CONTIG;
    u64 msn = p.esn - L.h.snOffset;
    u64 mts = p.ets - L.h.tsOffset;
    L.h.extSecondLastSN = L.h.extLastSN;
    L.h.extLastSN = msn;
    L.h.extSecondLastTS = L.h.extLastTS;
    L.h.extLastTS = mts;
    setf(L, F_SECOND_LAST_MARKER, hasf(L, F_LAST_MARKER));
    setf(L, F_LAST_MARKER, marker);
    if (p.flags & LKF_PKT_KEYFRAME) {
      L.h.extRtxGateSn = msn;
      setf(L, F_RTX_GATE, true);
    }
    if (hasf(L, F_RTX_GATE) && (msn - L.h.extRtxGateSn) > 2000) setf(L, F_RTX_GATE, false);
    osn = msn;
    ots = mts;
    return MG_OK;
  }
  if (diff < 0) {
    ord = ORD_OOO;
    u64 off = 0;
    if (!rm_get(L, p.esn, off)) return MG_OOO_MISS;
    u64 esn = p.esn - off;
    if (esn >= L.h.extLastSN) return MG_OOO_MISS;
    osn = esn;
    ots = p.ets - L.h.tsOffset;
    return MG_OK;
  }
  if (diff == 1) {
    L.h.extHighestIncomingSN = p.esn;
    rm_exclude(L, L.h.extHighestIncomingSN, L.h.extHighestIncomingSN + 1);
    mg_updateSnOffset(L);
    ord = ORD_CONTIG;
    return MG_PADDING;
  }
  ord = ORD_DUP;
  return MG_DUP;
}

// ---- VP8 munger rings (elliotchance/orderedmap semantics) ------------------
// All keys of a ring are distinct (map semantics), so a membership test is one
// ballot over the ring positions (wave-uniform key).
__device__ __forceinline__ int miss_find(const Lane &L, i32 key) {
  const u32 l = lane_id();
  for (int base = 0; base < int(L.h.missCount); base += 64) {
    const int i = base + int(l);
    const int idx = (L.h.missHead + i) % kMissCap;
    const u64 m = __ballot(i < int(L.h.missCount) && L.missKey[idx] == key);
    if (m) return (L.h.missHead + base + __ffsll((long long)m) - 1) % kMissCap;
  }
  return -1;
}
__device__ __forceinline__ bool set_has(const i32 *keys, u8 head, u8 count, i32 key) {  // per-lane key
  for (int i = 0; i < count; i++)
    if (keys[(head + i) % kSetCap] == key) return true;
  return false;
}
__device__ __forceinline__ bool set_has_u(const i32 *keys, u8 head, u8 count, i32 key) {  // wave-uniform key
  const u32 l = lane_id();
  return __ballot(l < count && keys[(head + l) % kSetCap] == key) != 0;
}
// Set(key,true) then trim to `keep` (vp8.go:242-247, :257-262); wave-uniform
__device__ __forceinline__ void set_add(i32 *keys, u8 &head, u8 &count, i32 key, int keep) {
  if (set_has_u(keys, head, count, key)) return;
  wave_lds_sync();
  keys[(head + count) % kSetCap] = key;
  count++;
  if (count > keep) {
    head = u8((head + count - keep) % kSetCap);
    count = u8(keep);
  }
  wave_lds_sync();
}

// The missing-picture loop of vp8.go:218-235, exact:
//   for lost in [prevMax, ext]: if !dropped(lost): missing.Set(lost, off)
//   trim missing to the newest 50.
// Equivalent bounded form: existing entries in range are updated in place;
// of the new keys only the newest 50 can survive the trim, appended in order.
// Wave form: the range [prevMax, prevMax+63] is a 64-bit mask; dropped and
// existing keys are OR-reduced into it, the new keys are its remaining bits.
__device__ void vp8_record_missing_wide(Lane &L, i32 prevMax, i32 ext, i32 off) {  // range > 64 pictures
  const int e0 = L.h.missCount;
  int inE = 0;  // existing (not dropped) keys inside the range
  for (int i = 0; i < e0; i++) {
    int idx = (L.h.missHead + i) % kMissCap;
    i32 k = L.missKey[idx];
    if (k >= prevMax && k <= ext && !set_has_u(L.dropKey, L.h.dropHead, L.h.dropCount, k)) {
      L.missVal[idx] = off;
      inE++;
    }
  }
  int nDrop = 0;
  for (int i = 0; i < L.h.dropCount; i++) {
    i32 k = L.dropKey[(L.h.dropHead + i) % kSetCap];
    if (k >= prevMax && k <= ext) nDrop++;
  }
  i64 nNew = i64(ext) - i64(prevMax) + 1 - nDrop - inE;
  if (nNew <= 0) return;
  int want = nNew > kMissKeep ? kMissKeep : int(nNew);
  i32 s = ext;
  int got = 0;
  for (i32 k = ext;; k--) {  // walking down from ext, the want-th new key
    if (!set_has_u(L.dropKey, L.h.dropHead, L.h.dropCount, k) && miss_find(L, k) < 0) {
      got++;
      if (got == want) {
        s = k;
        break;
      }
    }
    if (k == prevMax) break;
  }
  for (i32 k = s;; k++) {  // append new keys in [s, ext] in order
    if (!set_has_u(L.dropKey, L.h.dropHead, L.h.dropCount, k) && miss_find(L, k) < 0) {
      wave_lds_sync();
      int idx = (L.h.missHead + L.h.missCount) % kMissCap;
      L.missKey[idx] = k;
      L.missVal[idx] = off;
      L.h.missCount++;
      wave_lds_sync();
    }
    if (k == ext) break;
  }
  if (L.h.missCount > kMissKeep) {
    L.h.missHead = u8((L.h.missHead + L.h.missCount - kMissKeep) % kMissCap);
    L.h.missCount = u8(kMissKeep);
  }
}
__device__ __forceinline__ void vp8_record_missing(Lane &L, i32 prevMax, i32 ext, i32 off) {
  L.vcDirty = true;
  if (ext < prevMax) return;
  const i64 span = i64(ext) - i64(prevMax) + 1;
  if (span > 64) {
    vp8_record_missing_wide(L, prevMax, ext, off);
    return;
  }
  const u32 l = lane_id();
  const u64 rangeM = span == 64 ? ~0ull : ((1ull << span) - 1);
  u64 dropBits = 0;
  if (l < L.h.dropCount) {
    const i32 k = L.dropKey[(L.h.dropHead + l) % kSetCap];
    if (k >= prevMax && k <= ext) dropBits = 1ull << (k - prevMax);
  }
  const u64 dropM = wave_or_u64(dropBits);
  const int cnt = L.h.missCount;
  u64 exBits = 0;
  for (int base = 0; base < cnt; base += 64) {
    const int i = base + int(l);
    if (i < cnt) {
      const int idx = (L.h.missHead + i) % kMissCap;
      const i32 k = L.missKey[idx];
      if (k >= prevMax && k <= ext) {
        const u64 bit = 1ull << (k - prevMax);
        exBits |= bit;
        if (!(dropM & bit)) L.missVal[idx] = off;  // Set on an existing key: in place
      }
    }
  }
  u64 newM = rangeM & ~dropM & ~wave_or_u64(exBits);
  int nNew = __popcll(newM);
  if (nNew == 0) return;
  while (nNew > kMissKeep) {  // older new keys would be trimmed right away
    newM &= newM - 1;
    nNew--;
  }
  wave_lds_sync();
  if ((newM >> l) & 1) {
    const int r = __popcll(newM & ((1ull << l) - 1));
    const int idx = (L.h.missHead + cnt + r) % kMissCap;
    L.missKey[idx] = prevMax + i32(l);
    L.missVal[idx] = off;
  }
  wave_lds_sync();
  const int total = cnt + nNew;
  if (total > kMissKeep) {
    L.h.missHead = u8((L.h.missHead + total - kMissKeep) % kMissCap);
    L.h.missCount = u8(kMissKeep);
  } else {
    L.h.missCount = u8(total);
  }
}

// VP8PictureIdWrapHandler.Unwrap vp8.go:400-483
__device__ __forceinline__ i32 wr_unwrap(Lane &L, u16 pictureId, bool mBit) {
  i32 mp = L.h.wrMaxPictureId;
  bool maxM = hasf(L, F_WR_MAX_MBIT);
  if (mp > 0) mp = maxM ? (L.h.wrMaxPictureId & 0x7fff) : (L.h.wrMaxPictureId & 0x7f);
  i32 np = mBit ? i32(pictureId & 0x7fff) : i32(pictureId & 0x7f);
  if (L.h.wrTotalWrap > 0) {
    if ((L.h.wrMaxPictureId + (L.h.wrLastWrap >> 1)) < (np + L.h.wrTotalWrap))
      return np + L.h.wrTotalWrap - L.h.wrLastWrap;
  }
  i32 wrap = 0;
  if (maxM) {
    if (np < mp && (mp - np) > (1 << 14)) wrap = 1 << 15;
  } else {
    if (np < mp && (mp - np) > (1 << 6)) wrap = 1 << 7;
  }
  L.h.wrTotalWrap += wrap;
  if (wrap != 0) L.h.wrLastWrap = wrap;
  return np + L.h.wrTotalWrap;
}
__device__ __forceinline__ void wr_init(Lane &L, i32 ext, bool m) {
  L.h.wrMaxPictureId = ext;
  setf(L, F_WR_MAX_MBIT, m);
  L.h.wrTotalWrap = 0;
  L.h.wrLastWrap = 0;
}

// buffer.VP8.MarshalTo helpers.go:170-227, bytes packed little-endian into a
// u64 (byte i = bits 8i..8i+7); returns HeaderSize (or -1 if the fields need
// more than hs bytes: Go would panic on the index).
__device__ __forceinline__ int vp8_marshal(u8 first, bool I, bool M, u16 pid, bool Lb, u8 tl0, bool T, u8 tid,
                                           bool Y, bool K, u8 keyidx, int hs, u64 &out) {
  if (hs < 1 || hs > 6) return -1;
  out = 0;
  if (I || Lb || T || K) {
    out = u64(u8(first | 0x80));  // X bit
    u32 xval = 0;
    int idx = 2;
    if (I) {
      xval |= 0x80;
      if (M) {
        if (idx + 1 >= hs) return -1;
        out |= u64(0x80 | ((pid >> 8) & 0x7f)) << (8 * idx);
        out |= u64(pid & 0xff) << (8 * (idx + 1));
        idx += 2;
      } else {
        if (idx >= hs) return -1;
        out |= u64(pid & 0xff) << (8 * idx);
        idx++;
      }
    }
    if (Lb) {
      xval |= 0x40;
      if (idx >= hs) return -1;
      out |= u64(tl0) << (8 * idx);
      idx++;
    }
    if (T || K) {
      if (idx >= hs) return -1;
      u32 b = 0;
      if (T) {
        xval |= 0x20;
        b = u32(tid << 6) & 0xff;
        if (Y) b |= 0x20;
      }
      if (K) {
        xval |= 0x10;
        b |= keyidx & 0x1f;
      }
      out |= u64(b) << (8 * idx);
      idx++;
    }
    if (hs < 2) return -1;
    out |= u64(xval) << 8;
  } else {
    out = u64(u8(first & 0x7f));
  }
  return hs;
}

enum { CM_OK = 0, CM_FILTERED, CM_PICID_MISS, CM_ERR };
// VP8.UpdateAndGet vp8.go:161-302
__device__ __forceinline__ int vp8_update(Lane &L, const PktV &p, bool ooo, bool gap, i32 maxTL, u64 &cb,
                                           int &cbLen) {
  const bool I = p.vbits & LKF_VP8_I, M = p.vbits & LKF_VP8_M, Lb = p.vbits & LKF_VP8_L;
  const bool T = p.vbits & LKF_VP8_T, Y = p.vbits & LKF_VP8_Y, K = p.vbits & LKF_VP8_K;
  i32 ext = wr_unwrap(L, p.pid, M);
  if (ooo) {
    int idx = miss_find(L, ext);
    if (idx < 0) return CM_PICID_MISS;
    i32 off = L.missVal[idx];
    u16 mpid = u16((ext - off) & 0x7fff);
    bool mM = mpid > 127;
    int hs = int(p.vhs) + (mM == M ? 0 : (mM ? 1 : -1));
    cbLen = vp8_marshal(p.vfirst, I, mM, mpid, Lb, u8(p.tl0 - L.h.tl0Off), T, p.tid, Y, K,
                        u8(p.keyidx - L.h.keyIdxOff), hs, cb);
    return cbLen < 0 ? CM_ERR : CM_OK;
  }
  i32 prevMax = L.h.wrMaxPictureId;
  L.h.wrMaxPictureId = ext;  // UpdateMaxPictureId
  setf(L, F_WR_MAX_MBIT, M);
  if (gap) {
    vp8_record_missing(L, prevMax, ext, L.h.pictureIdOffset);
    if (T && p.tid > u8(maxTL)) {
      L.vcDirty = true;
      set_add(L.exKey, L.h.exHead, L.h.exCount, ext, kExemptKeep);
    }
  } else {
    if (T && p.tid > u8(maxTL)) {
      if (!set_has_u(L.exKey, L.h.exHead, L.h.exCount, ext)) {
        if (I && prevMax != ext) {
          L.vcDirty = true;
          set_add(L.dropKey, L.h.dropHead, L.h.dropCount, ext, kDropKeep);
          L.h.pictureIdOffset += 1;
        }
        return CM_FILTERED;
      }
    }
  }
  i32 mext = ext - L.h.pictureIdOffset;
  u16 mpid = u16(mext & 0x7fff);
  u8 mtl0 = u8(p.tl0 - L.h.tl0Off);
  u8 mkey = u8((p.keyidx - L.h.keyIdxOff) & 0x1f);
  L.h.extLastPictureId = mext;
  L.h.lastTl0 = mtl0;
  L.h.lastKeyIdx = mkey;
  bool mM = mpid > 127;
  int hs = int(p.vhs) + (mM == M ? 0 : (mM ? 1 : -1));
  cbLen = vp8_marshal(p.vfirst, I, mM, mpid, Lb, mtl0, T, p.tid, Y, K, mkey, hs, cb);
  return cbLen < 0 ? CM_ERR : CM_OK;
}
// VP8.SetLast vp8.go:111-134
__device__ void vp8_setLast(Lane &L, const PktV &p) {
  if (!(p.flags & LKF_PKT_VP8)) return;
  bool I = p.vbits & LKF_VP8_I;
  setf(L, F_PICID_USED, I);
  if (I) {
    wr_init(L, i32(p.pid) - 1, p.vbits & LKF_VP8_M);
    L.h.extLastPictureId = i32(p.pid);
  }
  bool Lb = p.vbits & LKF_VP8_L;
  setf(L, F_TL0_USED, Lb);
  if (Lb) L.h.lastTl0 = p.tl0;
  setf(L, F_TID_USED, p.vbits & LKF_VP8_T);
  bool K = p.vbits & LKF_VP8_K;
  setf(L, F_KEYIDX_USED, K);
  if (K) L.h.lastKeyIdx = p.keyidx;
}
// VP8.UpdateOffsets vp8.go:136-159
__device__ void vp8_updateOffsets(Lane &L, const PktV &p) {
  if (!(p.flags & LKF_PKT_VP8)) return;
  if (hasf(L, F_PICID_USED)) {
    wr_init(L, i32(p.pid) - 1, p.vbits & LKF_VP8_M);
    L.h.pictureIdOffset = i32(p.pid) - L.h.extLastPictureId - 1;
  }
  if (hasf(L, F_TL0_USED)) L.h.tl0Off = u8(p.tl0 - L.h.lastTl0 - 1);
  if (hasf(L, F_KEYIDX_USED)) L.h.keyIdxOff = u8((p.keyidx - L.h.lastKeyIdx - 1) & 0x1f);
  L.h.missHead = L.h.missCount = 0;
  L.h.dropHead = L.h.dropCount = 0;
  L.h.exHead = L.h.exCount = 0;
}

// ---- Forwarder control (forwarder.go) --------------------------------------
__device__ __forceinline__ void fw_resync(Lane &L) {  // :1391-1397
  L.h.curS = INVALID;
  L.h.curT = INVALID;
  L.h.lastSSRC = 0;
  if (hasf(L, F_PUBMUTED)) setf(L, F_RESUME_BEHIND, true);
}
__device__ __forceinline__ void apply_ctl(Lane &L, const DevEvent &ev) {
  const bool video = hasf(L, F_VIDEO);
  switch (ev.op) {
    case LKF_CTL_MUTE: {  // :377-413
      bool m = ev.a[0] != 0;
      if (hasf(L, F_MUTED) == m) break;
      if (m && ev.a[1] == 0) break;
      setf(L, F_MUTED, m);
      if (m) fw_resync(L);
      break;
    }
    case LKF_CTL_PUBMUTE: {  // :422-438
      bool m = ev.a[0] != 0;
      if (hasf(L, F_PUBMUTED) == m) break;
      setf(L, F_PUBMUTED, m);
      if (m) fw_resync(L);
      break;
    }
    case LKF_CTL_SET_MAX_SPATIAL:  // :454-470
      if (video && i32(ev.a[0]) != L.h.maxS) L.h.maxS = i32(ev.a[0]);
      break;
    case LKF_CTL_SET_MAX_TEMPORAL:  // :472-488
      if (video && i32(ev.a[0]) != L.h.maxT) L.h.maxT = i32(ev.a[0]);
      break;
    case LKF_CTL_SET_MAX_SEEN_SPATIAL:  // :241-253
      if (i32(ev.a[0]) > L.h.seenS) L.h.seenS = i32(ev.a[0]);
      break;
    case LKF_CTL_SET_MAX_SEEN_TEMPORAL:  // :255-267
      if (i32(ev.a[0]) > L.h.seenT) L.h.seenT = i32(ev.a[0]);
      break;
    case LKF_CTL_SET_ALLOCATION: {  // updateAllocation :1353-1382
      if (!video) break;
      i32 ts = i32(ev.a[0]), tt = i32(ev.a[1]);
      bool valid = ts != INVALID && tt != INVALID;
      if (valid && L.codec == LKF_CODEC_H264) tt = 0;
      setf(L, F_DEFICIENT, ev.a[3] != 0);
      L.h.ptgtS = ts;
      L.h.ptgtT = tt;
      L.h.tgtS = ts;
      L.h.tgtT = tt;
      L.h.reqS = valid ? i32(ev.a[2]) : INVALID;
      if (!valid) fw_resync(L);
      break;
    }
    case LKF_CTL_RESYNC:
      fw_resync(L);
      break;
    case LKF_CTL_SET_TARGET:
      L.h.ptgtS = L.h.tgtS = i32(ev.a[0]);
      L.h.ptgtT = L.h.tgtT = i32(ev.a[1]);
      break;
    case LKF_CTL_PLAYOUT_ACKED:
      setf(L, F_PLAYOUT_ACKED, ev.a[0] != 0);
      break;
    case kOpLayerOffsets: {  // the track's layerOffsets from this packet on (lkf_sender_report)
      const u32 l = lane_id();
      if (l < 9) L.offs[l] = l < 8 ? u32(u64(ev.a[l >> 1]) >> (32 * (l & 1))) : u32(u64(ev.pad));
      break;
    }
    default:
      break;
  }
}

// processSourceSwitch forwarder.go:1456-1647 on the virtual clock (now = arrival)
__device__ bool fw_sourceSwitch(Lane &L, const PktV &p, i32 layer) {
  if (!hasf(L, F_STARTED)) {
    setf(L, F_STARTED, true);
    L.h.referenceLayerSpatial = layer;
    mg_setLastSnTs(L, p.esn, p.ets);
    if (hasf(L, F_VP8)) vp8_setLast(L, p);
    return true;
  } else if (L.h.referenceLayerSpatial == INVALID) {
    L.h.referenceLayerSpatial = layer;
  }
  const u64 extLastTS = L.h.extLastTS;
  u64 extExpectedTS = extLastTS;
  u64 extRefTS = extExpectedTS;
  if (L.hasRefTS) {  // StreamTrackerManager.GetReferenceLayerRTPTimestamp :660-679
    i32 ref = L.h.referenceLayerSpatial;
    if (layer < 0 || layer >= 3 || ref < 0 || ref >= 3) return false;
    // isSVC (:667-671): one stream, one timeline -> offset 0
    const bool svc = L.codec == LKF_CODEC_VP9 || L.codec == LKF_CODEC_AV1;  // IsSvcCodec receiver.go:142-150
    const u32 off = svc ? 0u : L.offs[ref * 3 + layer];
    if (!svc && layer != ref && off == 0) return false;
    u32 ts = u32(p.ets) + off;
    extRefTS = (extRefTS & 0xFFFFFFFF00000000ull) + u64(ts);
    u32 e32 = u32(extExpectedTS);
    if (u32(ts - e32) < (1u << 31) && ts < e32) extRefTS += (1ull << 32);
    if (u32(e32 - ts) < (1u << 31) && e32 < ts && extRefTS >= (1ull << 32)) extRefTS -= (1ull << 32);
  }
  if (hasf(L, F_HAS_EXPECTED)) {  // DownTrack.getExpectedRTPTimestamp downtrack.go:1765
    if (hasf(L, F_STATS_INIT)) {
      i64 diff = (p.arr - L.h.statsFirstTime) * i64(L.clockRate) / 1000000000LL;
      extExpectedTS = L.h.statsExtStartTS + u64(diff);
    } else if (L.h.preStartTime != 0) {
      i64 since = p.arr - L.h.preStartTime;
      u64 rtpDiff = u64(since * i64(L.clockRate) / 1000000000LL);
      extExpectedTS = L.h.extFirstTS + rtpDiff;
      if (L.h.refTSOffset == 0) L.h.refTSOffset = extExpectedTS - extRefTS;
    }
  }
  extRefTS += L.h.refTSOffset;
  u64 extNextTS;
  const double cr = double(L.clockRate);
  if (L.h.lastSSRC == 0) {
    double diffSeconds = double(i64(extExpectedTS - extRefTS)) / cr;
    if (diffSeconds >= 0.0) {
      if (hasf(L, F_RESUME_BEHIND) && diffSeconds > 0.2)
        extNextTS = extExpectedTS;
      else if (diffSeconds > 2.0)
        extNextTS = extExpectedTS;
      else
        extNextTS = extRefTS;
    } else {
      extNextTS = extRefTS;
    }
    setf(L, F_RESUME_BEHIND, false);
  } else {
    double diffSeconds = double(i64(extRefTS - extLastTS)) / cr;
    if (diffSeconds < 0.0) {
      if (fabs(diffSeconds) > 0.05) return false;
      extNextTS = extLastTS + 1;
    } else {
      extNextTS = extRefTS;
    }
  }
  if (i64(extNextTS - extLastTS) <= 0) extNextTS = extLastTS + 1;
  mg_updateSnTsOffsets(L, p.esn, p.ets, 1, extNextTS - extLastTS);
  if (hasf(L, F_VP8)) vp8_updateOffsets(L, p);
  return true;
}

// getTranslationParamsCommon :1650-1671 -> drop reason or -1 (forward)
__device__ __forceinline__ int fw_common(Lane &L, const PktV &p, i32 layer, bool marker, int &ord, u64 &osn,
                                         u64 &ots) {
  if (L.h.lastSSRC != p.ssrc) {
    if (!fw_sourceSwitch(L, p, layer)) return LKF_DROP_SWITCH;
    L.h.lastSSRC = p.ssrc;
  }
  int r = mg_update(L, p, marker, ord, osn, ots);
  if (r == MG_PADDING) return LKF_DROP_PADDING;
  if (r == MG_DUP) return LKF_DROP_DUPLICATE;
  if (r == MG_OOO_MISS) return LKF_DROP_OOO_MISS;
  return -1;
}

template <bool DDK = false>
__device__ __forceinline__ void vls_rollback(Lane &L) {  // base.go Rollback
  if (DDK && hasf(L, F_DD)) {  // DependencyDescriptor.Rollback dependencydescriptor.go:357-361
    L.dd->mask = L.dd->prevMask;
    if (L.dd->flags & DS_HAS_PREV_MASK)
      L.dd->flags |= DS_HAS_MASK;
    else
      L.dd->flags &= ~u32(DS_HAS_MASK);
  }
  L.h.curS = L.h.prevS;
  L.h.curT = L.h.prevT;
  L.h.tgtS = L.h.ptgtS;
  L.h.tgtT = L.h.ptgtT;
}

struct Fwd {
  int ord;
  u64 osn, ots;
  bool switching, resuming, marker;
  int cbLen;
  u64 cb;  // munged VP8 descriptor bytes, little-endian packed
  int ddLen;  // marshalled dependency descriptor in L.ddBuf (tp.ddBytes)
};

// Forwarder.GetTranslationParams forwarder.go:1436-1765 for one (packet, DownTrack).
// DDK: the instantiation for DownTracks with the dependency-descriptor
// selector (k_decide_dt<true>); the others never compile its code.
template <bool DDK>
__device__ int fw_translate(Lane &L, const PktV &p, u32 k, Fwd &o) {
  o.switching = o.resuming = o.marker = false;
  o.cbLen = 0;
  o.cb = 0;
  o.ddLen = 0;
  const i32 layer = p.layer;
  if (hasf(L, F_MUTED) || hasf(L, F_PUBMUTED)) return LKF_DROP_MUTED;
  if (!hasf(L, F_VIDEO)) return fw_common(L, p, layer, false, o.ord, o.osn, o.ots);
  // ---- video :1679-1765
  if (L.h.tgtS == INVALID || L.h.tgtT == INVALID) return LKF_DROP_PAUSED;
  // vls.Select: Simulcast simulcast.go:42-122 (Null selector: never selected)
  bool isSelected = false, isSwitching = false, isResuming = false;
  const bool kf = p.flags & LKF_PKT_KEYFRAME;
  const bool pktMarker = p.hdr1 & 0x80;
  if (hasf(L, F_SIMULCAST)) {
    if (L.h.curS != L.h.tgtS) {
      bool isActive = L.h.curS != INVALID && L.h.curT != INVALID;
      bool found = false;
      if (kf) {
        if (layer > L.h.curS && layer <= L.h.tgtS) found = true;
        if (layer < L.h.curS && layer >= L.h.tgtS) found = true;
      }
      if (found) {
        L.h.prevS = L.h.curS;
        L.h.prevT = L.h.curT;
        L.h.curS = layer;
        L.h.curT = p.temporal;
        L.h.ptgtS = L.h.tgtS;
        L.h.ptgtT = L.h.tgtT;
        if (L.h.curS >= L.h.maxS || L.h.curS == L.h.seenS) L.h.tgtS = L.h.curS;
        isSwitching = true;
        if (!isActive) isResuming = true;
      }
    }
    if (L.h.curS > L.h.maxS && layer <= L.h.maxS && kf) {
      L.h.prevS = L.h.curS;
      L.h.prevT = L.h.curT;
      L.h.curS = layer;
      L.h.ptgtS = L.h.tgtS;
      L.h.ptgtT = L.h.tgtT;
      if (L.h.curS >= L.h.maxS || L.h.curS == L.h.seenS) L.h.tgtS = layer;
      isSwitching = true;
    }
    isSelected = layer == L.h.curS;
  }
  bool marker = pktMarker;
  if (hasf(L, F_VP9)) {  // VP9.Select videolayerselector/vp9.go:43-109
    bool relevant = false;
    if (p.flags & LKF_PKT_VP9) {
      const bool U = p.vp9 & LKF_VP9_U, B = p.vp9 & LKF_VP9_B, E = p.vp9 & LKF_VP9_E, P = p.vp9 & LKF_VP9_P;
      const i32 pS = p.spatial, pT = p.temporal;
      i32 cS = L.h.curS, cT = L.h.curT;  // the local currentLayer copy (vp9.go:49)
      bool zero = false;
      if (L.h.curS != L.h.tgtS || L.h.curT != L.h.tgtT) {
        i32 uS = L.h.curS, uT = L.h.curT;
        const bool curValid = L.h.curS != INVALID && L.h.curT != INVALID;
        if (!curValid) {
          if (!kf)
            zero = true;  // zero result: not selected, not relevant (vp9.go:55-57)
          else {
            uS = pS;
            uT = pT;
          }
        } else {
          if (L.h.curT != L.h.tgtT) {
            if (L.h.curT < L.h.tgtT) {
              if (pT > L.h.curT && pT <= L.h.tgtT && U && B) cT = uT = pT;
            } else if (E) {
              uT = L.h.tgtT;
            }
          }
          if (L.h.curS != L.h.tgtS) {
            if (L.h.curS < L.h.tgtS) {
              if (pS > L.h.curS && pS <= L.h.tgtS && !P && B) cS = uS = pS;
            } else if (E) {
              uS = L.h.tgtS;
            }
          }
        }
        if (!zero && (uS != L.h.curS || uT != L.h.curT)) {
          isSwitching = true;
          if (!curValid && uS != INVALID && uT != INVALID) isResuming = true;
          L.h.prevS = L.h.curS;
          L.h.prevT = L.h.curT;
          L.h.curS = uS;
          L.h.curT = uT;
        }
      }
      if (!zero) {
        if (E && pS == cS && (P || L.h.tgtS <= L.h.curS)) marker = true;
        isSelected = !(pS > cS || (pS == cS && pT > cT));
        relevant = true;
      }
    }
    if (!isSelected) {
      // forwarder.go:1694-1702: a relevant drop still advances the munger
      if (relevant && hasf(L, F_STARTED)) {
        int ord;
        u64 a, b;
        if (mg_update(L, p, marker, ord, a, b) == MG_OK && ord == ORD_CONTIG) mg_packetDropped(L, p.esn);
      }
      return LKF_DROP_NOT_SELECTED;
    }
  }
  if (DDK && hasf(L, F_DD)) {  // DependencyDescriptor.Select videolayerselector/dependencydescriptor.go:65-355
    // (the descriptor is staged in LDS: dd_select's state writes and its
    // reads of the descriptor go through generic pointers, so every read
    // after a write is a reload — from LDS, not from HBM)
    const bool inDD = (p.flags & LKF_PKT_DD) && L.ddPkts;
    if (inDD) {
      const u32 ln = lane_id();
      if (ln < sizeof(DDPkt) / 16)
        reinterpret_cast<uint4 *>(L.ddPktL)[ln] = reinterpret_cast<const uint4 *>(L.ddPkts + k)[ln];
      wave_lds_sync();
    }
    const bool hasDD = inDD && (L.ddPktL->flags & DP_VALID);
#if LKF_SVC_STATS
    const u64 tS0 = __builtin_amdgcn_s_memtime();
#endif
    const dd::SelResult r = dd::dd_select(*L.dd, L.ddRing, hasDD ? L.ddPktL : nullptr, pktMarker, L.h.curS, L.h.curT, L.h.prevS,
                                          L.h.prevT, L.h.tgtS, L.h.tgtT, L.ddBuf, L.ddS, L.ddSSlot, L.ddSpill);
#if LKF_SVC_STATS
    if (lane_id() == 0) {  // g_svc[13..14]: dd_select cycles, calls
      SVC_ADD(13, __builtin_amdgcn_s_memtime() - tS0);
      SVC_ADD(14, 1ull);
    }
#endif
    if (r.limit && lane_id() == 0) atomicOr(L.err, 16u);
    L.ddSSlot = r.stagedSlot;
    if (!r.selected) {
      if (r.relevant && hasf(L, F_STARTED)) {  // forwarder.go:1694-1702 (RTPMarker false)
        int ord;
        u64 a, b;
        if (mg_update(L, p, false, ord, a, b) == MG_OK && ord == ORD_CONTIG) mg_packetDropped(L, p.esn);
      }
      return LKF_DROP_NOT_SELECTED;
    }
    isSelected = true;
    isSwitching = r.switching;
    isResuming = r.resuming;
    marker = r.marker;
    o.ddLen = r.ddLen;
  }
  if (!isSelected) return LKF_DROP_NOT_SELECTED;  // IsRelevant == false for Simulcast
  o.resuming = isResuming;
  o.switching = isSwitching;
  o.marker = marker;
  if (hasf(L, F_DEFICIENT) && L.h.tgtS < L.h.curS) {  // FlagPauseOnDowngrade :1709
    if (isSwitching) vls_rollback<DDK>(L);
    return LKF_DROP_DOWNGRADE;
  }
  int dr = fw_common(L, p, layer, marker, o.ord, o.osn, o.ots);
  if (dr >= 0 || p.plen == 0) {
    if (isSwitching) vls_rollback<DDK>(L);
    return dr;
  }
  // vls.SelectTemporal base.go:143-168 + temporallayerselector/vp8.go:32-56
  i32 tl = L.h.curT;
  bool tSwitch = false;
  if (hasf(L, F_TLS_VP8)) {
    i32 cur = L.h.curT, tgt = L.h.tgtT, nxt = cur;
    if (cur != tgt && (p.flags & LKF_PKT_VP8) && (p.vbits & LKF_VP8_T)) {
      i32 tid = i32(p.tid);
      if (cur < tgt) {
        if (tid > cur && tid <= tgt && (p.vbits & LKF_VP8_S) && (p.vbits & LKF_VP8_Y)) {
          tl = tid;
          nxt = tid;
        }
      } else if (pktMarker) {
        nxt = tgt;
      }
    }
    if (nxt != L.h.curT) {
      tSwitch = true;
      L.h.prevS = L.h.curS;
      L.h.prevT = L.h.curT;
      L.h.curT = nxt;
    }
  }
  if (hasf(L, F_VP8)) {
    int cr;
    if (!(p.flags & LKF_PKT_VP8))
      cr = CM_ERR;  // ErrNotVP8
    else
      cr = vp8_update(L, p, o.ord == ORD_OOO, o.ord == ORD_GAP, tl, o.cb, o.cbLen);
    if (cr != CM_OK) {
      if (cr == CM_FILTERED) mg_packetDropped(L, p.esn);
      if (isSwitching || tSwitch) vls_rollback<DDK>(L);
      return cr == CM_FILTERED ? LKF_DROP_TEMPORAL : cr == CM_PICID_MISS ? LKF_DROP_PICID_MISS : LKF_DROP_OTHER;
    }
  }
  return -1;
}


// Records go to HBM as whole, aligned dwordx4 stores (the byte-field struct
// copy compiles to sub-dword and misaligned stores, which the memory pipeline
// splits into many transactions and which every later vmcnt wait then drains).
__device__ __forceinline__ u32 pack4(u8 a, u8 b, u8 c, u8 d) {
  return u32(a) | (u32(b) << 8) | (u32(c) << 16) | (u32(d) << 24);
}
struct __attribute__((aligned(8))) U4x8 {  // 16 B at an 8-B aligned address (one dwordx4 access)
  u32 x, y, z, w;
};
// a forwarded record (FwdRec): one dwordx4 + one dwordx2 store; its full SN /
// TS go to the wide side array too when they lie 2^31 or more from the base
__device__ __forceinline__ void store_fwd(FwdRec *dst, FwdBase *wdst, u64 bSN, u64 bTS, u64 sn, u64 ts, u32 pkt,
                                          u32 relOff, u32 outLen, u32 flags, u32 ddLen, u32 aux) {
  if ((((sn - bSN) + 0x80000000ull) >> 32) != 0 || (((ts - bTS) + 0x80000000ull) >> 32) != 0) {
    flags |= T_WIDE;
    *wdst = FwdBase{sn, ts};
  }
  *reinterpret_cast<U4x8 *>(dst) = U4x8{u32(sn), u32(ts), pkt, relOff >> 4};
  reinterpret_cast<uint2 *>(dst)[2] = make_uint2(outLen | (flags << 16) | (ddLen << 24), aux);
}
// FwdRec.aux of a munged VP8 descriptor: its picture id, TL0PICIDX and KEYIDX
__device__ __forceinline__ u32 vp8_aux(u32 mpid, u32 mtl0, u32 mkey) {
  return (mpid & 0xffffu) | ((mtl0 & 0xffu) << 16) | ((mkey & 0x1fu) << 24);
}
// ... read back from marshalled bytes (vp8_marshal's layout, byte i = bits 8i..8i+7)
__device__ __forceinline__ u32 vp8_aux_of(u64 cb) {
  if (!(cb & 0x80)) return 0;  // no extension byte: none of the fields
  const u32 x = u32(cb >> 8) & 0xff;
  int idx = 2;
  u32 pid = 0, tl0 = 0, key = 0;
  if (x & 0x80) {
    const u32 b = u32(cb >> (8 * idx)) & 0xff;
    if (b & 0x80) {
      pid = ((b & 0x7f) << 8) | (u32(cb >> (8 * (idx + 1))) & 0xff);
      idx += 2;
    } else {
      pid = b;
      idx++;
    }
  }
  if (x & 0x40) tl0 = u32(cb >> (8 * idx++)) & 0xff;
  if (x & 0x30) key = u32(cb >> (8 * idx)) & 0x1f;
  return vp8_aux(pid, tl0, key);
}
__device__ __forceinline__ void store_rec(SeqMeta *dst, const SeqMeta &m) {  // 2 x dwordx4 (pad = 0)
  uint4 *d = reinterpret_cast<uint4 *>(dst);
  d[0] = make_uint4(u32(m.sourceSeqNo) | (u32(m.targetSeqNo) << 16), m.timestamp, m.lastNack,
                    pack4(m.marker, m.nacked, u8(m.layer), m.codecLen));
  d[1] = make_uint4(pack4(m.codec[0], m.codec[1], m.codec[2], m.codec[3]),
                    pack4(m.codec[4], m.codec[5], m.codec[6], m.codec[7]), 0u, 0u);
}

// invalidateSlot (sequencer.go:351-366) of the n slots after the highest slot
__device__ __forceinline__ void seq_invalidate(Lane &L, u32 n) {
  const SeqMeta z = {};
  for (u32 i = lane_id(); i < n; i += 64) {
    u32 x = u32(L.h.seqHighSlot) + 1 + i;
    while (x >= L.seqSize) x -= L.seqSize;
    store_rec(L.seq + x, z);
  }
}
// ---- the sequencer's RangeMap (SeqRM): serial forms, one thread or every
// lane of a wave with the same arguments.  Written only by pushPadding.
__device__ __forceinline__ RangeEntry *srm_ring(SeqRM *h) { return reinterpret_cast<RangeEntry *>(h + 1); }
// GetValue rangemap.go:134-169
__device__ bool srm_get(SeqRM *h, u32 cap, u64 key, u64 &out) {
  out = 0;
  if (key >= h->openStart) {
    out = h->openValue;
    return true;
  }
  const u32 nc = h->count;
  const RangeEntry *ring = srm_ring(h);
  if (nc == 0 || key < ring[h->head].start) return false;  // too old
  for (i32 idx = i32(nc); idx >= 0; idx--) {
    u64 start = h->openStart;
    if (idx != i32(nc)) {
      const RangeEntry rv = ring[(h->head + u32(idx)) % cap];
      if ((key - rv.start) < HALF64 && (rv.end - key) < HALF64) {
        out = rv.value;
        return true;
      }
      start = rv.start;
    }
    if (idx > 0) {
      const RangeEntry pv = ring[(h->head + u32(idx) - 1) % cap];
      const u64 before = key - pv.end, after = start - key;
      if (before > 0 && before < HALF64 && after > 0 && after < HALF64) return false;  // excluded
    }
  }
  return false;
}
// ExcludeRange rangemap.go:100-132 (prune :171: the newest cap closed ranges)
__device__ bool srm_exclude(SeqRM *h, u32 cap, u64 s, u64 e, bool store) {
  if (e == s || (e - s) > HALF64) return false;
  if (h->openStart > s) return false;
  const u64 nv = h->openValue + (e - s);
  if (h->openStart == s) {
    if (store) {
      h->openStart = e;
      h->openValue = nv;
    }
    return true;
  }
  if (store) {
    RangeEntry c;
    c.start = h->openStart;
    c.end = s - 1;
    c.value = h->openValue;
    RangeEntry *ring = srm_ring(h);
    if (h->count < cap) {
      ring[(h->head + h->count) % cap] = c;
      h->count++;
    } else {
      ring[h->head] = c;
      h->head = (h->head + 1) % cap;
    }
    h->openStart = e;
    h->openValue = nv;
  }
  return true;
}
// sequencer.push sequencer.go:123-209 for a DownTrack whose sequencer has
// padding exclusions (F_SEQ_RM) and a push that needs them: the first push
// (updateSNOffset :136) or one below the highest SN (the RangeMap lookup
// :160-170).  Rare, and out of line with plain pointer arguments so the
// decide kernel's register allocation does not see it.
__device__ __noinline__ void seq_push_rm(DTHot *h, SeqMeta *seq, u32 size, SeqRM *srm, u32 cap, u64 esn,
                                         const SeqMeta *rec, u64 ets) {
  const bool init = !(h->flags & F_SEQ_INIT);
  u64 snOff = srm->snOffset;
  if (init) {
    h->flags |= F_SEQ_INIT;
    h->seqExtStartSN = esn;
    h->seqExtHighestSN = esn;
    h->seqExtHighestTS = ets;
    u64 off = 0;
    if (srm_get(srm, cap, esn + 1, off)) snOff = off;
    if (lane_id() == 0) srm->snOffset = snOff;
    h->seqHighSlot = u16((esn - snOff) % size);
  }
  if (esn < h->seqExtStartSN) return;
  const u64 adjH = h->seqExtHighestSN - snOff;
  u64 adjM = esn - snOff;
  if (esn < h->seqExtHighestSN) {
    u64 off = 0;
    if (!srm_get(srm, cap, esn, off)) return;
    adjM = esn - off;
  }
  const i64 delta = i64(adjM - adjH);
  if (delta <= -i64(size)) return;
  u32 slot;
  if (delta >= 0) {
    slot = u32((u64(h->seqHighSlot) + u64(delta) % size) % size);
  } else {
    const i32 sl = i32(h->seqHighSlot) + i32(delta);
    slot = u32(sl < 0 ? sl + i32(size) : sl);
  }
  if (adjM > adjH + 1) {  // invalidate the skipped slots (sequencer.go:179-189)
    const u64 nInv = (adjM - adjH - 1) < u64(size) ? (adjM - adjH - 1) : u64(size);
    for (u32 i = lane_id(); i < u32(nInv); i += 64) seq[(u32(h->seqHighSlot) + 1 + i) % size] = SeqMeta{};
  }
  if (lane_id() == 0) seq[slot] = *rec;
  if (esn > h->seqExtHighestSN) {
    h->seqExtHighestSN = esn;
    h->seqHighSlot = u16(slot);
  }
  if (ets > h->seqExtHighestTS) h->seqExtHighestTS = ets;
}

// sequencer.push sequencer.go:123-209.  Without padding exclusions (F_SEQ_RM
// clear) the sequencer's RangeMap maps everything to 0: slot = extModifiedSN
// % size, kept as seqHighSlot + the distance to the highest SN.
template <bool RM>
__device__ void seq_push(Lane &L, i64 arrMs, u64 inSN, u64 esn, u64 ets, bool marker, int8_t layer, u64 cb,
                         int cbLen) {
  const u32 size = L.seqSize;
  if (hasf(L, F_SEQ_INIT) && esn == L.h.seqExtHighestSN + 1) {  // in-order: next slot, nothing skipped
    u32 slot = u32(L.h.seqHighSlot) + 1;
    if (slot == size) slot = 0;
    SeqMeta m = {};
    m.sourceSeqNo = u16(inSN);
    m.targetSeqNo = u16(esn);
    m.timestamp = u32(ets);
    m.lastNack = u32(arrMs - L.h.seqStartMs);
    m.marker = marker;
    m.layer = layer;
    m.codecLen = u8(cbLen);
#pragma unroll
    for (int i = 0; i < 8; i++) m.codec[i] = u8(cb >> (8 * i));
    CHK(slot < size, CK_DEC_SEQ, slot, size);
    if (lane_id() == 0) store_rec(L.seq + slot, m);  // wave-uniform record: one lane stores it
    L.h.seqExtHighestSN = esn;
    L.h.seqHighSlot = u16(slot);
    if (ets > L.h.seqExtHighestTS) L.h.seqExtHighestTS = ets;
    return;
  }

  if (hasf(L, F_SEQ_RM) && (!hasf(L, F_SEQ_INIT) || esn < L.h.seqExtHighestSN)) {  // padding was sent
    if (!RM) {  // the host schedules such DownTracks in k_decide_dt<true>: never reached
      if (lane_id() == 0) atomicOr(L.err, 32u);
      return;
    }
    SeqMeta m = {};
    m.sourceSeqNo = u16(inSN);
    m.targetSeqNo = u16(esn);
    m.timestamp = u32(ets);
    m.lastNack = u32(arrMs - L.h.seqStartMs);
    m.marker = marker;
    m.layer = layer;
    m.codecLen = u8(cbLen);
#pragma unroll
    for (int i = 0; i < 8; i++) m.codec[i] = u8(cb >> (8 * i));
    __shared__ SeqMeta sRec;
    if (lane_id() == 0) sRec = m;
    __syncthreads();
    seq_push_rm(&L.h, L.seq, size, L.srm, L.srmCap, esn, &sRec, ets);
    __syncthreads();
    return;
  }
  if (!hasf(L, F_SEQ_INIT)) {
    setf(L, F_SEQ_INIT, true);
    L.h.seqExtStartSN = esn;
    L.h.seqExtHighestSN = esn;
    L.h.seqExtHighestTS = ets;
    L.h.seqHighSlot = u16(esn % size);  // once per DownTrack lifetime
  }
  if (esn < L.h.seqExtStartSN) return;
  const u64 adjH = L.h.seqExtHighestSN;
  const u64 adjM = esn;
  const i64 delta = i64(adjM - adjH);
  if (delta <= -i64(size)) return;
  // slot of adjM from the highest slot without a 64-bit modulo
  u32 slot;
  if (delta >= 0) {
    u32 dm = delta < i64(size) ? u32(delta) : u32(u64(delta) % size);
    slot = L.h.seqHighSlot + dm;
    if (slot >= size) slot -= size;
  } else {
    i32 sl = i32(L.h.seqHighSlot) + i32(delta);
    slot = u32(sl < 0 ? sl + i32(size) : sl);
  }
  if (adjM > adjH + 1) {  // invalidate the skipped slots (sequencer.go:179-189), one per lane
    const u64 nInv = (adjM - adjH - 1) < u64(size) ? (adjM - adjH - 1) : u64(size);
    seq_invalidate(L, u32(nInv));
  }
  SeqMeta m = {};
  m.sourceSeqNo = u16(inSN);
  m.targetSeqNo = u16(esn);
  m.timestamp = u32(ets);
  m.lastNack = u32(arrMs - L.h.seqStartMs);
  m.marker = marker;
  m.nacked = 0;
  m.layer = layer;
  m.codecLen = u8(cbLen);
#pragma unroll
  for (int i = 0; i < 8; i++) m.codec[i] = u8(cb >> (8 * i));
  CHK(slot < size, CK_DEC_SEQ, slot, size);
  L.seq[slot] = m;
  if (esn > L.h.seqExtHighestSN) {
    L.h.seqExtHighestSN = esn;
    L.h.seqHighSlot = u16(slot);
  }
  if (ets > L.h.seqExtHighestTS) L.h.seqExtHighestTS = ets;
}

__device__ __forceinline__ u64 wave_sum(u64 v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------
// k_batch_init: zeroes one batch context's per-track ranges, per-DownTrack
// forward counters, error word and counters (one launch instead of seven
// fills ahead of the decide stage).
// ---------------------------------------------------------------------------
__global__ void k_batch_init(u32 ntracks, u32 ndts, u32 nstats, u32 *__restrict__ tBegin, u32 *__restrict__ tEnd,
                             u32 *__restrict__ tRuns, u32 *__restrict__ err, u64 *__restrict__ stats,
                             u32 *__restrict__ fwdCnt, u64 *__restrict__ fwdBytes) {
  const u32 stride = gridDim.x * blockDim.x;
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < ntracks || i < ndts || i < nstats || i < 4; i += stride) {
    if (i < ntracks) {
      tBegin[i] = 0;
      tEnd[i] = 0;
      tRuns[i] = 0;
    }
    if (i < ndts) {
      fwdCnt[i] = 0;
      fwdBytes[i] = 0;
    }
    if (i < nstats) stats[i] = 0;
    if (i < 4) err[i] = 0;
  }
}

// ---------------------------------------------------------------------------
// k_track_ranges: packets grouped by track -> [begin, end) (+ grouping check)
// ---------------------------------------------------------------------------
// nDev (optional): the batch length lives on the device (an ingest-produced
// batch); n is then only the launch bound.
__global__ void k_track_ranges(const RunDesc *__restrict__ desc, u32 ntracks, u32 *__restrict__ tBegin,
                               u32 *__restrict__ tEnd, u32 *__restrict__ tRuns, u32 *__restrict__ err) {
  const lkf_pkt *__restrict__ pkts = reinterpret_cast<const lkf_pkt *>(desc->pkts);
  u32 n = desc->n;
  const u64 *nDev = reinterpret_cast<const u64 *>(desc->nDev);
  u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (nDev && *nDev < n) n = u32(*nDev);
  if (i >= n) return;
  u32 t = pkts[i].track;
  if (t >= ntracks) {
    atomicOr(err, 1u);
    return;
  }
  u32 tp = i > 0 ? pkts[i - 1].track : 0xffffffffu;
  u32 tn = i + 1 < n ? pkts[i + 1].track : 0xffffffffu;
  if (tp != t) {
    tBegin[t] = i;
    if (atomicAdd(&tRuns[t], 1u) != 0) atomicOr(err, 2u);
  }
  if (tn != t) tEnd[t] = i + 1;
}

// ---------------------------------------------------------------------------
// Scans (one launch: k_scan_1p).
// Value = (a, b) u64 pairs; mode selects how the input is formed.
// ---------------------------------------------------------------------------
constexpr int SCAN_T = 256;
#ifndef LKF_SCAN_ITEMS  // items per thread (tile = 256 x this): fewer tiles, a shorter look-back chain
#define LKF_SCAN_ITEMS 4
#endif
constexpr int SCAN_ITEMS = LKF_SCAN_ITEMS;
constexpr int SCAN_TILE = SCAN_T * SCAN_ITEMS;

struct ScanIn {
  int mode;  // 0: slots = npkts(track(d)) if active; 1: (fwdCnt, fwdBytes); 2: u32 flags;
             // 3: (word != 0, low 16 bits) of u32 words (RTCP NACKs and their pairs)
  const u32 *perm;  // position -> DownTrack (nullptr: identity)
  const DevDT *dts;
  const u32 *tBegin, *tEnd;
  const u32 *cnt;
  const u64 *bytes;
  u32 *gFirst;  // mode 1: emit group index (group g -> position owning record g*EMIT_G)
  u64 gCap;     // output record capacity (groups beyond it are never read)
};

__device__ __forceinline__ void scan_load(const ScanIn &in, u32 i, u64 &a, u64 &b) {
  const u32 d = in.perm ? in.perm[i] : i;
  if (in.mode == 3) {
    a = in.cnt[i] != 0 ? 1 : 0;
    b = in.cnt[i] & 0xffffu;
    return;
  }
  if (in.mode == 2) {  // u32 flags (ingress forward flags)
    a = in.cnt[i];
    b = 0;
    return;
  }
  if (in.mode == 0) {
    DevDT dt = in.dts[d];
    a = dt.active ? u64(in.tEnd[dt.track] - in.tBegin[dt.track]) : 0;
    b = 0;
  } else {
    a = in.cnt[d];
    b = in.bytes[d];
  }
}

__device__ __forceinline__ void block_scan_excl(u64 &a, u64 &b, u64 &ta, u64 &tb) {
  // inclusive wave scan
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  u64 ia = a, ib = b;
  for (int o = 1; o < 64; o <<= 1) {
    u64 xa = __shfl_up(ia, o, 64), xb = __shfl_up(ib, o, 64);
    if (lane >= o) {
      ia += xa;
      ib += xb;
    }
  }
  __shared__ u64 wa[SCAN_T / 64], wb[SCAN_T / 64];
  if (lane == 63) {
    wa[wid] = ia;
    wb[wid] = ib;
  }
  __syncthreads();
  u64 pa = 0, pb = 0;
  ta = tb = 0;
  for (int w = 0; w < SCAN_T / 64; w++) {
    if (w < wid) {
      pa += wa[w];
      pb += wb[w];
    }
    ta += wa[w];
    tb += wb[w];
  }
  __syncthreads();
  a = pa + ia - a;
  b = pb + ib - b;
}

// Single-pass scan (decoupled look-back): one launch instead of reduce / top
// / down — each is a dispatch on the prep or decide stream, and pipelined
// the stream's kernels wait for free CU slots one after another.  Tiles take
// ordered tickets; a tile publishes its aggregate at once, then looks back
// over its predecessors (aggregates, up to the first inclusive prefix) and
// publishes its own inclusive prefix.  A tile only waits on tiles that took
// their tickets earlier, so no co-residency is needed.  The hand-off is the
// guide's R2 form: each published value is 32-bit halves in 8-B {tag, value}
// granules stored and polled with agent-scope relaxed atomics (write-through
// sc1 stores, L1-bypassing loads), the tag the flag.  The last tile to arrive
// clears the granules and counters for the next launch on this state (the
// allocation is zeroed for the first); launches on one state are
// stream-ordered.
//   state: [0] tickets, [1] arrivals (u32 each in a u64 word), [2..15] pad,
//          then per tile 8 granules: aggregate (a lo, a hi, b lo, b hi),
//          inclusive prefix (a lo, a hi, b lo, b hi)
constexpr u32 kScanStHead = 16;
constexpr u32 kScanSpin = 1u << 22;  // polls before a look-back gives up (totals -> ~0: capacity errors)

// tag 1: the value; tag 2: poisoned (a look-back behind it gave up, so every
// prefix built on it is wrong: tiles that read it publish poison in turn and
// the last tile reports ~0 totals, a capacity error for the caller)
__device__ __forceinline__ void gr_put(u64 *g, u32 v, u32 tag = 1) {
  __hip_atomic_store(g, (u64(tag) << 32) | u64(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(SCAN_T) k_scan_1p(ScanIn in, u32 n, u32 nb, u64 *__restrict__ st,
                                                    u64 *__restrict__ outA, u64 *__restrict__ outB,
                                                    u64 *__restrict__ totA, u64 *__restrict__ totB) {
  __shared__ u32 sTile, sLast;
  __shared__ u64 sPre[2];
  __shared__ u32 sBad;
  u32 *const ctr = reinterpret_cast<u32 *>(st);
  u64 *const gr = st + kScanStHead;
  const u32 tid = threadIdx.x, lane = tid & 63;
  if (tid == 0) {
    sTile = atomicAdd(&ctr[0], 1u);
    sBad = 0;
  }
  __syncthreads();
  const u32 tile = sTile;
  const u32 i0 = tile * SCAN_TILE + tid * SCAN_ITEMS;  // blocked: a thread's items are consecutive
  u64 va[SCAN_ITEMS], vb[SCAN_ITEMS], ta = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    va[k] = vb[k] = 0;
    if (i0 + k < n) scan_load(in, i0 + k, va[k], vb[k]);
    ta += va[k];
    tb += vb[k];
  }
  u64 ea = ta, eb = tb, TA, TB;
  block_scan_excl(ea, eb, TA, TB);
  u64 *const g = gr + 8 * size_t(tile);
  if (tid == 0) {
    if (tile == 0) {
      gr_put(g + 4, u32(TA)), gr_put(g + 5, u32(TA >> 32)), gr_put(g + 6, u32(TB)), gr_put(g + 7, u32(TB >> 32));
      sPre[0] = sPre[1] = 0;
    } else {
      gr_put(g + 0, u32(TA)), gr_put(g + 1, u32(TA >> 32)), gr_put(g + 2, u32(TB)), gr_put(g + 3, u32(TB >> 32));
    }
  }
  if (tile > 0 && tid < 64) {  // look-back: lanes 0-7 read one predecessor's granules per poll
    u64 pa = 0, pb = 0;
    int j = int(tile) - 1;
    for (u32 spins = 0;;) {
      const u64 x = lane < 8 ? __hip_atomic_load(gr + 8 * size_t(j) + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : 0ull;
      const u64 rdy = __ballot(lane < 8 && (x >> 32) != 0);
      const u64 poison = __ballot(lane < 8 && (x >> 32) == 2);
      const u32 v = u32(x);
      if ((rdy & 0xF0) == 0xF0 || (rdy & 0x0F) == 0x0F) {
        const int o = (rdy & 0xF0) == 0xF0 ? 4 : 0;
        if (poison & (0x0Full << o)) {  // built on a look-back that gave up
          if (lane == 0) sBad = 1;
          break;
        }
        const u64 a = (u64(u32(__shfl(int(v), o + 1, 64))) << 32) | u32(__shfl(int(v), o, 64));
        const u64 b = (u64(u32(__shfl(int(v), o + 3, 64))) << 32) | u32(__shfl(int(v), o + 2, 64));
        pa += a;
        pb += b;
        if (o == 4) break;  // an inclusive prefix ends the walk (tile 0 always has one)
        j--;
        spins = 0;
        continue;
      }
      if (++spins > kScanSpin) {
        if (lane == 0) sBad = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) {
      const u64 ia = pa + TA, ib = pb + TB;
      const u32 tag = sBad ? 2u : 1u;
      gr_put(g + 4, u32(ia), tag), gr_put(g + 5, u32(ia >> 32), tag), gr_put(g + 6, u32(ib), tag),
          gr_put(g + 7, u32(ib >> 32), tag);
      sPre[0] = pa;
      sPre[1] = pb;
    }
  }
  __syncthreads();
  u64 ca = sPre[0] + ea, cb = sPre[1] + eb;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const u32 d = i0 + k;
    if (d < n) {
      outA[d] = ca;
      if (outB) outB[d] = cb;
      // emit groups of 64 records whose first record belongs to position d
      if (in.gFirst && va[k]) {
        const u64 r0 = ca, r1 = min(r0 + va[k], in.gCap);
        for (u64 gg = (r0 + 63) >> 6; (gg << 6) < r1; gg++) in.gFirst[gg] = d;
      }
    }
    ca += va[k];
    cb += vb[k];
  }
  if (tile == nb - 1 && tid == 0) {
    *totA = sBad ? ~0ull : sPre[0] + TA;
    if (totB) *totB = sBad ? ~0ull : sPre[1] + TB;
  }
  // the last tile to arrive clears the state for the next launch
  __syncthreads();
  if (tid == 0) sLast = atomicAdd(&ctr[2], 1u) == nb - 1 ? 1u : 0u;
  __syncthreads();
  if (sLast) {
    for (u32 k = tid; k < 8 * nb; k += SCAN_T)
      __hip_atomic_store(gr + k, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) {
      __hip_atomic_store(&ctr[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctr[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// k_decide_dt arguments.
// ---------------------------------------------------------------------------
struct DecideArgs {
  const u32 *sched;      // lane -> DownTrack (0xffffffff = idle lane)
  const u32 *waveTrack;  // wave -> track (every lane of a wave serves one track)
  u32 nlanes;
  DTHot *hot;
  const DevDT *dts;
  const DevTrack *tracks;
  RangeEntry *rm;
  VP8Cold *vc;
  SeqMeta *seq;
  u32 seqSize;
  u8 *srm;  // SeqRM regions (stride srmStride), read with F_SEQ_RM
  u64 srmStride;
  u32 srmCap;
  const lkf_pkt *pkts;
  const u32 *tBegin, *tEnd;
  const u64 *slotBase;
  FwdRec *recs;
  FwdBase *fbase;  // per DownTrack: its first forwarded record's munged SN / TS (FwdRec widening)
  FwdBase *wide;   // per tuple slot: the full SN / TS of a T_WIDE record
  u64 tupleCap;
  u32 *err;
  SenderStats *ss;  // RTPStatsSender per DownTrack (+ snInfo ring, gap histogram)
  u32 *ssRing, *ssGap;
  u32 *dtOffs;      // per DownTrack reference-layer offsets (kDTOffsWords)
  const DevEvent *events;
  const u32 *evOff;  // per lane [evOff[l], evOff[l+1])
  u32 *fwdCnt;
  u64 *fwdBytes;
  DTCum *dtCum;  // per DownTrack totals (sendingPacket counters)
  u64 *stats;  // lkf_stats as u64[15]
  const u32 *layerList, *layerBefore, *layerCnt;  // k_layer_index
  u32 pktStride;
  u32 waveBase;  // schedule index of this launch's first wave
  u32 waveEnd;   // schedule index after this launch's last wave
  u32 perWave;   // DownTracks (schedule slots) per wave: 1 for long batches, more for short ticks
  // dependency descriptor (F_DD DownTracks)
  const DDPkt *ddPkts;
  const DDStruct *ddStructs;
  DDState *ddState;
  u8 *ddArena;
  u64 *ddUsed;
  u64 ddCap;
  const u16 *ddSpill;
  // capacities (checked builds test device-computed indices against them)
  u32 maxDts, maxTracks, npkts, nev;
};

struct SsEnt;
// One wave per (track, <=64 DownTracks): the packet loop is wave-uniform, so
// packet descriptors come through the scalar cache and every branch on packet
// fields is a scalar branch; lanes diverge only on per-DownTrack state.
// Per (packet, DownTrack) body of DownTrack.WriteRTP (downtrack.go:680-760).
struct LaneOut {
  FwdRec *outT;
  FwdBase *outW;  // the wide side array at this DownTrack's first slot (T_WIDE records)
  u64 nFwd, nBytes, nTuples;
  u64 bSN, bTS;  // the batch's first forwarded munged SN / TS (FwdBase)
  SenderStats *ss;  // the DownTrack's RTPStatsSender, staged in LDS
  u32 *ssRing, *ssGap;
  SsEnt *ssBuf;  // this chunk's forwarded tuples for ss_flush (LDS)
  u32 ssN;
  i32 sentDiff;  // sendingPacket's bytesSent - sum of out_len: incoming minus outgoing header bytes
  u32 relOff;
  u32 drops[LKF_DROP_NREASONS];
  u8 *ddArena;  // this batch's marshalled DD bytes (bump-allocated)
  u64 *ddUsed;
  u64 ddCap;
#if LKF_CHECKED
  u64 tupBase, tupCap;  // this DownTrack's first tuple slot, the batch's capacity
#endif
};

__device__ __forceinline__ double rl_f64(double v, u32 k) {
  return __builtin_bit_cast(double, rl64(__builtin_bit_cast(u64, v), k));
}

// DownTrack.sendingPacket -> RTPStatsSender.Update (downtrack.go:1930-1959,
// rtpstats_sender.go:229-432) inside the decide wave.  Every forwarded tuple
// appends one 24-B entry to the wave's LDS buffer (SsEnt: munged SN / TS low
// bits against the batch base, arrival, incoming header size, forwarded
// payload, marker / key frame) in send order; at the end of each chunk (at
// most 64 packets, so at most 64 entries) ss_flush folds the buffer into the
// DownTrack's RTPStatsSender (LDS copy, written back once per batch).  The
// fold runs where the chunk's registers are dead, so the run body keeps its
// register budget.
struct SsEnt {
  u32 sn, ts;   // low 32 bits of the munged extended SN / TS (widened against FwdBase)
  i64 t;        // arrival (the virtual clock of sendingPacket)
  u32 hp;       // incoming header size | forwarded payload << 16
  u32 fl;       // 1 marker, 2 key frame
};
static_assert(sizeof(SsEnt) == 24, "SsEnt is 24 B");
__device__ __forceinline__ void ss_put(SsEnt *e, u64 sn, u64 ts, i64 t, u32 hdr, u32 pay, bool marker, bool kf) {
  *reinterpret_cast<uint2 *>(e) = make_uint2(u32(sn), u32(ts));
  reinterpret_cast<uint2 *>(e)[1] = make_uint2(u32(u64(t)), u32(u64(t) >> 32));
  reinterpret_cast<uint2 *>(e)[2] = make_uint2(hdr | (pay << 16), (marker ? 1u : 0u) | (kf ? 2u : 0u));
}

// The fold of m entries, lane = entry.  A segment of in-order entries — each
// above the one before it by at most 64, with a payload, not moving the
// timestamp backwards — only accumulates: per lane the gap histogram, the
// cleared snInfo slots of the SNs it skips and its own slot (distinct: a
// segment spans at most 4096 SNs); the counters as wave sums; the highest
// timestamp and its time from the last lane that raised it; the jitter filter
// (a float64 recurrence, rtpstats_base.go:775-813) stepped over the segment's
// new frames on uniform values.  The entry that ends a segment (out of order,
// duplicate, a larger gap, the first packet) takes the scalar Update,
// wave-uniform.
#ifndef LKF_SS_SCALAR  // chunks of at most this many forwarded tuples fold entry by entry
#define LKF_SS_SCALAR 0  // (3 measured slower: headline +1.5 %, tick +1.2 %; r5 A/B)
#endif
__device__ __forceinline__ void ss_flush(SenderStats &S, u32 *ring, u32 *gap, const SsEnt *buf, u32 m, u64 bSN,
                                      u64 bTS) {
  if (m <= u32(LKF_SS_SCALAR)) {  // a short chunk (the short ticks): the scalar Update per entry,
    for (u32 i = 0; i < m; i++) {  // cheaper than the segment's cross-lane reductions
      const SsEnt &e = buf[i];
      ss::ss_update(S, ring, gap, e.t, widen32(bSN, e.sn), widen32(bTS, e.ts), (e.fl & 1) != 0, e.hp & 0xffffu,
                    e.hp >> 16, 0);
      if (e.fl & 2) S.keyFrames++;  // UpdateKeyFrame(1) rtpstats_base.go:429-439
      wave_lds_sync();
    }
    return;
  }
  const u32 lane = lane_id();
  const u64 lt = (1ull << lane) - 1;
  const bool valid = lane < m;
  u64 esn = 0, ets = 0;
  i64 t = 0;
  u32 hdr = 0, pay = 0;
  bool marker = false, kf = false;
  if (valid) {
    const SsEnt &e = buf[lane];
    esn = widen32(bSN, e.sn);
    ets = widen32(bTS, e.ts);
    t = e.t;
    hdr = e.hp & 0xffffu;
    pay = e.hp >> 16;
    marker = e.fl & 1;
    kf = e.fl & 2;
  }
  const u64 pEsn = sh64(esn, lane ? int(lane) - 1 : 0), pEts = sh64(ets, lane ? int(lane) - 1 : 0);
  u32 pos = 0;
  while (pos < m) {
    const bool inSeg = valid && lane >= pos;
    const u64 prev = lane > pos ? pEsn : S.extHighestSN;
    const u64 g = esn - prev;
    const bool ok = S.initialized && pay > 0 && i64(g) > 0 && g <= 64 && ets >= S.extStartTS &&
                    (lane == pos || ets >= pEts);
    const u64 badM = __ballot(inSeg && !ok);
    const u32 end = badM ? u32(__ffsll((long long)badM) - 1) : m;
    if (end > pos) {
      const bool act = lane >= pos && lane < end;
      if (act && g >= 2) {  // updateGapHistogram; clearSnInfos(prev + 1, esn)
        atomicAdd(&gap[g - 1 > u64(kGapBins) ? kGapBins - 1 : u32(g - 2)], 1u);
        for (u64 q = prev + 1; q != esn; q++) ring[q & ss::kSnMask] = 0;
      }
      if (act)  // setSnInfo
        ring[esn & ss::kSnMask] =
            u32(u16(hdr + pay)) | (u32(u8(hdr)) << 16) | ((marker ? ss::kFlagMarker : 0u) << 24);
      // highest timestamp: the lanes above every earlier one (non-decreasing in the segment)
      const u64 before = (lane > pos && pEts > S.extHighestTS) ? pEts : S.extHighestTS;
      const u64 upM = __ballot(act && ets > before);
      // the jitter's new frames: a timestamp other than the previous packet's
      const bool isNew = act && ets != (lane > pos ? pEts : S.lastJitterExtTimestamp);
      const u64 newM = __ballot(isNew);
      const i64 since = i64(u64(t) - u64(S.firstTime));
      const u64 rtp = u64(i64(u64(since) * u64(i64(S.clockRate))) / 1000000000LL);
      const u64 transit = rtp - ets;
      const int pn = prev_in(newM, lt);
      const u64 pnT = sh64(transit, pn >= 0 ? pn : int(lane));
      const u64 prevTransit = pn >= 0 ? pnT : S.lastTransit;
      i64 dj = i64(transit - prevTransit);
      if (dj < 0) dj = i64(0 - u64(dj));
      const double dd = double(dj);
      const u64 useM = __ballot(isNew && prevTransit != 0);
      // the segment's totals (<= 64 packets: the sums fit 32 bits)
      const u32 sumB = wave_sum_u32(act ? hdr + pay : 0u), sumH = wave_sum_u32(act ? hdr : 0u);
      const u32 lost = wave_sum_u32((act && g >= 2) ? u32(g - 1) : 0u);
      const u32 frames = u32(__popcll(__ballot(act && marker))), kfs = u32(__popcll(__ballot(act && kf)));
      double j = S.jitter, mj = S.maxJitter;
      for (u64 w = newM; w; w &= w - 1) {
        const u32 k = u32(__ffsll((long long)w) - 1);
        if ((useM >> k) & 1) {
          j += (rl_f64(dd, k) - j) / 16;
          if (j > mj) mj = j;
        }
      }
      const u64 lastEsn = rl64(esn, end - 1);
      u64 trL = 0, etsL = 0, tU = 0, etsU = 0;
      if (newM) {
        const u32 kl = 63 - __clzll(newM);
        trL = rl64(transit, kl);
        etsL = rl64(ets, kl);
      }
      if (upM) {
        const u32 ku = 63 - __clzll(upM);
        tU = rl64(u64(t), ku);
        etsU = rl64(ets, ku);
      }
      wave_lds_sync();
      if (lane == 0) {
        S.jitter = j;
        S.maxJitter = mj;
        if (newM) {
          S.lastTransit = trL;
          S.lastJitterExtTimestamp = etsL;
        }
        if (upM) {
          S.highestTime = i64(tU);
          S.extHighestTS = etsU;
        }
        S.extHighestSN = lastEsn;
        S.packetsLost += lost;
        S.bytes += sumB;
        S.headerBytes += sumH;
        S.frames += frames;
        S.keyFrames += kfs;
      }
      wave_lds_sync();
    }
    pos = end;
    if (pos < m) {  // the entry that ends the segment: the scalar Update (every lane, uniform arguments)
      ss::ss_update(S, ring, gap, i64(rl64(u64(t), pos)), rl64(esn, pos), rl64(ets, pos), rl32(u32(marker), pos) != 0,
                    rl32(hdr, pos), rl32(pay, pos), 0);
      if (rl32(u32(kf), pos)) S.keyFrames++;  // UpdateKeyFrame(1) rtpstats_base.go:429-439
      wave_lds_sync();
      pos++;
    }
  }
}

// FwdBase: a DownTrack's first forwarded record of the batch sets it
__device__ __forceinline__ void fwd_base(LaneOut &o, u64 fwM, u64 osn, u64 ots) {
  if (!fwM || o.nFwd != 0) return;
  const u32 f0 = u32(__ffsll((long long)fwM) - 1);
  o.bSN = rl64(osn, f0);
  o.bTS = rl64(ots, f0);
}

template <bool DDK>
__device__ __forceinline__ void decide_step(Lane &L, const PktV &p, u32 k, LaneOut &o) {
  o.nTuples++;
  Fwd f;
  // Fast classification (pre-state + packet only); anything not covered
  // takes the full restatement fw_translate.  Each fast case is exactly the
  // path forwarder.go would take for it:
  //   muted/pubMuted -> drop (:1440); video with invalid target -> drop (:1687);
  //   no switch possible in Simulcast.Select and layer != current -> drop (:1694);
  //   pause-on-downgrade -> drop (:1709);
  //   same SSRC, contiguous SN with payload -> UpdateAndGetSnTs in-order branch,
  //   then (video) SelectTemporal + VP8 UpdateAndGet without gap/OOO.
  const u32 fl = L.h.flags;
  const bool contig = p.ssrc == L.h.lastSSRC && p.plen != 0 && p.esn == L.h.extHighestIncomingSN + 1;
  int dr;
  f.switching = f.resuming = false;
  f.cbLen = 0;
  f.cb = 0;
  f.ddLen = 0;
  f.ord = ORD_CONTIG;
  int cls;  // -1 fast forward, -2 slow, >= 0 drop
  const i32 layer = p.layer;
  const bool kf = p.flags & LKF_PKT_KEYFRAME;
  if (fl & (F_MUTED | F_PUBMUTED)) {
    cls = LKF_DROP_MUTED;
  } else if (!(fl & F_VIDEO)) {
    cls = contig ? -1 : -2;
  } else if (L.h.tgtS == INVALID || L.h.tgtT == INVALID) {
    cls = LKF_DROP_PAUSED;
  } else if (!(fl & F_SIMULCAST)) {
    cls = (fl & (F_VP9 | F_DD)) ? -2 : LKF_DROP_NOT_SELECTED;  // SVC: full step (relevant drops move the munger)
  } else {
    const bool willSwitch =
        kf && ((L.h.curS != L.h.tgtS && ((layer > L.h.curS && layer <= L.h.tgtS) ||
                                         (layer < L.h.curS && layer >= L.h.tgtS))) ||
               (L.h.curS > L.h.maxS && layer <= L.h.maxS));
    if (willSwitch)
      cls = -2;
    else if (layer != L.h.curS)
      cls = LKF_DROP_NOT_SELECTED;
    else if ((fl & F_DEFICIENT) && L.h.tgtS < L.h.curS)
      cls = LKF_DROP_DOWNGRADE;
    else if (contig && (fl & F_VP8) && (p.flags & LKF_PKT_VP8) && (fl & F_TLS_VP8))
      cls = -1;
    else
      cls = -2;
  }
  if (cls >= 0) {
    dr = cls;
  } else if (cls == -2) {
    dr = fw_translate<DDK>(L, p, k, f);
  } else if (!(fl & F_VIDEO)) {
    f.marker = false;
    mg_inorder(L, p, false, f.osn, f.ots);
    dr = -1;
  } else {
    const bool pktMarker = p.hdr1 & 0x80;
    f.marker = pktMarker;
    mg_inorder(L, p, pktMarker, f.osn, f.ots);
    // SelectTemporal (base.go:143-168, temporallayerselector/vp8.go:32-56)
    i32 tl = L.h.curT;
    bool tSwitch = false;
    {
      const i32 cur = L.h.curT, tgt = L.h.tgtT;
      i32 nxt = cur;
      if (cur != tgt && (p.vbits & LKF_VP8_T)) {
        const i32 tid = i32(p.tid);
        if (cur < tgt) {
          if (tid > cur && tid <= tgt && (p.vbits & LKF_VP8_S) && (p.vbits & LKF_VP8_Y)) {
            tl = tid;
            nxt = tid;
          }
        } else if (pktMarker) {
          nxt = tgt;
        }
      }
      if (nxt != L.h.curT) {
        tSwitch = true;
        L.h.prevS = L.h.curS;
        L.h.prevT = L.h.curT;
        L.h.curT = nxt;
      }
    }
    const int cr = vp8_update(L, p, false, false, tl, f.cb, f.cbLen);
    if (cr != CM_OK) {
      if (cr == CM_FILTERED) mg_packetDropped(L, p.esn);
      if (tSwitch) vls_rollback(L);
      dr = cr == CM_FILTERED ? LKF_DROP_TEMPORAL : cr == CM_PICID_MISS ? LKF_DROP_PICID_MISS : LKF_DROP_OTHER;
    } else {
      dr = -1;
    }
  }
  if (dr >= 0) {
#pragma unroll
    for (int i = 0; i < LKF_DROP_NREASONS; i++) o.drops[i] += (dr == i) ? 1u : 0u;
    return;
  }
  // ---- output shape (downtrack.go:693-723, pacer/base.go:71-100): the DD
  // element first (pion picks the two-byte profile when it exceeds 16 B),
  // then playout delay, then abs-send-time
  const int cc = p.hdr0 & 0xf;
  const bool playout = L.extPlayout && !hasf(L, F_PLAYOUT_ACKED);
  const bool ddOn = DDK && f.ddLen > 0 && L.extDD;
  const int eh = (ddOn && f.ddLen > 16) ? 2 : 1;  // element header bytes
  // (+ the transport-cc element pion's TWCC interceptor appends after the pacer's, 2 bytes)
  int extBytes = (ddOn ? eh + f.ddLen : 0) + (playout ? eh + 3 : 0) + (L.extAbs ? eh + 3 : 0) + (L.extTcc ? eh + 2 : 0);
  int extBlock = extBytes ? 4 + ((extBytes + 3) & ~3) : 0;
  int hdrLen = 12 + 4 * cc + extBlock;
  const bool useCodec = f.cbLen > 0 && (p.flags & LKF_PKT_VP8);
  int payLen = useCodec ? (f.cbLen + int(p.plen) - int(p.vhs)) : int(p.plen);
  const bool marker = f.marker || (p.hdr1 & 0x80);
  u32 flags = (f.switching ? LKF_OUT_SWITCHING : 0) | (f.resuming ? LKF_OUT_RESUMING : 0) |
              ((p.flags & LKF_PKT_KEYFRAME) ? LKF_OUT_KEYFRAME : 0) | (marker ? LKF_OUT_MARKER : 0) |
              (playout ? T_PLAYOUT : 0) | (useCodec ? T_CODEC : 0) | (ddOn ? T_DD : 0);
  u32 ddLen = ddOn ? u32(f.ddLen) : 0u;
  u32 aux = useCodec ? vp8_aux_of(f.cb) : 0u;
  if (DDK && ddOn) {  // the marshalled DD bytes go to the batch's DD arena (read by k_emit)
    u64 off = 0;
    if (lane_id() == 0) off = atomicAdd((unsigned long long *)o.ddUsed, (unsigned long long)f.ddLen);
    off = rl64(off, 0);
    if (off + u64(f.ddLen) > o.ddCap) {
      if (lane_id() == 0) atomicOr(L.err, 64u);  // (the DD arena)
      flags &= ~u32(T_DD);
      ddLen = 0;
    } else {
      wave_lds_sync();
      for (int i = int(lane_id()); i < f.ddLen; i += 64) o.ddArena[off + u64(i)] = L.ddBuf[i];
      aux = u32(off);
    }
  }
#if LKF_CHECKED
  CHK(o.tupBase + o.nFwd < o.tupCap, CK_DEC_TUPLE, o.tupBase + o.nFwd, o.tupCap);
#endif
  fwd_base(o, 1ull, f.osn, f.ots);
  if (lane_id() == 0)  // wave-uniform record: one lane stores it
    store_fwd(o.outT + o.nFwd, o.outW + o.nFwd, o.bSN, o.bTS, f.osn, f.ots, k, o.relOff, u32(hdrLen + payLen), flags,
              ddLen, aux);
  // sequencer.push (downtrack.go:724-735)
  seq_push<DDK>(L, p.arr / 1000000LL, p.esn, f.osn, f.ots, marker, p.layer, f.cb, f.cbLen);
  // sendingPacket -> RTPStatsSender.Update start (rtpstats_sender.go:245-262)
  if (!hasf(L, F_STATS_INIT) && payLen > 0) {
    setf(L, F_STATS_INIT, true);
    L.h.statsFirstTime = p.arr;
    L.h.statsExtStartTS = f.ots;
  }
  // sendingPacket -> RTPStatsSender.Update (downtrack.go:1930-1959): the
  // incoming header's size (getTranslatedRTPHeader keeps its extensions) and
  // the forwarded payload, folded at the end of the chunk (ss_flush)
  if (lane_id() == 0)
    ss_put(o.ssBuf + o.ssN, f.osn, f.ots, p.arr, p.poff, u32(payLen), marker, (p.flags & LKF_PKT_KEYFRAME) != 0);
  o.ssN++;
  o.nFwd++;
  o.nBytes += u64(hdrLen + payLen);
  o.sentDiff += i32(p.poff) - hdrLen;  // getTranslatedRTPHeader keeps the incoming extensions (downtrack.go:1714-1726)
  o.relOff += u32((hdrLen + payLen + 15) & ~15);
}

// ---------------------------------------------------------------------------
// k_decide_dt: one wave per DownTrack, lanes = packets of its track.
//
// The per-DownTrack recurrence is serial in the reference (one Forwarder
// behind a mutex), but almost every packet takes a branch whose effect on
// the state is a prefix count: packets of other simulcast layers are dropped
// without touching state (simulcast.go:42-122 with no switch possible), and
// in-order contiguous packets of the current layer either forward with
// SN = esn - snOffset (rtpmunger.go:186-217) or are dropped by the VP8
// temporal filter, which shifts snOffset and pictureIdOffset by one
// (rtpmunger.go:156-181, vp8.go:266-280).  A chunk of 64 packets is loaded
// one per lane; every lane classifies its packet against the DownTrack state
// at the start of the run; the longest prefix of lanes whose packets are
// covered is decided in parallel (ballot + popcount prefixes give the
// offsets, output slots and sequencer slots), and the state is advanced once.
// The first packet that is not covered (gap, reorder, duplicate, layer or
// temporal switch point, keyframe, SSRC change, picture-id wrap, pending
// control op) goes through decide_step — the full restatement — executed by
// the whole wave on the broadcast packet, and the run restarts after it.
// ---------------------------------------------------------------------------

#ifndef LKF_DECIDE_WAVES  // occupancy floor (waves per SIMD); 4 and 6 measured slower (r3, r5)
#define LKF_DECIDE_WAVES 5
#endif
// (the DD selector's instantiation cannot reach that floor: at 3 waves per
// SIMD it fits 168 VGPRs with 176 B of spills, 2 % faster on configs[4] than 2
// waves at 254 VGPRs; asked for 5 the compiler gives up and drops to 1 wave)
#ifndef LKF_DECIDE_DD_WAVES
#define LKF_DECIDE_DD_WAVES 3
#endif
#define DECIDE_ATTR __attribute__((amdgpu_waves_per_eu(DDK ? LKF_DECIDE_DD_WAVES : LKF_DECIDE_WAVES, 8)))

// Consume the chunk's descriptor registers here, once.  gfx9 counts stores in
// vmcnt too: a first use sunk into the run loop would wait there for every
// tuple/sequencer store issued so far (one HBM write round trip per run).
// Waits for this wave's outstanding vector-memory ops (s_waitcnt vmcnt(0);
// gfx9 encoding: expcnt and lgkmcnt left at their maxima).  Placed at the end
// of the rare paths that load from global memory (control ops, the full
// per-packet step), so the waitcnt pass does not see a load that may still be
// pending at the run-loop head and insert a vmcnt(0) there — which, with
// stores counted in vmcnt, would stall every run on the previous run's
// tuple/sequencer stores.
__device__ __forceinline__ void vm_drain() {
  __builtin_amdgcn_s_waitcnt(0x0F70);
}

__device__ __forceinline__ void pin_loaded(const uint4 &a, const uint4 &b, const uint4 &c, const uint4 &d) {
  asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(c.x),
               "v"(c.y), "v"(c.z), "v"(c.w), "v"(d.x), "v"(d.y), "v"(d.z), "v"(d.w));
}

__device__ __forceinline__ bool steady_state(const Lane &L) {
  const u32 fl = L.h.flags;
  return (fl & F_VIDEO) && (fl & F_SIMULCAST) && !(fl & (F_MUTED | F_PUBMUTED)) &&
         L.h.tgtS != INVALID && L.h.tgtT != INVALID && L.h.curS == L.h.tgtS && L.h.curS <= L.h.maxS &&
         L.h.curS >= 0 && L.h.curS < 3;
}

// Per-track layer lists for the steady-state chunks of k_decide_dt: one wave
// per track; for each simulcast layer l, list[l][tBegin + j] = the j-th packet
// of layer l and before[l][i] = the number of layer-l packets of the track
// before packet i.
__global__ void __launch_bounds__(64) k_layer_index(const RunDesc *__restrict__ desc, const u32 *__restrict__ tBegin,
                                                    const u32 *__restrict__ tEnd, u32 stride, u32 *__restrict__ list,
                                                    u32 *__restrict__ before, u32 *__restrict__ cnt,
                                                    u64 *__restrict__ zero2) {
  const lkf_pkt *__restrict__ pkts = reinterpret_cast<const lkf_pkt *>(desc->pkts);
  const u32 t = blockIdx.x, lane = threadIdx.x;
  // (the batch's DD bump cursors start at zero: a kernel store on the prep
  // chain rather than a memset node in the captured prep graph)
  if (zero2 && t == 0 && lane < 2) zero2[lane] = 0;
  const u64 lt = (1ull << lane) - 1;
  const u32 b = tBegin[t], e = tEnd[t];
  u32 c0 = 0, c1 = 0, c2 = 0;
  for (u32 base = b; base < e; base += 64) {
    const u32 i = base + lane;
    const int l = i < e ? int(reinterpret_cast<const int8_t *>(pkts + i)[53]) : -1;  // lkf_pkt.layer
    const u64 m0 = __ballot(l == 0), m1 = __ballot(l == 1), m2 = __ballot(l == 2);
    if (i < e) {
      const u32 r0 = c0 + u32(__popcll(m0 & lt)), r1 = c1 + u32(__popcll(m1 & lt)), r2 = c2 + u32(__popcll(m2 & lt));
      before[i] = r0;
      before[stride + i] = r1;
      before[2 * size_t(stride) + i] = r2;
      if (l == 0) list[b + r0] = i;
      if (l == 1) list[stride + b + r1] = i;
      if (l == 2) list[2 * size_t(stride) + b + r2] = i;
    }
    c0 += u32(__popcll(m0));
    c1 += u32(__popcll(m1));
    c2 += u32(__popcll(m2));
  }
  if (lane == 0) {
    cnt[t * 3] = c0;
    cnt[t * 3 + 1] = c1;
    cnt[t * 3 + 2] = c2;
  }
}

// ---------------------------------------------------------------------------
// SVC runs (F_DD / F_VP9 DownTracks).  One SSRC carries every layer, so a
// packet the layer selector does not select is still relevant to it and
// advances the munger (forwarder.go:1694-1702): dropped at the highest SN it
// is excluded (rtpmunger.go:156-181, the prefix-count shape of a VP8 temporal
// drop); after a loss gap it takes its SN like a forwarded packet.  Per lane
// the selector's decision is a function of the packet and the state at the run
// start as long as no switch happens:
//   VP9.Select (videolayerselector/vp9.go:43-109): with a switch pending, a
//   packet that is not its switch point is decided against the current layers;
//   with no current layers, a non-key-frame packet is dropped unselected and
//   irrelevant;
//   DependencyDescriptor.Select (dependencydescriptor.go:65-355): the decode
//   target the state selects (uniform while no chain breaks) and the frame's
//   DTI for it; a frame already dropped drops its later packets (GetDecision);
//   chains and frame references are verified against the decision cache at
//   the run start plus the decisions of the run's earlier frames; frames added
//   to the cache (a dropped frame's first packet, a forwarded frame's packets
//   with frame integrity, :245-247) update it as addEntity does, gaps included.
// Muted / paused DownTracks drop every packet with no state change.  Packets
// without a descriptor, not selected, dropped by pause-on-downgrade (VP9) or
// before the Forwarder started drop as the reference does.  The longest
// prefix of lanes meeting these conditions is decided together; the first lane
// that does not (a switch point, a chain break, a structure or active-target
// update, a reorder, padding) goes through decide_step, as in the simulcast
// runs.
// ---------------------------------------------------------------------------
#ifndef LKF_SVC_CHAINS  // chain breaks / restarts decided in SVC runs (0: they end the run; A/B)
#define LKF_SVC_CHAINS 1
#endif
constexpr int kSvcDDBytes = 48;  // per-lane marshal buffer (a descriptor without a structure fits)
constexpr int kSvcFrames = 72;   // frame decisions of one run: frame cLast + up to 64 later frames
enum : u32 { SK_BAD = 0, SK_FWD = 1, SK_MDROP = 2, SK_NDROP = 3 };  // lane kinds of an SVC run

// LKF_SVC_STATS=1 (diagnostic builds): where SVC runs stop.  g_svc[0] runs,
// [1] packets decided in runs, [2] full steps after a run, [3] runs refused
// at the start (no keyframe / cache yet), [16 + c] the stopping lane's first
// failed condition c (the SVC_WHY codes below; 15: the window ended).
#if LKF_SVC_STATS
#define SVC_WHY(c) \
  if (why == 0 && inWin && !good) why = (c)
#else
#define SVC_WHY(c)
#endif

template <bool DDK>
__device__ __forceinline__ u32 svc_run(Lane &L, LaneOut &o, const PktV &p, u32 pi, u32 n, u32 pos, u32 nextAt,
                                       bool valid, i32 &sentAcc, u8 *sScr, u8 *sFD) {
  const u32 lane = lane_id();
  const u64 lt = (1ull << lane) - 1;
  const u32 fl = L.h.flags;
  const bool inWin = valid && lane >= pos && pi < nextAt;
  const u64 winM = __ballot(inWin);
  const bool dd = DDK && (fl & F_DD);
  // ---- muted / paused: every packet of the window drops with no state change
  // (forwarder.go:1440, :1687)
  {
    const int ns = (fl & (F_MUTED | F_PUBMUTED)) ? LKF_DROP_MUTED
                   : (L.h.tgtS == INVALID || L.h.tgtT == INVALID) ? LKF_DROP_PAUSED
                                                                  : -1;
    if (ns >= 0) {
      const u32 k = u32(__popcll(winM));
      o.nTuples += k;
      if (ns == LKF_DROP_MUTED)
        o.drops[LKF_DROP_MUTED] += k;
      else
        o.drops[LKF_DROP_PAUSED] += k;
      return pos + k;
    }
  }
  const bool curValid = L.h.curS != INVALID && L.h.curT != INVALID;
  const bool started = fl & F_STARTED;
  const bool relevantDrop = curValid && started;  // a not-selected packet advances the munger
  // ---- dependency-descriptor selector: the uniform part
  bool uni = true;
  const DDStruct *s = nullptr;
  int hiPos = -1, maxTgt = -1;
  u32 hiTarget = 0;
  bool swAll = false;  // a selected packet would switch layers
  // chains whose restart would change the selection: those of the eligible
  // decode targets above the selected one (all broken, or one would have been
  // picked); the selected target's own chain (hiChain) may not break in a run
  u32 aboveM = 0, hiChain = 0xffffffffu;
  if (DDK && dd) {
    const DDState &d = *L.dd;
    uni = (d.flags & DS_KF_VALID) && (d.flags & DS_CACHE_INIT);
    uni = uni && u32(d.slot) == L.ddSSlot;  // (the structure in force is the staged one)
    s = L.ddS;
    for (int i = 0; uni && i < int(d.numTargets); i++) {  // the decode target Select picks (:133-176)
      if (!((d.dtActive >> i) & 1) || i32(s->dtS[i]) > L.h.tgtS || i32(s->dtT[i]) > L.h.tgtT) continue;
      const int target = s->dtTarget[i];
      maxTgt = max(maxTgt, target);
      if (d.numChains == 0 || !((d.chBroken >> s->protectedBy[target]) & 1)) {
        hiPos = i;
        hiTarget = u32(target);
        if (d.numChains) hiChain = s->protectedBy[target];
        break;
      }
      aboveM |= 1u << s->protectedBy[target];
    }
    swAll = hiPos >= 0 && (i32(s->dtS[hiPos]) != L.h.curS || i32(s->dtT[hiPos]) != L.h.curT);
  }
#if LKF_SVC_STATS
  if (!uni && lane == 0) SVC_ADD(3, 1ull);
  u32 why = 0;
#endif
  if (!uni) return pos;
#if LKF_SVC_STATS
  const u64 tA = __builtin_amdgcn_s_memtime();
  u64 tB = tA, tC = tA;
#endif
  bool good = inWin;
  u32 kind = SK_BAD;
  int nsr = LKF_DROP_NOT_SELECTED;  // reason of an SK_NDROP lane
  bool mk = false;                  // marker passed to UpdateAndGetSnTs
  int ddLen = 0;
  u64 ddEfn = 0;
  bool ddPut = false, ddFwdSel = false;
  u32 chBrk = 0, chRst = 0;  // chains this lane breaks / restarts (FrameChain.OnFrame)
  if (!dd) {  // ---- VP9.Select
    const bool isV = p.flags & LKF_PKT_VP9;
    const bool U = p.vp9 & LKF_VP9_U, B = p.vp9 & LKF_VP9_B, E = p.vp9 & LKF_VP9_E, P = p.vp9 & LKF_VP9_P;
    const i32 pS = p.spatial, pT = p.temporal;
    const bool kf = p.flags & LKF_PKT_KEYFRAME;
    bool zero = !isV, sw = false;
    if (isV && (L.h.curS != L.h.tgtS || L.h.curT != L.h.tgtT)) {
      if (!curValid) {
        if (kf)
          sw = true;
        else
          zero = true;  // (vp9.go:55-57)
      } else {
        i32 uS = L.h.curS, uT = L.h.curT;
        if (L.h.curT != L.h.tgtT) {
          if (L.h.curT < L.h.tgtT) {
            if (pT > L.h.curT && pT <= L.h.tgtT && U && B) uT = pT;
          } else if (E) {
            uT = L.h.tgtT;
          }
        }
        if (L.h.curS != L.h.tgtS) {
          if (L.h.curS < L.h.tgtS) {
            if (pS > L.h.curS && pS <= L.h.tgtS && !P && B) uS = pS;
          } else if (E) {
            uS = L.h.tgtS;
          }
        }
        sw = uS != L.h.curS || uT != L.h.curT;
      }
    }
    good = good && !sw;  // a switch point: full step
    SVC_WHY(2);
    const bool sel = !zero && !(pS > L.h.curS || (pS == L.h.curS && pT > L.h.curT));
    mk = (p.hdr1 & 0x80) || (!zero && E && pS == L.h.curS && (P || L.h.tgtS <= L.h.curS));
    if (!sel) {
      kind = (!zero && started) ? SK_MDROP : SK_NDROP;
    } else if ((fl & F_DEFICIENT) && L.h.tgtS < L.h.curS) {  // FlagPauseOnDowngrade :1709
      kind = SK_NDROP;
      nsr = LKF_DROP_DOWNGRADE;
    } else {
      kind = SK_FWD;
    }
  } else if (DDK) {  // ---- DependencyDescriptor.Select
    DDState &d = *L.dd;
    DDPkt dp;  // (the scalar fields only: the frame diffs, chain diffs and the marshal read dpg)
    const bool hasDD = inWin && (p.flags & LKF_PKT_DD) && L.ddPkts;
    const DDPkt *const dpg = L.ddPkts + (hasDD ? pi : 0u);
    {
      const uint4 *src = reinterpret_cast<const uint4 *>(dpg);
      uint4 *dst = reinterpret_cast<uint4 *>(&dp);
#pragma unroll
      for (int k = 0; k < int(kDDPktScalar / 16); k++) dst[k] = hasDD ? src[k] : make_uint4(0, 0, 0, 0);
    }
    const bool ddLane = hasDD && (dp.flags & DP_VALID);  // (no descriptor: not selected, no DD state change)
    // a descriptor read with the structure in force and without custom fields
    // carries its template's lists: they are read from the structure in LDS
    const bool tmplSrc = LKF_DD_FASTBEST && u32(dp.slot) == u32(d.slot) && dp.custom == 0 &&
                         !(dp.flags & DP_ATTACHED) && dp.tmplIdx < s->numTmpl;
    const DDTmpl &tq = s->t[tmplSrc ? dp.tmplIdx : 0];
    auto chainDiff = [&](int c) -> u32 { return tmplSrc ? dd_tmpl_chain(tq, c) : dd_chain_diff(*dpg, c); };
    const u64 cl0 = d.cLast;
    const u64 efn = dp.extFN;
    const u64 ddM = __ballot(ddLane);
    const int pdl = prev_in(ddM, lt);
    const u64 pEfnL = sh64(efn, pdl >= 0 ? pdl : int(lane));
    const u64 pEfn = pdl >= 0 && u32(pdl) >= pos ? pEfnL : cl0;  // the previous descriptor's frame
    const u64 fi = efn - cl0;  // the frame's index in the run (0: frame cLast)
    if (ddLane) good = good && efn >= pEfn && fi < u64(kSvcFrames) - 8;  // frames in order (a reorder: full step)
    SVC_WHY(3);
    const bool newF = ddLane && efn != pEfn;
    const u32 dti = hiPos >= 0 ? dd::dti_at(dp.dtis, int(hiTarget)) : 0u;
    const bool t0 = hiPos >= 0 && dti != 0;  // the tentative decision (:160-190)
    if (ddLane) good = good && (maxTgt < 0 || int(dp.ndti) > maxTgt);  // (DecodeTarget.OnFrame errors: serial)
    SVC_WHY(4);
    // the frame's first descriptor lane in the run, and the next frame's
    const u64 newM = __ballot(inWin && newF);
    const u64 upto = newM & (lt | (1ull << lane));
    const u32 head = (fi == 0 || !upto) ? pos : u32(63 - __clzll(upto));
    const u64 after = newM & ~((2ull << lane) - 1);
    const u32 nextHead = after ? u32(__ffsll((long long)after) - 1) : 64u;
    const u64 frameM = (nextHead >= 64 ? ~0ull : ((1ull << nextHead) - 1)) & ~((1ull << head) - 1) & ddM;
    const int headL = frameM ? __ffsll((long long)frameM) - 1 : int(lane);
    const bool t0Head = sh32(u32(t0), headL) != 0;
    const u32 cache0 = dd::c_get(d, cl0);
    // GetDecision -> dropped returns before any state change (:86-95): every
    // packet after a frame's first dropped one, all of frame cLast's if it is
    // cached dropped.  The DTI is the frame's, so the frame's packets share the
    // head's decision (one that does not: full step).
    const bool drop0 = fi == 0 && cache0 == dd::SD_DROPPED;
    const bool early = ddLane && (drop0 || (!t0Head && int(lane) != headL));
    const bool eval = ddLane && !early;
    if (eval) good = good && t0 == t0Head;
    SVC_WHY(5);
    if (eval)
      good = good && !(dp.flags & DP_ATTACHED) && !(dp.extFlags & (LKF_DD_STRUCTURE_UPDATED | LKF_DD_ACTIVE_UPDATED)) &&
             dp.extKFN == d.extKeyFrameNum && int(dp.nchain) == int(d.numChains);
    SVC_WHY(6);
    ddFwdSel = eval && t0;
    if (ddFwdSel) good = good && !swAll && (d.flags & DS_FN_INIT);  // (a switch, the first frame number: full step)
    SVC_WHY(7);
    // frames the packet adds to the cache, and the decisions later frames see
    // Only the in-order prefix of the window can be decided: a lane past the
    // first out-of-order frame must not publish its frame's decision (a
    // reordered earlier frame would otherwise be looked up from the future)
    const u64 ordBadM = __ballot(ddLane && inWin && !(efn >= pEfn && fi < u64(kSvcFrames) - 8));
    const u32 ordEnd = ordBadM ? u32(__ffsll((long long)ordBadM) - 1) : 64u;
    const bool adds = inWin && lane < ordEnd && eval && (!t0 || (dp.extFlags & LKF_DD_INTEGRITY));
    // Frames an unbroken chain waits on (FrameChain.expectFrames): adding one
    // fires its callback, and so would marking it missing or aging it out of
    // the window; a lane whose add could do any of these takes the full step
    // (bounds: the missing marks of an add lie in [cLast - kNack, efn - kNack))
    // (the missing marks [cl0 - kNack, efn - kNack), the aged-out [cl0 - 256, efn - 256))
    for (int c = 0; c < int(d.numChains); c++) {
      if (((d.chBroken >> c) & 1) || !adds) continue;
      bool hit = dd::x_has(d, c, efn);
      if (efn > cl0) {
        const u64 k0 = cl0 >= dd::kNack ? cl0 - dd::kNack : 0, k1 = efn >= dd::kNack ? efn - dd::kNack : 0;
        const u64 a0 = cl0 >= dd::kEntries ? cl0 - dd::kEntries : 0, a1 = efn >= dd::kEntries ? efn - dd::kEntries : 0;
        hit = hit || dd::x_any_frames(d, c, k0, k1) || dd::x_any_frames(d, c, a0, a1);
      }
      if (hit) good = false;
    }
    SVC_WHY(14);
    const u64 addM = __ballot(adds);
    const bool firstAdd = adds && !(addM & frameM & lt);
    if (lane < u32(kSvcFrames)) sFD[lane] = u8(lane == 0 ? cache0 : dd::SD_UNKNOWN);
    if (lane + 64 < u32(kSvcFrames)) sFD[lane + 64] = u8(dd::SD_UNKNOWN);
    wave_lds_sync();
    if (firstAdd && fi < u64(kSvcFrames)) sFD[fi] = u8(t0 ? dd::SD_FORWARDED : dd::SD_DROPPED);  // (a lane past the run may be out of range)
    wave_lds_sync();
    auto dec = [&](u64 e) -> u32 {  // GetDecision(e) as this packet sees it (e < efn)
      if (e >= cl0 && e < efn) return sFD[e - cl0];
      bool old;
      return dd::c_decision(d, e, old);
    };
    // FrameChain.OnFrame (framechain.go:43-92) of every active chain, before
    // the selection: a restart (diff 0) clears the chain's broken bit and its
    // expected frames; an intact chain whose previous frame is not forwarded
    // breaks.  In a run: breaks of chains that do not protect the selected
    // target, and restarts of chains that protect no eligible target above it
    // and wait on no frame, leave every lane's selection as the run start has
    // it; they are recorded per lane (chBrk / chRst) and the chain's state
    // after the run is its last event's.  A lane sees a chain broken by an
    // earlier lane of the run as broken (the reference skips it) and so
    // records nothing it would not; restarts and breaks of the selected
    // target's chain, and frames still undecided (an expectation), take the
    // full step.
    if (eval && good)  // restarts
      for (int c = 0; c < int(d.numChains); c++) {
        if (!((d.chActive >> c) & 1) || int(dp.nchain) <= c || chainDiff(c) != 0) continue;
        if (((aboveM >> c) & 1) || dd::x_any(d, c) || (!LKF_SVC_CHAINS && ((d.chBroken >> c) & 1)))
          good = false;
        else if (LKF_SVC_CHAINS)
          chRst |= 1u << c;
      }
    u32 rstSeen = 0;  // chains an earlier lane of the window restarted (intact from there)
    for (int c = 0; c < int(d.numChains); c++)
      if (__ballot(inWin && ((chRst >> c) & 1)) & lt) rstSeen |= 1u << c;
    if (eval && good)  // breaks
      for (int c = 0; c < int(d.numChains); c++) {
        if (!((d.chActive >> c) & 1) || int(dp.nchain) <= c) continue;
        const u32 diff = chainDiff(c);
        if (diff == 0 || (((d.chBroken & ~rstSeen) >> c) & 1)) continue;  // (a restart; a chain broken before this lane)
        const u32 sd = dec(efn - diff);
        if (sd == dd::SD_FORWARDED) continue;
        if (sd == dd::SD_UNKNOWN || u32(c) == hiChain || !LKF_SVC_CHAINS)  // (expectFrames / the selection)
          good = false;
        else
          chBrk |= 1u << c;
      }
    SVC_WHY(8);
    if (ddFwdSel) good = good && (tmplSrc || dp.fdKind == FD_INLINE);  // (a custom pooled or spilled list: full step)
    if (ddFwdSel && good)  // a referenced frame that was dropped drops this one (:192-201): full step
      for (int j = 0; j < int(dp.nfd) && (tmplSrc || j < kDDFdInline); j++) {
        const u32 f = tmplSrc ? u32(s->fdPool[tq.fdOff + j]) : u32(dpg->fd[j]);
        if (f != 0 && dec(efn - f) == dd::SD_DROPPED) good = false;
      }
    SVC_WHY(9);
#if LKF_SVC_STATS
    tB = __builtin_amdgcn_s_memtime();
#endif
    if (ddFwdSel && good) {
      // frame number (FrameNumberWrapper without a structure update) and the
      // descriptor marshalled with the active mask in force (:223-262)
      const bool hasMask = d.flags & DS_HAS_MASK;
      const bool hasActive = (dp.flags & DP_ACTIVE) || hasMask;
      const u32 active = hasMask ? d.mask : dp.activeMask;
      ddLen = tmplSrc ? dd::dd_marshal_tmpl(*s, dp.tmplIdx, dp.flags, u16(efn + d.fnOffset), hasActive, active,
                                            sScr + lane * kSvcDDBytes, kSvcDDBytes)
                      : dd::dd_marshal_inl(*s, *dpg, u16(efn + d.fnOffset), hasActive, active,
                                           sScr + lane * kSvcDDBytes, kSvcDDBytes, nullptr, nullptr, false);
      if (ddLen < 0) good = false;
      mk = (p.hdr1 & 0x80) || ((dp.flags & DP_LAST) && L.h.curS == i32(dp.sid));
    }
    SVC_WHY(10);
#if LKF_SVC_STATS
    tC = __builtin_amdgcn_s_memtime();
#endif
    kind = ddFwdSel ? SK_FWD : (relevantDrop ? SK_MDROP : SK_NDROP);  // (RTPMarker false for the drops)
    ddEfn = efn;
    ddPut = firstAdd;
  }
  // ---- munger / sequencer (UpdateAndGetSnTs in order, sequencer.push)
  const bool adv = kind == SK_FWD || kind == SK_MDROP;
  if (kind == SK_FWD) good = good && started && (fl & F_SEQ_INIT) && (fl & F_STATS_INIT);  // (start: full step)
  SVC_WHY(1);
  const u64 advM = __ballot(inWin && adv);
  const int pa = prev_in(advM, lt);
  const u64 paEsn = sh64(p.esn, pa >= 0 ? pa : int(lane));
  const u64 prevEsn = pa >= 0 && u32(pa) >= pos ? paEsn : L.h.extHighestIncomingSN;
  const u64 dEsn = p.esn - prevEsn;
  const bool contig = dEsn == 1;
  const bool gap = dEsn > 1 && dEsn < u64(L.seqSize) - 64;
  if (adv) good = good && p.ssrc == L.h.lastSSRC && p.plen != 0 && (contig || gap);  // (reorder, dup, padding: full step)
  SVC_WHY(11);
  const bool excl = kind == SK_MDROP && contig;  // PacketDropped at the highest SN
  if (excl) good = good && L.h.snOffset == L.h.rmOpenValue && L.h.rmOpenStart <= p.esn;
  SVC_WHY(12);
  const u64 exM = __ballot(inWin && excl);
  const u64 fwdM = __ballot(inWin && kind == SK_FWD);
  const u64 snOff = L.h.snOffset + u64(__popcll(exM & lt));
  const u64 osn = p.esn - snOff;
  const u64 ots = p.ets - L.h.tsOffset;
  const int pf = prev_in(fwdM, lt);
  const int pfs = pf >= 0 ? pf : int(lane);
  const u64 pfOsn = sh64(osn, pfs), pfOts = sh64(ots, pfs);
  const u64 prevOsn = pf >= 0 && u32(pf) >= pos ? pfOsn : L.h.seqExtHighestSN;
  const u64 hiTS = pf >= 0 && u32(pf) >= pos ? pfOts : L.h.seqExtHighestTS;
  if (kind == SK_FWD)
    good = good && ots >= hiTS && osn - prevOsn >= 1 && osn - prevOsn < u64(L.seqSize) - 64 &&
           osn - L.h.seqExtHighestSN < u64(L.seqSize) - 64;
  SVC_WHY(13);
  const u64 stopM = __ballot(inWin ? !good : (valid && lane >= pos));
  const u32 x = stopM ? u32(__ffsll((long long)stopM) - 1) : n;
#if LKF_SVC_STATS
  {
    const u32 wx = x < 64 ? rl32(why, x) : 0u;
    if (lane == 0) {
      SVC_ADD(0, 1ull);
      SVC_ADD(1, (unsigned long long)(x > pos ? x - pos : 0));
      if (x < n) SVC_ADD(16 + (wx ? wx : 15), 1ull);
    }
  }
#endif
#if LKF_SVC_STATS
  const u64 tD = __builtin_amdgcn_s_memtime();
  if (lane == 0 && dd) {
    SVC_ADD(10, (unsigned long long)(tB - tA));
    SVC_ADD(11, (unsigned long long)(tC - tB));
    SVC_ADD(12, (unsigned long long)(tD - tC));
  }
#endif
  if (x <= pos) return pos;
  const u64 runM = (x >= 64 ? ~0ull : ((1ull << x) - 1)) & ~((1ull << pos) - 1);
  const bool inRun = (runM >> lane) & 1;
  if (DDK && dd) {
    // ---- frame chains: each chain ends in the state of its run's last event
    // (a break sets its bit, a restart clears it; restarts here wait on no
    // frame, so its expected frames stay empty)
    {
      DDState &d = *L.dd;
      for (int c = 0; c < int(d.numChains); c++) {
        const u64 bm = __ballot(inRun && ((chBrk >> c) & 1)), rm = __ballot(inRun && ((chRst >> c) & 1));
        if (!(bm | rm)) continue;
        const int lb = bm ? 63 - __clzll(bm) : -1, lr = rm ? 63 - __clzll(rm) : -1;
        if (lane == 0) d.chBroken = lb > lr ? (d.chBroken | (1u << c)) : (d.chBroken & ~(1u << c));
      }
      wave_lds_sync();
    }
    // ---- decision cache (selectordecisioncache.go:112-165) for the frames the
    // run added, in lane order: a new frame fills the entries it skipped with
    // unknown, marks the entries kNack behind the previous last frame missing
    // if still unknown (they lie before the run: read at the run-start state),
    // then takes its decision; a frame at or below the last one only sets it
    DDState &d = *L.dd;
    const u64 pM = __ballot(inRun && ddPut);
    const int pp = prev_in(pM, lt);
    const u64 ppE = sh64(ddEfn, pp >= 0 ? pp : int(lane));
    const u64 cur = pp >= 0 ? ppE : d.cLast;  // cLast when this lane adds
    const bool put = inRun && ddPut && ddEfn > d.cBase;
    const bool grow = put && ddEfn > cur;  // addEntity's new-entity path
    const u64 g1M = __ballot(grow && ddEfn == cur + 1);
    const u64 gNM = __ballot(grow && ddEfn > cur + 1);
    // one-frame steps: at most one missing mark each, in parallel
    u64 missE = 0;
    bool miss = false;
    if ((g1M >> lane) & 1) {
      const u64 ms = cur > dd::kNack + d.cBase ? cur - dd::kNack : d.cBase;
      const u64 me = ddEfn > dd::kNack + d.cBase ? ddEfn - dd::kNack : d.cBase;
      if (me > ms && dd::c_get(d, ms) == dd::SD_UNKNOWN) {
        miss = true;
        missE = ms;
      }
    }
    // gaps (lost frames): one lane at a time, the wave over the entries
    for (u64 m = gNM; m; m &= m - 1) {
      const u32 b = u32(__ffsll((long long)m) - 1);
      const u64 e = rl64(ddEfn, b), c0 = rl64(cur, b);
      const u64 ms = c0 > dd::kNack + d.cBase ? c0 - dd::kNack : d.cBase;
      const u64 me = e > dd::kNack + d.cBase ? e - dd::kNack : d.cBase;
      u32 st = dd::SD_UNKNOWN + 1;  // (none)
      u64 ent = 0;
      if (lane < u32(e - c0 - 1)) {  // [c0 + 1, e) -> unknown (no callbacks)
        ent = c0 + 1 + lane;
        st = dd::SD_UNKNOWN;
      }
      const u64 mk2 = (me > ms && lane < u32(me - ms)) ? ms + lane : 0;
      const bool mMiss = me > ms && lane < u32(me - ms) && dd::c_get(d, mk2) == dd::SD_UNKNOWN;
      wave_lds_sync();
      if (st == dd::SD_UNKNOWN) {
        const u64 off = (ent - d.cBase) % dd::kEntries;
        const u32 bp = u32(off & 31) * 2;
        atomicOr(reinterpret_cast<unsigned long long *>(&d.masks[off >> 5]), 3ull << bp);
      }
      if (mMiss) {
        const u64 off = (mk2 - d.cBase) % dd::kEntries;
        const u32 bp = u32(off & 31) * 2;
        unsigned long long *w = reinterpret_cast<unsigned long long *>(&d.masks[off >> 5]);
        atomicAnd(w, ~(3ull << bp));
        atomicOr(w, u64(dd::SD_MISSING) << bp);
      }
      wave_lds_sync();
    }
    wave_lds_sync();
    if (miss) {
      const u64 off = (missE - d.cBase) % dd::kEntries;
      const u32 bp = u32(off & 31) * 2;
      unsigned long long *w = reinterpret_cast<unsigned long long *>(&d.masks[off >> 5]);
      atomicAnd(w, ~(3ull << bp));
      atomicOr(w, u64(dd::SD_MISSING) << bp);
    }
    if (put) {
      const u64 off = (ddEfn - d.cBase) % dd::kEntries;
      const u32 bp = u32(off & 31) * 2;
      unsigned long long *w = reinterpret_cast<unsigned long long *>(&d.masks[off >> 5]);
      atomicAnd(w, ~(3ull << bp));
      atomicOr(w, u64(kind == SK_FWD ? dd::SD_FORWARDED : dd::SD_DROPPED) << bp);
    }
    wave_lds_sync();
    const u64 aM = __ballot(put);
    const u64 eLast = aM ? rl64(ddEfn, 63 - __clzll(aM)) : 0;  // frames are in order: the last added is the highest
    const u64 fM = __ballot(inRun && ddFwdSel);
    const u64 eF = fM ? rl64(ddEfn, 63 - __clzll(fM)) : 0;
    wave_lds_sync();
    if (aM && eLast > d.cLast) d.cLast = eLast;
    if (fM && eF > d.fnLast) d.fnLast = eF;  // FrameNumberWrapper.UpdateAndGet of the selected frames
    wave_lds_sync();
  }
  // ---- decide lanes [pos, x)
  const u64 fwR = fwdM & runM, exR = exM & runM;
  const u64 advR = advM & runM;
  const u64 setR = advR & ~exR;  // lanes that set the munger's last SN/TS (forwards, drops after a gap)
  const bool f = inRun && kind == SK_FWD;
  o.nTuples += x - pos;
  {
    const bool nd = inRun && kind == SK_NDROP;
    o.drops[LKF_DROP_NOT_SELECTED] += u32(__popcll(__ballot(inRun && kind == SK_MDROP))) +
                                      u32(__popcll(__ballot(nd && nsr == LKF_DROP_NOT_SELECTED)));
    o.drops[LKF_DROP_DOWNGRADE] += u32(__popcll(__ballot(nd && nsr == LKF_DROP_DOWNGRADE)));
  }
  // output shape (downtrack.go:693-723, pacer/base.go:71-100): DD element first
  const int cc = p.hdr0 & 0xf;
  const bool playout = L.extPlayout && !(fl & F_PLAYOUT_ACKED);
  const bool ddOn = DDK && f && ddLen > 0 && L.extDD;
  const int eh = (ddOn && ddLen > 16) ? 2 : 1;
  const int extBytes =
      (ddOn ? eh + ddLen : 0) + (playout ? eh + 3 : 0) + (L.extAbs ? eh + 3 : 0) + (L.extTcc ? eh + 2 : 0);
  const int extBlock = extBytes ? 4 + ((extBytes + 3) & ~3) : 0;
  const int hdrLen = 12 + 4 * cc + extBlock;
  const u32 outLen = f ? u32(hdrLen + int(p.plen)) : 0u;
  const u32 aligned = (outLen + 15) & ~15u;
  const u32 relEx = excl_scan_u32(aligned, lane);
  bool ddKeep = ddOn;
  u32 ddOff = 0;
  if (DDK && dd) {  // the run's marshalled descriptors: one bump of the batch's DD arena
    const u32 dl = ddOn ? u32(ddLen) : 0u;
    const u32 dEx = excl_scan_u32(dl, lane);
    const u32 dTot = rl32(dEx + dl, 63);
    if (dTot) {
      u64 base = 0;
      if (lane == 0) base = atomicAdd(reinterpret_cast<unsigned long long *>(o.ddUsed), (unsigned long long)dTot);
      base = rl64(base, 0);
      if (base + dTot > o.ddCap) {
        if (lane == 0) atomicOr(L.err, 64u);  // (the DD arena)
        ddKeep = false;
      } else if (ddOn) {
        // (a fixed-trip copy: a loop bounded by the per-lane length made the
        // register allocator give this instantiation 225 VGPRs)
        u8 *dst = o.ddArena + base + dEx;
        const u32 *srcw = reinterpret_cast<const u32 *>(sScr + lane * kSvcDDBytes);
#pragma unroll
        for (int w = 0; w < kSvcDDBytes / 4; w++) {
          const u32 v = srcw[w];
#pragma unroll
          for (int b = 0; b < 4; b++)
            if (4 * w + b < ddLen) dst[4 * w + b] = u8(v >> (8 * b));
        }
        ddOff = u32(base + dEx);
      }
    }
  }
  const bool kf = p.flags & LKF_PKT_KEYFRAME;
  const u32 j = u32(__popcll(fwR & lt));
  fwd_base(o, fwR, osn, ots);
  if (f) {
#if LKF_CHECKED
    CHK(o.tupBase + o.nFwd + j < o.tupCap, CK_DEC_TUPLE, o.tupBase + o.nFwd + j, o.tupCap);
#endif
    store_fwd(o.outT + o.nFwd + j, o.outW + o.nFwd + j, o.bSN, o.bTS, osn, ots, pi, o.relOff + relEx, outLen,
              (kf ? LKF_OUT_KEYFRAME : 0) | (mk ? LKF_OUT_MARKER : 0) | (playout ? T_PLAYOUT : 0) | (ddKeep ? T_DD : 0),
              ddKeep ? u32(ddLen) : 0u, ddKeep ? ddOff : 0u);
    u32 slot = u32(L.h.seqHighSlot) + u32(osn - L.h.seqExtHighestSN);  // sequencer.push, in order
    while (slot >= L.seqSize) slot -= L.seqSize;
    SeqMeta m = {};
    m.sourceSeqNo = u16(p.esn);
    m.targetSeqNo = u16(osn);
    m.timestamp = u32(ots);
    m.lastNack = u32(p.arr / 1000000LL - L.h.seqStartMs);
    m.marker = mk;
    m.layer = p.layer;
    m.codecLen = 0;
    CHK(slot < L.seqSize, CK_DEC_SEQ, slot, L.seqSize);
    store_rec(L.seq + slot, m);
  }
  // sequencer slots a push skipped (sequencer.go:179-189): invalidated
  for (u64 gm = __ballot(f && osn - prevOsn > 1); gm; gm &= gm - 1) {
    const u32 b = u32(__ffsll((long long)gm) - 1);
    const u64 from = rl64(prevOsn, b), to = rl64(osn, b);
    const u32 nsk = u32(to - from - 1);
    const u32 base = u32(L.h.seqHighSlot) + u32(from - L.h.seqExtHighestSN) + 1;
    for (u32 i = lane; i < nsk; i += 64) {
      u32 x2 = base + i;
      while (x2 >= L.seqSize) x2 -= L.seqSize;
      store_rec(L.seq + x2, SeqMeta{});
    }
  }
  if (f) ss_put(o.ssBuf + o.ssN + j, osn, ots, p.arr, p.poff, p.plen, mk, kf);
  o.ssN += u32(__popcll(fwR));
  const u32 sumLen = wave_sum_u32(outLen);
  sentAcc += f ? i32(p.poff) - hdrLen : 0;
  if (fwR) {
    o.nBytes += sumLen;
    o.nFwd += u32(__popcll(fwR));
    const u32 lastF = 63 - __clzll(fwR);
    u32 slot = u32(L.h.seqHighSlot) + u32(rl64(osn, lastF) - L.h.seqExtHighestSN);
    while (slot >= L.seqSize) slot -= L.seqSize;
    L.h.seqHighSlot = u16(slot);
    L.h.seqExtHighestSN = rl64(osn, lastF);
    L.h.seqExtHighestTS = rl64(ots, lastF);
    o.relOff += rl32(relEx + aligned, lastF);
  }
  if (advR) {  // ---- the munger past the run
    const u64 mkM = __ballot(mk);
    const u32 lastA = 63 - __clzll(advR);
    L.h.extHighestIncomingSN = rl64(p.esn, lastA);
    const bool lastSets = (setR >> lastA) & 1;
    const u64 psM = setR & ((1ull << lastA) - 1);
    u64 sSN = L.h.extLastSN, sTS = L.h.extLastTS;
    bool sMk = fl & F_LAST_MARKER;
    if (psM) {
      const u32 b = 63 - __clzll(psM);
      sSN = rl64(osn, b);
      sTS = rl64(ots, b);
      sMk = (mkM >> b) & 1;
    }
    if (lastSets) {
      L.h.extSecondLastSN = sSN;
      L.h.extSecondLastTS = sTS;
      L.h.extLastSN = rl64(osn, lastA);
      L.h.extLastTS = rl64(ots, lastA);
      setf(L, F_SECOND_LAST_MARKER, sMk);
      setf(L, F_LAST_MARKER, (mkM >> lastA) & 1);
    } else {
      L.h.extSecondLastSN = L.h.extLastSN = sSN;
      L.h.extSecondLastTS = L.h.extLastTS = sTS;
      setf(L, F_SECOND_LAST_MARKER, sMk);
      setf(L, F_LAST_MARKER, sMk);
    }
    // RTX gate (rtpmunger.go:204-208): the last key frame sets it, the
    // 2000-packet expiry is checked against the run's highest munged SN
    const u64 kfM = __ballot(((advR >> lane) & 1) && kf);
    if (kfM) {
      L.h.extRtxGateSn = rl64(osn, 63 - __clzll(kfM));
      setf(L, F_RTX_GATE, true);
    }
    if (hasf(L, F_RTX_GATE) && (rl64(osn, lastA) - L.h.extRtxGateSn) > 2000) setf(L, F_RTX_GATE, false);
    // exclusions: one per group of drops with consecutive SNs
    u64 m = exR;
    while (m) {
      const u32 b = u32(__ffsll((long long)m) - 1);
      const u64 s0 = rl64(p.esn, b);
      u64 e0 = s0 + 1;
      m &= m - 1;
      while (m) {
        const u32 b2 = u32(__ffsll((long long)m) - 1);
        if (rl64(p.esn, b2) != e0) break;
        e0++;
        m &= m - 1;
      }
      rm_exclude(L, s0, e0);
    }
    if (exR) L.h.snOffset = L.h.rmOpenValue;
  }
  return x;
}
#undef SVC_WHY

#ifndef LKF_DD_RESTAGE
#define LKF_DD_RESTAGE 1
#endif
// The structure in force staged in LDS: its decode targets, chains and
// templates are read on every descriptor (selection, marshalling).  The ring
// entries are fixed while the batch decides (k_dd_decode filled them); a
// descriptor that attaches a new structure moves the DownTrack to another
// slot, which is then staged in turn (dd_restage).
__device__ __forceinline__ void dd_stage_struct(Lane &L, const DDState *sDD, u8 *sDDSRaw, u32 lane) {
  const u32 slot = __builtin_amdgcn_readfirstlane(u32(sDD->slot));
  const uint4 *gs = reinterpret_cast<const uint4 *>(L.ddRing + slot);
  uint4 *ls = reinterpret_cast<uint4 *>(sDDSRaw);
  // the header and the templates in use, then the used part of the pool
  const u32 nT = __builtin_amdgcn_readfirstlane(u32(L.ddRing[slot].numTmpl));
  const u32 nP = __builtin_amdgcn_readfirstlane(u32(L.ddRing[slot].nfdPool));
  constexpr u32 kTOff = __builtin_offsetof(DDStruct, t) / 16, kPOff = __builtin_offsetof(DDStruct, fdPool) / 16;
  const u32 nHead = kTOff + nT * (sizeof(DDTmpl) / 16), nPool = (nP + 15) / 16;
  for (u32 i = lane; i < nHead + nPool; i += 64) {
    const u32 k = i < nHead ? i : kPOff + (i - nHead);
    ls[k] = gs[k];
  }
  L.ddSSlot = slot;
  __syncthreads();
}
__device__ __forceinline__ void dd_restage(Lane &L, const DDState *sDD, u8 *sDDSRaw, u32 lane) {
  wave_lds_sync();
  const bool moved = __builtin_amdgcn_readfirstlane(int((sDD->flags & DS_KF_VALID) && u32(sDD->slot) != L.ddSSlot));
  if (LKF_DD_RESTAGE && moved) dd_stage_struct(L, sDD, sDDSRaw, lane);
}

constexpr u32 kDecideMaxK = 8;  // schedule slots per decide wave (LKF_DECIDE_K is clamped to it; 8 and 16 measured slower than 4)
#ifndef LKF_DEC_PREFETCH  // a single-chunk track's packets loaded with the DownTrack's state
#define LKF_DEC_PREFETCH 0  // (measured: the headline 1.3 % slower with it, the tick flat; r5 A/B)
#endif
template <bool DDK>
__global__ void __launch_bounds__(64) DECIDE_ATTR k_decide_dt(DecideArgs A, const lkf_pkt *__restrict__ pkts) {
  __shared__ i32 sDrop[kSetCap];
  __shared__ i32 sEx[kSetCap];
  __shared__ i32 sMissKey[kMissCap];
  __shared__ i32 sMissVal[kMissCap];
  __shared__ RangeEntry sRm[kRangeCap];
  // (the plain instantiation keeps a 16-B stub: LDS is allocated per instantiation)
  __shared__ __attribute__((aligned(16))) u8 sDDRaw[DDK ? sizeof(DDState) + kDDMaxBytes + 1 : 16];
  __shared__ __attribute__((aligned(16))) u8 sSvcScr[DDK ? 64 * kSvcDDBytes : 16];  // svc_run: per-lane marshalled descriptors
  // the structure in force (the staged part: not its serialization)
  __shared__ __attribute__((aligned(16))) u8 sDDSRaw[DDK ? __builtin_offsetof(DDStruct, serBits) : 16];
  __shared__ u8 sSvcFD[kSvcFrames];                    // svc_run: decisions of the run's frames
  DDState *const sDD = reinterpret_cast<DDState *>(sDDRaw);
  u8 *const sDDBuf = sDDRaw + (DDK ? sizeof(DDState) : 0);
  // A wave serves perWave schedule slots of its XCD's list (slot index = q * 8
  // + XCD, q consecutive), one DownTrack after the other.  Short ticks have a
  // few packets per DownTrack, and one workgroup per DownTrack would leave the
  // kernel bound by the workgroup dispatch rate (≈30 waves/µs per XCD).
  // Round 1: lane j fetches slot j's DownTrack, track and control-op range and
  // then the track's packet range, so the whole wave's list costs two
  // dependent loads.  A DownTrack with neither packets nor control ops in the
  // batch is skipped: its state does not change and k_batch_init zeroed its
  // counters.
  // The list is kept in LDS (not registers) across the DownTrack loop.
  __shared__ uint4 sSlot[2 * kDecideMaxK];
  u64 todo;
  {
    const u32 K = A.perWave, lane = threadIdx.x;
    const u32 wj = A.waveBase + ((blockIdx.x >> 3) * K + lane) * 8 + (blockIdx.x & 7);
    u32 dj = 0xffffffffu, tj = 0, ej = 0, eej = 0, pbj = 0, pej = 0, cj = 0;
    if (lane < K && wj < A.waveEnd) {
      dj = A.sched[wj];
      tj = A.waveTrack[wj];
      ej = A.evOff[wj];
      eej = A.evOff[wj + 1];
    }
    if (dj != 0xffffffffu) {  // (0xffffffff: padding slot of the per-XCD schedule)
      pbj = A.tBegin[tj];
      pej = A.tEnd[tj];
      cj = A.tracks[tj].codec;  // (the VP8 maps are then loaded with the hot state)
    }
    todo = __ballot(dj != 0xffffffffu && (pbj < pej || ej < eej));
    if (lane < K) {
      sSlot[2 * lane] = make_uint4(wj, dj, tj, ej);
      sSlot[2 * lane + 1] = make_uint4(eej, pbj, pej, cj);
    }
    wave_lds_sync();
  }
  while (todo) {
  const u32 jw = u32(__ffsll(static_cast<long long>(todo))) - 1;
  todo &= todo - 1;
#if LKF_SVC_STATS
  // per-phase cycles of the SVC DownTracks (g_svc[4..9]: prologue, runs,
  // full steps after runs, chunk tails, epilogue, DownTracks)
  const u64 tP0 = __builtin_amdgcn_s_memtime();
  u64 tRun = 0, tStep = 0, tLoad = 0, tSs = 0;
#endif
  // The lane index again, opaque to the compiler, so lane-derived values are
  // recomputed per DownTrack rather than hoisted out of the loop and held in
  // registers across the whole body.
  u32 laneR;
  asm volatile("v_mov_b32 %0, %1" : "=v"(laneR) : "v"(threadIdx.x));
  const u32 lane = laneR;
  const u64 lt = (1ull << lane) - 1;
  // Round 2: everything keyed by the DownTrack, including the VP8 munger maps
  // (read whole, whatever their fill, so the copy does not wait for the hot
  // state).
  const uint4 sa = sSlot[2 * jw], sb = sSlot[2 * jw + 1];
  const u32 w = __builtin_amdgcn_readfirstlane(sa.x);
  const u32 d = __builtin_amdgcn_readfirstlane(sa.y);
  const u32 track = __builtin_amdgcn_readfirstlane(sa.z);
  u32 ev = __builtin_amdgcn_readfirstlane(sa.w);
  const u32 evEnd = __builtin_amdgcn_readfirstlane(sb.x);
  CHK(d < A.maxDts, CK_DEC_DT, d, A.maxDts);
  CHK(track < A.maxTracks, CK_DEC_TRACK, track, A.maxTracks);
  CHK(evEnd <= A.nev, CK_DEC_EVENT, evEnd, A.nev);
  const DevDT dt = A.dts[d];
  const u32 pb = __builtin_amdgcn_readfirstlane(sb.y);
  u32 pe = __builtin_amdgcn_readfirstlane(sb.z);
  const u64 slot0 = A.slotBase[d];
  // A track with at most 64 packets in the batch is one chunk: its packets
  // are loaded together with the DownTrack's state (one round trip fewer)
  bool pre = LKF_DEC_PREFETCH && pe - pb <= 64u;  // (cleared once the chunk takes them)
  uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0, r2 = r0, r3 = r0;
  if (pre && lane < pe - pb) {
    CHK(pb + lane < A.npkts, CK_DEC_PKT, pb + lane, A.npkts);
    const uint4 *ps = reinterpret_cast<const uint4 *>(pkts) + u64(pb + lane) * 4;
    r0 = ps[0];
    r1 = ps[1];
    r2 = ps[2];
    r3 = ps[3];
  }
  LaneOut o;
  o.nFwd = o.nBytes = o.nTuples = 0;
  o.sentDiff = 0;
  i32 sentAcc = 0;  // per lane: run-path forwarded packets' incoming minus outgoing header bytes
  o.relOff = 0;
  o.bSN = o.bTS = 0;
  for (int i = 0; i < LKF_DROP_NREASONS; i++) o.drops[i] = 0;
  __shared__ __attribute__((aligned(16))) DTHot sHot;
  __shared__ __attribute__((aligned(16))) SenderStats sSS;  // the DownTrack's RTPStatsSender (ss_flush)
  __shared__ u32 sHot0[64];  // the state as loaded: only the dwords the batch changes go back
  Lane L{sHot};
  {
    const u32 h0 = reinterpret_cast<const u32 *>(A.hot + d)[lane];  // 64 dwords
    reinterpret_cast<u32 *>(&sHot)[lane] = h0;
    sHot0[lane] = h0;
  }
  if (lane < sizeof(SenderStats) / 16)
    reinterpret_cast<uint4 *>(&sSS)[lane] = reinterpret_cast<const uint4 *>(A.ss + d)[lane];
  // VP8 munger maps live in LDS for the batch: the picture-id sets here, the
  // live entries of the missing-picture ring once the hot state is in
  const bool vp8Track = __builtin_amdgcn_readfirstlane(sb.w) == LKF_CODEC_VP8;
  if (vp8Track && lane < u32(kSetCap)) {
    sDrop[lane] = A.vc[d].dropKey[lane];
    sEx[lane] = A.vc[d].exKey[lane];
  }
  __shared__ __attribute__((aligned(16))) SsEnt sSsBuf[64];  // one chunk's forwarded tuples (ss_flush)
  o.ss = &sSS;
  o.ssBuf = sSsBuf;
  o.ssN = 0;
  o.ssRing = A.ssRing + size_t(d) * kSnInfoSize;
  o.ssGap = A.ssGap + size_t(d) * kGapWords;
  __syncthreads();
#if LKF_SVC_STATS
  const u64 tPa = __builtin_amdgcn_s_memtime();
#endif
  RangeEntry *const rmG = A.rm + size_t(d) * kRangeCap;
  L.rm = sRm;
  L.rmG = rmG;
  L.rmNew = 0;
  L.rmLoaded = false;
  L.vcDirty = false;
  L.vc = A.vc + d;
  L.dropKey = sDrop;
  L.exKey = sEx;
  L.missKey = sMissKey;
  L.missVal = sMissVal;
  if (vp8Track) {
    for (u32 i = lane; i < L.h.missCount; i += 64) {  // the live entries of the missing-picture ring
      const u32 idx = (L.h.missHead + i) % kMissCap;
      sMissKey[idx] = L.vc->missKey[idx];
      sMissVal[idx] = L.vc->missVal[idx];
    }
  }
  if (slot0 + (pe - pb) > A.tupleCap) {  // tuple slots exhausted: skip, flag
    if (lane == 0) atomicOr(A.err, 8u);
    pe = pb;
  }
  __syncthreads();
  L.seq = A.seq + size_t(d) * A.seqSize;
  L.seqSize = A.seqSize;
  L.srm = DDK ? reinterpret_cast<SeqRM *>(A.srm + size_t(d) * A.srmStride) : nullptr;  // (only <true> reads it)
  L.srmCap = A.srmCap;
  const DevTrack &tk = A.tracks[track];
  L.kind = tk.kind;
  L.codec = tk.codec;
  L.hasRefTS = tk.hasRefTS;
  L.clockRate = tk.clockRate;
  L.offs = A.dtOffs + size_t(d) * kDTOffsWords;
  L.extPlayout = dt.extPlayout;
  L.extAbs = dt.extAbs;
  L.extDD = dt.extDD;
  L.extTcc = dt.extTcc;
  L.err = A.err;
  L.ddPkts = A.ddPkts;
  __shared__ __attribute__((aligned(16))) DDPkt sDDPkt;
  L.ddPktL = &sDDPkt;
  L.ddSpill = A.ddSpill;
  L.ddRing = nullptr;
  L.ddS = reinterpret_cast<DDStruct *>(sDDSRaw);
  L.ddSSlot = 0xffffffffu;
  L.dd = sDD;
  L.ddBuf = sDDBuf;
  o.ddArena = A.ddArena;
  o.ddUsed = A.ddUsed;
  o.ddCap = A.ddCap;
#if LKF_CHECKED
  o.tupBase = slot0;
  o.tupCap = A.tupleCap;
  CHK(pe <= A.npkts, CK_DEC_PKT, pe, A.npkts);
#endif
  const bool ddDT = DDK && (L.h.flags & F_DD) && A.ddState;
  if (ddDT) {  // the DD selector state lives in LDS for the batch
    L.ddRing = A.ddStructs + size_t(tk.ddIdx) * kDDSlots;
    const uint4 *g = reinterpret_cast<const uint4 *>(A.ddState + d);
    uint4 *l = reinterpret_cast<uint4 *>(sDD);
    // the head and the expectFrames rows of the chains in use (a structure
    // update zeroes every row's count, so rows past them are never read first)
    const u32 nc0 = __builtin_amdgcn_readfirstlane(u32(A.ddState[d].numChains));
    const u32 nDD = (kDDStateHead + nc0 * kDDExpRow * 8) / 16;
    for (u32 i = lane; i < nDD; i += 64) l[i] = g[i];
    __syncthreads();
    if (sDD->flags & DS_KF_VALID) dd_stage_struct(L, sDD, sDDSRaw, lane);
  }
  o.outT = A.recs + slot0;
  o.outW = A.wide + slot0;
  // SVC DownTracks (one SSRC, every packet relevant to the selector): svc_run
  // (the host schedules them in k_decide_dt<true>)
  const bool svcDT = DDK && (L.h.flags & F_VIDEO) && !(L.h.flags & F_SIMULCAST) &&
                     ((L.h.flags & F_VP9) || ((L.h.flags & F_DD) && ddDT));
  u32 nextAt = ev < evEnd ? A.events[ev].at : 0xffffffffu;
  const uint4 *src = reinterpret_cast<const uint4 *>(pkts);

  u32 kpos = pb;  // first packet of the track not yet decided
#if LKF_SVC_STATS
  const u64 tP1 = __builtin_amdgcn_s_memtime();
#endif
  while (kpos < pe) {
#if LKF_SVC_STATS
    const u64 tc0 = __builtin_amdgcn_s_memtime();
#endif
    if (nextAt <= kpos) {
      while (nextAt <= kpos) {
        apply_ctl(L, A.events[ev++]);
        nextAt = ev < evEnd ? A.events[ev].at : 0xffffffffu;
      }
      vm_drain();
    }
    // Steady state: a simulcast DownTrack on its target layer with no switch
    // possible drops every packet of another layer as NOT_SELECTED with no
    // state change (simulcast.go:42-122: curS == tgtS <= maxS, forwarder.go
    // :1440/:1687 not taken).  Its chunk is then the next 64 packets of its
    // own layer (per-track layer lists); the skipped packets are counted.
    // (A track with at most 64 packets in the batch is one chunk either way:
    // read it directly instead of through the layer list, two dependent
    // loads fewer for the short ticks.)
    const bool steady = pe - pb > 64 && steady_state(L);
    u32 pi, n, lim;  // lane -> packet index; packets in the chunk; packet index after it
    if (steady) {
      const u32 ls = u32(L.h.curS);
      CHK(size_t(ls) * A.pktStride + kpos < 3 * size_t(A.pktStride), CK_DEC_LAYER, size_t(ls) * A.pktStride + kpos,
          3 * size_t(A.pktStride));
      const u32 j = A.layerBefore[size_t(ls) * A.pktStride + kpos] + lane;
      pi = j < A.layerCnt[track * 3 + ls] ? A.layerList[size_t(ls) * A.pktStride + pb + j] : 0xffffffffu;
      const u32 stopAt = min(nextAt, pe);
      n = u32(__popcll(__ballot(pi < stopAt)));  // list is increasing: a prefix of the lanes
      lim = n == 64 ? rl32(pi, 63) + 1 : stopAt;
    } else {
      n = min(64u, pe - kpos);
      pi = kpos + lane;
      lim = kpos + n;
    }
    const bool valid = lane < n;
    if (!pre) {  // (pre: the prefetched chunk, pi = pb + lane)
      r0 = r1 = r2 = r3 = make_uint4(0, 0, 0, 0);
      if (valid) {
        CHK(pi < A.npkts, CK_DEC_PKT, pi, A.npkts);
        const u64 q = u64(pi) * 4;
        r0 = src[q];
        r1 = src[q + 1];
        r2 = src[q + 2];
        r3 = src[q + 3];
      }
    }
    pre = false;
    pin_loaded(r0, r1, r2, r3);
#if LKF_SVC_STATS
    {
      u64 tl0;  // (the loads' wait: the chunk's first use of the registers)
      const u32 dep = __builtin_amdgcn_readfirstlane(r0.x ^ r3.w);  // (waits for the loads)
      asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(tl0) : "s"(dep));
      tLoad += tl0 - tc0;
    }
#endif
    const PktV p = decode_pkt(r0, r1, r2, r3);
    u32 pos = 0;
    u32 own = n;  // packets of the chunk decided (steady: the rest of the range is skipped drops)
    while (pos < n) {
      if (nextAt <= rl32(pi, pos)) {
        while (nextAt <= rl32(pi, pos)) {
          apply_ctl(L, A.events[ev++]);
          nextAt = ev < evEnd ? A.events[ev].at : 0xffffffffu;
        }
        vm_drain();
      }
      u32 x;
      bool gapStop = false;  // the stopping lane starts the next run (no full step)
      if (DDK && svcDT) {
        // SVC DownTrack: a run, then the stopping packet's full step (its
        // descriptor reloaded wave-uniform, so the chunk's raw registers are
        // dead on this path)
#if LKF_SVC_STATS
        const u64 tr0 = __builtin_amdgcn_s_memtime();
#endif
        x = svc_run<DDK>(L, o, p, pi, n, pos, nextAt, valid, sentAcc, sSvcScr, sSvcFD);
        pos = x;
#if LKF_SVC_STATS
        const u64 tr1 = __builtin_amdgcn_s_memtime();
        tRun += tr1 - tr0;
#endif
        if (x < n && rl32(pi, x) < nextAt) {
          const u32 px = rl32(pi, x);
          decide_step<DDK>(L, load_pkt(pkts + px), px, o);
          vm_drain();
          if (ddDT) dd_restage(L, sDD, sDDSRaw, lane);
#if LKF_SVC_STATS
          tStep += __builtin_amdgcn_s_memtime() - tr1;
#endif
#if LKF_SVC_STATS
          if (lane == 0) SVC_ADD(2, 1ull);
#endif
          pos = x + 1;
        }
        continue;
      } else {
      const bool inWin = valid && lane >= pos && pi < nextAt;
      // ---- classification against the state at the start of the run
      const u32 fl = L.h.flags;
      const bool video = fl & F_VIDEO;
      const i32 layer = p.layer;
      const bool kf = p.flags & LKF_PKT_KEYFRAME;
      const bool pktMarker = p.hdr1 & 0x80;
      int cls;  // >= 0: drop with no state change; -1: current-layer candidate; -2: serial
      if (fl & (F_MUTED | F_PUBMUTED)) {
        cls = LKF_DROP_MUTED;
      } else if (!video) {
        cls = -1;  // (a keyframe's RTX-gate move is applied with the run's state advance)
      } else if (L.h.tgtS == INVALID || L.h.tgtT == INVALID) {
        cls = LKF_DROP_PAUSED;
      } else if (!(fl & F_SIMULCAST)) {
        cls = (fl & (F_VP9 | F_DD)) ? -2 : LKF_DROP_NOT_SELECTED;  // SVC: full step
      } else {
        const bool willSwitch =
            kf && ((L.h.curS != L.h.tgtS && ((layer > L.h.curS && layer <= L.h.tgtS) ||
                                             (layer < L.h.curS && layer >= L.h.tgtS))) ||
                   (L.h.curS > L.h.maxS && layer <= L.h.maxS));
        if (willSwitch)
          cls = -2;
        else if (layer != L.h.curS)
          cls = LKF_DROP_NOT_SELECTED;
        else if ((fl & F_DEFICIENT) && L.h.tgtS < L.h.curS)
          cls = LKF_DROP_DOWNGRADE;
        else if ((fl & F_VP8) && (fl & F_TLS_VP8) && (p.flags & LKF_PKT_VP8))
          cls = -1;
        else
          cls = -2;
      }
      const bool cand = inWin && cls == -1;
      const bool candIn = cand;  // (an out-of-order candidate is not ok: the full step)
      const u64 candM = __ballot(candIn);
      const int pc = prev_in(candM, lt);
      const int pcs = pc >= 0 ? pc : int(lane);  // cross-lane reads run on every lane
      const u64 pcEsn = sh64(p.esn, pcs);
      const u64 prevEsn = pc >= 0 ? pcEsn : L.h.extHighestIncomingSN;
      // A loss gap (diff > 1, rtpmunger.go:186-190) is taken in the run when it
      // is the run's first candidate: its side effects (missing/exempted
      // pictures vp8.go:218-255, skipped sequencer slots sequencer.go:179-189)
      // are applied before the run, from the state at the run start.
      const u64 dEsn = p.esn - prevEsn;
      const bool gapLane = candIn && dEsn > 1 && dEsn < u64(L.seqSize) - 64 &&
                           p.plen != 0 && p.ssrc == L.h.lastSSRC;
      bool ok = candIn && (dEsn == 1 || gapLane) && p.plen != 0 && p.ssrc == L.h.lastSSRC;
      // a gap behind other candidates ends this run and starts the next one
      const bool gapLater = candIn && pc >= 0 && dEsn > 1 && dEsn < u64(L.seqSize) - 64 && p.plen != 0 &&
                            p.ssrc == L.h.lastSSRC;
      // (diag: run-body split below)
      // VP8 picture id (VP8PictureIdWrapHandler.Unwrap vp8.go:400-483 without a wrap)
      const bool M = p.vbits & LKF_VP8_M, I = p.vbits & LKF_VP8_I, T = p.vbits & LKF_VP8_T;
      const i32 np = M ? i32(p.pid & 0x7fff) : i32(p.pid & 0x7f);
      const i32 ext = np + L.h.wrTotalWrap;
      const i32 pcExt = i32(sh32(u32(ext), pcs));
      const bool pcM = sh32(u32(M), pcs) != 0;
      const i32 prevExt = pc >= 0 ? pcExt : L.h.wrMaxPictureId;
      const bool prevM = pc >= 0 ? pcM : ((fl & F_WR_MAX_MBIT) != 0);
      bool dropT = false;
      u64 tswM = 0;  // candidate lanes at a temporal switch point (the first ends the run)
      bool overT = false;
      if (video) {
        i32 mp = prevExt;
        if (mp > 0) mp = prevM ? (prevExt & 0x7fff) : (prevExt & 0x7f);
        const bool wrapBack = L.h.wrTotalWrap > 0 && (prevExt + (L.h.wrLastWrap >> 1)) < (np + L.h.wrTotalWrap);
        const bool wraps = np < mp && (mp - np) > (prevM ? (1 << 14) : (1 << 6));
        // SelectTemporal would switch here (base.go:143-168, temporallayerselector/vp8.go:32-56)
        const i32 cT = L.h.curT, gT = L.h.tgtT;
        const bool tsw = cT != gT && T &&
                         (cT < gT ? (i32(p.tid) > cT && i32(p.tid) <= gT && (p.vbits & LKF_VP8_S) &&
                                     (p.vbits & LKF_VP8_Y))
                                  : pktMarker);
        overT = candIn && T && p.tid > u8(cT);
        // a gap lane forwards whatever its layer and exempts its picture
        // (vp8.go:249-255): later lanes of that picture forward too
        bool exIn = false;
        for (u64 ge = __ballot(gapLane && overT); ge; ge &= ge - 1) {
          const u32 k = u32(__ffsll((long long)ge) - 1);
          exIn = exIn || (lane > k && ext == i32(rl32(u32(ext), k)));
        }
        dropT = overT && !gapLane && !exIn;
        if (__ballot(dropT) && L.h.exCount)  // exempted pictures forward (vp8.go:270)
          dropT = dropT && !set_has(L.exKey, L.h.exHead, L.h.exCount, ext);
        // A temporal switch point is decided in the run and ends it: up, the
        // packet's own TID is the filter limit (thisL = tid, so it forwards);
        // down (at a marker), thisL is still the current layer and the packet
        // must forward — a filtered one would roll the selector back (serial).
        if (tsw && cT < gT) dropT = false;
        const bool tswOk = tsw && !gapLane && !dropT;
        ok = ok && !wrapBack && !wraps && (!tsw || tswOk) && (!dropT || L.h.snOffset == L.h.rmOpenValue);
        tswM = __ballot(inWin && ok && tsw);
      }
      // (diag: run-body split below)
      const u64 tdM = __ballot(ok && dropT);
      const u64 snOff = L.h.snOffset + u64(__popcll(tdM & lt));
      u64 osn = p.esn - snOff;  // (an out-of-order lane's is set from the RangeMap below)
      const u64 ots = p.ets - L.h.tsOffset;
      const bool picDrop = ok && dropT && I && ext != prevExt;
      const i32 picOff = L.h.pictureIdOffset + i32(__popcll(__ballot(picDrop) & lt));
      // forwarded: munged descriptor (vp8.go:283-301) + output shape
      const bool fwdIn = ok && !dropT;
      const i32 mext = ext - picOff;
      const u16 mpid = u16(mext & 0x7fff);
      const u8 mtl0 = u8(p.tl0 - L.h.tl0Off);
      const u8 mkey = u8((p.keyidx - L.h.keyIdxOff) & 0x1f);
      u64 cb = 0;
      int cbLen = 0;
      if (video) {
        const bool mM = mpid > 127;
        const int hs = int(p.vhs) + (mM == M ? 0 : (mM ? 1 : -1));
        cbLen = vp8_marshal(p.vfirst, I, mM, mpid, p.vbits & LKF_VP8_L, mtl0, T, p.tid, p.vbits & LKF_VP8_Y,
                            p.vbits & LKF_VP8_K, mkey, hs, cb);
      }
      // (diag: run-body split below)
      // the munger's / sequencer's highest before each lane: the previous in-order push
      const u64 fwC = __ballot(fwdIn);
      const int pf = prev_in(fwC, lt);
      const int pfs = pf >= 0 ? pf : int(lane);
      const u64 pfOsn = sh64(osn, pfs);
      const u64 prevOsn = pf >= 0 ? pfOsn : L.h.seqExtHighestSN;
      const u64 pfOts = sh64(ots, pfs);
      const u64 hiTS = pf >= 0 ? pfOts : L.h.seqExtHighestTS;  // the sequencer's highest TS
      bool fwd = fwdIn;
      // sequencer highest TS = max over pushes; runs keep TS non-decreasing so it is the last one
      const bool tsMono = ots >= hiTS;
      // the first push of a run may skip slots (a gap lane: osn - highest < size - 64)
      // the sequencer slots of a run lie within size - 64 of its highest at the run start
      const bool seqOk = (fl & F_SEQ_INIT) && (fl & F_STATS_INIT) && cbLen >= 0 && tsMono &&
                         (osn == prevOsn + 1 || (gapLane && osn - prevOsn > 1 &&
                                                 osn - prevOsn < u64(L.seqSize) - 64)) &&
                         osn - L.h.seqExtHighestSN < u64(L.seqSize) - 64;
      const bool bad =
          inWin && ((cls == -2) || (cls == -1 && !ok) || (fwdIn && !seqOk));
      const u64 stopM = __ballot(bad || (valid && lane >= pos && !inWin));
      x = stopM ? u32(__ffsll((long long)stopM) - 1) : n;
      if (tswM & ~((1ull << pos) - 1)) x = min(x, u32(__ffsll((long long)(tswM & ~((1ull << pos) - 1))) - 1) + 1u);
      // ---- decide lanes [pos, x) together
      if (x > pos) {
        const u64 runM = (x >= 64 ? ~0ull : ((1ull << x) - 1)) & ~((1ull << pos) - 1);
        const bool inRun = (runM >> lane) & 1;
        const u64 tdR = tdM & runM;
        fwd = fwd && inRun;
        const u64 fwR = __ballot(fwd);             // every forwarded lane (output order)
        const u64 fwInR = fwR;                     // in-order pushes (every forward)
        const u64 selR = tdR | fwInR;              // lanes that advance the munger
        o.nTuples += x - pos;
        // the run's drops: the classification's no-state-change reasons + temporal filter
        o.drops[LKF_DROP_MUTED] += u32(__popcll(__ballot(inRun && cls == LKF_DROP_MUTED)));
        o.drops[LKF_DROP_PAUSED] += u32(__popcll(__ballot(inRun && cls == LKF_DROP_PAUSED)));
        o.drops[LKF_DROP_NOT_SELECTED] += u32(__popcll(__ballot(inRun && cls == LKF_DROP_NOT_SELECTED)));
        o.drops[LKF_DROP_DOWNGRADE] += u32(__popcll(__ballot(inRun && cls == LKF_DROP_DOWNGRADE)));
        o.drops[LKF_DROP_TEMPORAL] += u32(__popcll(tdR));
        // Gap lanes (forwarded after a loss) and picture drops, in lane order:
        // the missing pictures a gap records skip the pictures dropped so far
        // (vp8.go:218-247), a gap exempts its own picture (:249-255), and the
        // sequencer slots it skips are invalidated (sequencer.go:179-189).
        // Sequencer slots are the run-start highest slot + (osn - highest SN).
        const u64 pdR = video ? __ballot(picDrop && inRun) : 0ull;
        const u64 gR = __ballot(gapLane && inRun);
        if (gR) {
          for (u64 m = gR | pdR; m; m &= m - 1) {
            const u32 b = u32(__ffsll((long long)m) - 1);
            const i32 eb = i32(rl32(u32(ext), b));
            if ((pdR >> b) & 1) {
              L.vcDirty = true;
              set_add(L.dropKey, L.h.dropHead, L.h.dropCount, eb, kDropKeep);
              continue;
            }
            if (video) {
              vp8_record_missing(L, i32(rl32(u32(prevExt), b)), eb, i32(rl32(u32(picOff), b)));
              if (rl32(u32(overT), b)) {
                L.vcDirty = true;
                set_add(L.exKey, L.h.exHead, L.h.exCount, eb, kExemptKeep);
              }
            }
            const u64 from = rl64(prevOsn, b), to = rl64(osn, b);  // slots of (from, to) skipped
            const u32 n = u32(to - from - 1);
            u32 base = u32(L.h.seqHighSlot) + u32(from - L.h.seqExtHighestSN) + 1;
            for (u32 i = lane; i < n; i += 64) {  // stores only: no drain needed
              u32 x2 = base + i;
              while (x2 >= L.seqSize) x2 -= L.seqSize;
              store_rec(L.seq + x2, SeqMeta{});
            }
          }
        }
        // output records + sequencer slots of the forwarded lanes
        const int cc = p.hdr0 & 0xf;
        const bool playout = L.extPlayout && !(fl & F_PLAYOUT_ACKED);
        const int extBytes = (playout ? 4 : 0) + (L.extAbs ? 4 : 0) + (L.extTcc ? 3 : 0);
        const int extBlock = extBytes ? 4 + ((extBytes + 3) & ~3) : 0;
        const int hdrLen = 12 + 4 * cc + extBlock;
        const bool useCodec = video && cbLen > 0 && (p.flags & LKF_PKT_VP8);
        const int payLen = useCodec ? (cbLen + int(p.plen) - int(p.vhs)) : int(p.plen);
        const u32 outLen = fwd ? u32(hdrLen + payLen) : 0u;
        const u32 aligned = (outLen + 15) & ~15u;
        const u32 relEx = excl_scan_u32(aligned, lane);
        const bool marker = pktMarker;  // tp.marker (= hdr.Marker for video, false for audio) || hdr.Marker
        const u32 j = u32(__popcll(fwR & lt));
        fwd_base(o, fwR, osn, ots);
        if (fwd) {
#if LKF_CHECKED
          CHK(slot0 + o.nFwd + j < A.tupleCap, CK_DEC_TUPLE, slot0 + o.nFwd + j, A.tupleCap);
#endif
          store_fwd(o.outT + o.nFwd + j, o.outW + o.nFwd + j, o.bSN, o.bTS, osn, ots, pi, o.relOff + relEx, outLen,
                    ((p.flags & LKF_PKT_KEYFRAME) ? LKF_OUT_KEYFRAME : 0) | (marker ? LKF_OUT_MARKER : 0) |
                        (playout ? T_PLAYOUT : 0) | (useCodec ? T_CODEC : 0),
                    0u, useCodec ? vp8_aux(mpid, mtl0, mkey) : 0u);
          // sequencer.push (sequencer.go:123-209): in order, the slot the SN's
          // distance past the highest
          u32 slot = u32(L.h.seqHighSlot) + u32(osn - L.h.seqExtHighestSN);
          while (slot >= L.seqSize) slot -= L.seqSize;
          SeqMeta m = {};
          m.sourceSeqNo = u16(p.esn);
          m.targetSeqNo = u16(osn);
          m.timestamp = u32(ots);
          m.lastNack = u32(p.arr / 1000000LL - L.h.seqStartMs);
          m.marker = marker;
          m.layer = p.layer;
          m.codecLen = u8(video ? cbLen : 0);
#pragma unroll
          for (int i = 0; i < 8; i++) m.codec[i] = u8(cb >> (8 * i));
          CHK(slot < L.seqSize, CK_DEC_SEQ, slot, L.seqSize);
          store_rec(L.seq + slot, m);
        }
        if (fwd) ss_put(o.ssBuf + o.ssN + j, osn, ots, p.arr, p.poff, u32(payLen), marker, kf);
        o.ssN += u32(__popcll(fwR));
        const u32 sumLen = wave_sum_u32(outLen);
        sentAcc += fwd ? i32(p.poff) - hdrLen : 0;  // (reduced once per DownTrack)
        // ---- advance the DownTrack state past the run (uniform)
        if (fwR) {
          o.nBytes += sumLen;
          o.nFwd += u32(__popcll(fwR));
        }
        if (fwInR) {
          const u32 lastF = 63 - __clzll(fwInR);
          u32 slot = u32(L.h.seqHighSlot) + u32(rl64(osn, lastF) - L.h.seqExtHighestSN);
          while (slot >= L.seqSize) slot -= L.seqSize;
          L.h.seqHighSlot = u16(slot);
          L.h.seqExtHighestSN = rl64(osn, lastF);
          L.h.seqExtHighestTS = rl64(ots, lastF);  // >= every earlier push (tsMono)
          if (video) {
            L.h.extLastPictureId = i32(rl32(u32(mext), lastF));
            L.h.lastTl0 = u8(rl32(mtl0, lastF));
            L.h.lastKeyIdx = u8(rl32(mkey, lastF));
          }
        }
        if (selR) {
          const u32 lastSel = 63 - __clzll(selR);
          const u64 mk = __ballot(video && pktMarker);  // marker passed to UpdateAndGetSnTs
          L.h.extHighestIncomingSN = rl64(p.esn, lastSel);
          const bool lastIsF = (fwInR >> lastSel) & 1;
          const u64 pfM = fwInR & ((1ull << lastSel) - 1);
          u64 sSN = L.h.extLastSN, sTS = L.h.extLastTS;
          bool sMk = fl & F_LAST_MARKER;
          if (pfM) {
            const u32 b = 63 - __clzll(pfM);
            sSN = rl64(osn, b);
            sTS = rl64(ots, b);
            sMk = (mk >> b) & 1;
          }
          if (lastIsF) {
            L.h.extSecondLastSN = sSN;
            L.h.extSecondLastTS = sTS;
            L.h.extLastSN = rl64(osn, lastSel);
            L.h.extLastTS = rl64(ots, lastSel);
            setf(L, F_SECOND_LAST_MARKER, sMk);
            setf(L, F_LAST_MARKER, (mk >> lastSel) & 1);
          } else {
            L.h.extSecondLastSN = L.h.extLastSN = sSN;
            L.h.extSecondLastTS = L.h.extLastTS = sTS;
            setf(L, F_SECOND_LAST_MARKER, sMk);
            setf(L, F_LAST_MARKER, sMk);
          }
          if (hasf(L, F_RTX_GATE) && (rl64(osn, lastSel) - L.h.extRtxGateSn) > 2000) setf(L, F_RTX_GATE, false);
          // key frames in the run move the RTX gate to their munged SN
          // (rtpmunger.go:204-208); later lanes are < 64 past it, so the
          // 2000-packet expiry above cannot undo the last one
          const u64 kfM = __ballot(((selR >> lane) & 1) && kf);
          if (kfM) {
            L.h.extRtxGateSn = rl64(osn, 63 - __clzll(kfM));
            setf(L, F_RTX_GATE, true);
          }
          if (video) {
            L.h.wrMaxPictureId = i32(rl32(u32(ext), lastSel));
            setf(L, F_WR_MAX_MBIT, rl32(u32(M), lastSel) != 0);
            // temporal drops: one exclusion per run of consecutive dropped packets
            u64 m = tdR;
            while (m) {
              const u32 b = u32(__ffsll((long long)m) - 1);
              const u64 after = fwInR & ~((2ull << b) - 1);
              const u32 nf = after ? u32(__ffsll((long long)after) - 1) : 64u;
              const u64 runD = tdR & (nf >= 64 ? ~0ull : ((1ull << nf) - 1)) & ~((1ull << b) - 1);
              const u64 s0 = rl64(p.esn, b);
              rm_exclude(L, s0, s0 + u64(__popcll(runD)));
              m &= ~runD;
            }
            if (tdR) L.h.snOffset = L.h.rmOpenValue;
            const u64 tswR = tswM & runM;  // the run's last lane switched the temporal layer
            if (tswR) {
              const u32 b = 63 - __clzll(tswR);
              const i32 nxt = L.h.curT < L.h.tgtT ? i32(rl32(u32(p.tid), b)) : L.h.tgtT;
              L.h.prevS = L.h.curS;
              L.h.prevT = L.h.curT;
              L.h.curT = nxt;
            }
            u64 pd = pdR;
            L.h.pictureIdOffset += i32(__popcll(pd));
            while (pd && !gR) {  // (with gap lanes the drops went into the set in lane order above)
              const u32 b = u32(__ffsll((long long)pd) - 1);
              L.vcDirty = true;
              set_add(L.dropKey, L.h.dropHead, L.h.dropCount, i32(rl32(u32(ext), b)), kDropKeep);
              pd &= pd - 1;
            }
          }
        }
        if (fwR) o.relOff += rl32(relEx + aligned, 63 - __clzll(fwR));
      }
      gapStop = x < n && rl32(u32(gapLater), x) != 0;
      }  // (simulcast / audio runs)
      pos = x;
      if (x < n && rl32(pi, x) < nextAt && !gapStop) {
        // the packet at lane x needs the full restatement
        const uint4 a0 = make_uint4(rl32(r0.x, x), rl32(r0.y, x), rl32(r0.z, x), rl32(r0.w, x));
        const uint4 a1 = make_uint4(rl32(r1.x, x), rl32(r1.y, x), rl32(r1.z, x), rl32(r1.w, x));
        const uint4 a2 = make_uint4(rl32(r2.x, x), rl32(r2.y, x), rl32(r2.z, x), rl32(r2.w, x));
        const uint4 a3 = make_uint4(rl32(r3.x, x), rl32(r3.y, x), rl32(r3.z, x), rl32(r3.w, x));
        const u32 px = rl32(pi, x);
        decide_step<DDK>(L, decode_pkt(a0, a1, a2, a3), px, o);
        vm_drain();
        if (DDK && ddDT) dd_restage(L, sDD, sDDSRaw, lane);
        pos = x + 1;
        if (steady && !steady_state(L)) {  // left the steady state: the chunk ends after this packet
          own = x + 1;
          lim = px + 1;
          break;
        }
      }
    }
    if (steady) {  // the other layers' packets in [kpos, lim): NOT_SELECTED drops
      const u32 skipped = (lim - kpos) - own;
      o.nTuples += skipped;
      o.drops[LKF_DROP_NOT_SELECTED] += skipped;
    }
    if (o.ssN) {  // the chunk's forwarded tuples -> RTPStatsSender
      wave_lds_sync();
#if LKF_SVC_STATS
      const u64 ts0 = __builtin_amdgcn_s_memtime();
#endif
      ss_flush(sSS, o.ssRing, o.ssGap, sSsBuf, o.ssN, o.bSN, o.bTS);
#if LKF_SVC_STATS
      tSs += __builtin_amdgcn_s_memtime() - ts0;
#endif
      o.ssN = 0;
    }
    kpos = lim;
  }
#if LKF_SVC_STATS
  const u64 tP2 = __builtin_amdgcn_s_memtime();
#endif
  while (ev < evEnd) apply_ctl(L, A.events[ev++]);
  __syncthreads();
  {
    const u32 h1 = reinterpret_cast<const u32 *>(&sHot)[lane];
    if (h1 != sHot0[lane]) reinterpret_cast<u32 *>(A.hot + d)[lane] = h1;
  }
  if (o.nFwd && lane < sizeof(SenderStats) / 16)  // (only a forwarded packet changes it)
    reinterpret_cast<uint4 *>(A.ss + d)[lane] = reinterpret_cast<const uint4 *>(&sSS)[lane];
  if (L.rmNew) {  // the ranges appended this batch (the ring's newest): the older ones are unchanged in HBM
    wave_lds_sync();
    const u32 nc = L.h.rmCount, nn = min(L.rmNew, nc);
    for (u32 i = lane; i < nn; i += 64) {
      const u32 idx = (u32(L.h.rmHead) + nc - nn + i) % kRangeCap;
      rmG[idx] = sRm[idx];
    }
  }
  if (ddDT) {
    wave_lds_sync();
    uint4 *g = reinterpret_cast<uint4 *>(A.ddState + d);
    const uint4 *l = reinterpret_cast<const uint4 *>(sDD);
    const u32 nDD = (kDDStateHead + u32(sDD->numChains) * kDDExpRow * 8) / 16;
    for (u32 i = lane; i < nDD; i += 64) g[i] = l[i];
  }
  if ((L.h.flags & F_VP8) && L.vcDirty) {  // the maps go back only when a batch changed them
    if (lane < u32(kSetCap)) {
      L.vc->dropKey[lane] = sDrop[lane];
      L.vc->exKey[lane] = sEx[lane];
    }
    for (u32 i = lane; i < L.h.missCount; i += 64) {
      const u32 idx = (L.h.missHead + i) % kMissCap;
      L.vc->missKey[idx] = sMissKey[idx];
      L.vc->missVal[idx] = sMissVal[idx];
    }
  }
  const i32 sentRun = i32(wave_sum_u32(u32(sentAcc)));  // (every lane: a cross-lane reduction)
  if (lane == 0) {
    A.fwdCnt[d] = u32(o.nFwd);
    A.fwdBytes[d] = o.relOff;
    if (o.nFwd) A.fbase[d] = FwdBase{o.bSN, o.bTS};
    // DownTrack.sendingPacket: bytesSent += header + payload (downtrack.go:1934-1940)
    // (atomics without return: the wave does not wait for a read of the old totals)
    if (o.nFwd) atomicAdd((unsigned long long *)&A.dtCum[d].packets, (unsigned long long)o.nFwd);
    const u64 nSent = o.nBytes + u64(i64(sentRun) + o.sentDiff);
    if (nSent) atomicAdd((unsigned long long *)&A.dtCum[d].bytes, (unsigned long long)nSent);
    A.dtCum[d].flags = L.h.flags;
    // counters: one of kStatCopies partial copies per wave (same-address
    // atomics from every wave would serialise in one L2 channel); k_stats_reduce
    // folds the copies after the kernel
    u64 *st = A.stats + size_t(1 + (w % kStatCopies)) * kStatWords;
    if (o.nTuples) atomicAdd((unsigned long long *)&st[0], (unsigned long long)o.nTuples);
    if (o.nFwd) atomicAdd((unsigned long long *)&st[1], (unsigned long long)o.nFwd);
    if (o.nBytes) atomicAdd((unsigned long long *)&st[2], (unsigned long long)o.nBytes);
#pragma unroll
    for (int i = 0; i < LKF_DROP_NREASONS; i++)
      if (o.drops[i]) atomicAdd((unsigned long long *)&st[4 + i], (unsigned long long)o.drops[i]);
  }
#if LKF_SVC_STATS
  if (DDK && lane == 0 && (L.h.flags & (F_DD | F_VP9))) {
    const u64 tP3 = __builtin_amdgcn_s_memtime();
    SVC_ADD(4, (unsigned long long)(tP1 - tP0));
    SVC_ADD(5, (unsigned long long)tRun);
    SVC_ADD(6, (unsigned long long)tStep);
    SVC_ADD(7, (unsigned long long)(tP2 - tP1 - tRun - tStep));
    SVC_ADD(8, (unsigned long long)(tP3 - tP2));
    SVC_ADD(9, 1ull);
  }
  if (!DDK && lane == 0) {  // the plain DownTracks (g_svc[32..37]): hot-state load, rest of the
    const u64 tP3 = __builtin_amdgcn_s_memtime();  // prologue, body, epilogue, DownTracks, packets
    SVC_ADD(32, (unsigned long long)(tPa - tP0));
    SVC_ADD(33, (unsigned long long)(tP1 - tPa));
    SVC_ADD(34, (unsigned long long)(tP2 - tP1));
    SVC_ADD(35, (unsigned long long)(tP3 - tP2));
    SVC_ADD(36, 1ull);
    SVC_ADD(37, (unsigned long long)(pe - pb));
    SVC_ADD(38, tLoad);
    SVC_ADD(39, tSs);
  }
#endif
  }  // next DownTrack of this wave
}

// ---------------------------------------------------------------------------
// k_emit: wire bytes.  One wave per workgroup; waves run independently (no
// cross-wave barrier), so one wave's prefix phase (dependent loads) hides
// behind the other waves' copy phase.  A wave takes EMIT_G consecutive output
// records (grid-stride over groups):
//   prefix phase  lane = record: owning DownTrack from the group index
//                 (gFirst, a 1-3 step search), then the RTP header +
//                 extension block + munged VP8 descriptor ("prefix") in LDS.
//   copy phase    the group's output bytes as a flat sweep of 16-B chunks,
//                 two windows of 64 chunks per iteration (both loads in
//                 flight together).  A chunk's record comes from a
//                 wave-uniform cursor plus the record starts inside the
//                 window (readlane loop, no per-lane search).  Prefix chunks
//                 come from LDS, payload chunks are byte-shifted copies of the
//                 input packet (two dwordx4 loads + v_alignbyte).
// ---------------------------------------------------------------------------
constexpr int EMIT_T = 64;
constexpr int EMIT_G = 64;
constexpr int PRE_MAX = 96;  // 12 + 4*15 CSRC + 12 extension block + 6 VP8 descriptor = 90
// batches with dependency-descriptor tracks: 12 + 60 CSRC + 4 + (2 + 255) DD + 2 x (2 + 3)
// (two-byte extension profile) = 343
constexpr int PRE_MAX_DD = 352;

#ifndef LKF_EMIT_U  // 16-B chunks per lane in flight per copy iteration (6 with the round-6 residency cap;
#define LKF_EMIT_U 6  // 4, 6 and 8 measured alike at full occupancy, r4_ab_runs.txt)
#endif
constexpr int EMIT_U = LKF_EMIT_U;


struct EmitArgs {
  const u32 *perm;      // output position -> DownTrack (track-major order)
  const u64 *recBase;   // [position] exclusive scan of forwarded counts
  const u64 *byteBase;  // [position] exclusive scan of output bytes
  const u32 *gFirst;    // [group] position owning record group*EMIT_G
  const u64 *slotBase;
  const u64 *totals;    // [0] records, [1] bytes
  const FwdRec *recs;
  const FwdBase *fbase;  // per DownTrack: the base its records' 32-bit SN / TS widen against
  const FwdBase *wide;   // per tuple slot: a T_WIDE record's full SN / TS
  const lkf_pkt *pkts;
  const u8 *arena;
  const DevDT *dts;
  u32 ndts;
  lkf_out *out;
  u8 *outArena;
  u64 outCap, outByteCap;
  u32 *err;
  const u8 *ddArena;  // marshalled DD bytes of T_DD tuples
  const u32 *twccBase;  // per DownTrack: the batch's first transport-wide sequence number (k_twcc_base)
  // capacities (checked builds test device-computed indices against them)
  u32 maxDts, npkts;
  u64 tupleCap, arenaLen, ddCap, gCap;
};

__device__ __forceinline__ u32 align_byte(u32 hi, u32 lo, u32 sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
// the low kb (0..16) bytes of a 16-B chunk kept, the rest zeroed (two 64-bit
// shifts instead of four per-dword selects)
__device__ __forceinline__ uint4 keep_bytes(uint4 v, int kb) {
  const u32 bits = u32(kb < 0 ? 0 : kb > 16 ? 16 : kb) * 8;
  const u64 lo = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
  const u64 hi = bits <= 64 ? 0ull : bits >= 128 ? ~0ull : ((1ull << (bits - 64)) - 1);
  v.x &= u32(lo);
  v.y &= u32(lo >> 32);
  v.z &= u32(hi);
  v.w &= u32(hi >> 32);
  return v;
}
// bytes [s, s + 16) of the arena: one dword-aligned 16-B load plus the next
// dword (global loads need only dword alignment), funnel-shifted by s & 3
struct __attribute__((aligned(4))) U4A {
  u32 x, y, z, w;
};
__device__ __forceinline__ uint4 window_of(const U4A &a, u32 b, u32 rb) {
  uint4 v;
  v.x = align_byte(a.y, a.x, rb);
  v.y = align_byte(a.z, a.y, rb);
  v.z = align_byte(a.w, a.z, rb);
  v.w = align_byte(b, a.w, rb);
  return v;
}
__device__ __forceinline__ uint4 load_window(const u8 *arena, u64 s) {
  const u8 *q = arena + (s & ~u64(3));
  return window_of(*reinterpret_cast<const U4A *>(q), *reinterpret_cast<const u32 *>(q + 16), u32(s & 3));
}
__device__ __forceinline__ void store16(u8 *p, uint4 v) {
  __builtin_nontemporal_store(v.x, reinterpret_cast<u32 *>(p));
  __builtin_nontemporal_store(v.y, reinterpret_cast<u32 *>(p) + 1);
  __builtin_nontemporal_store(v.z, reinterpret_cast<u32 *>(p) + 2);
  __builtin_nontemporal_store(v.w, reinterpret_cast<u32 *>(p) + 3);
}

#ifndef LKF_EMIT_XCD  // (A/B) the XCD-aware group partition (1) or a plain grid-stride (0)
#define LKF_EMIT_XCD 1
#endif
// Round 6: emit's resident workgroups capped through LDS.  With the
// compiler's 6 waves per SIMD (24 one-wave workgroups per CU, 768 per XCD) the
// payload lines that the DownTracks of one track re-read are evicted from the
// XCD's 4 MiB L2 between their readers: exact read bytes (request counters by
// size) 651 MB per configs[1] batch for 319 MB of payload.  Extra LDS per
// workgroup bounds residency (A/B in one GPU call, profiles/r6_ab_runs.txt):
// 12 per CU -> 524 MB, 8 -> 449 MB, 4 -> 339 MB.  The cap is reserved at
// launch as dynamic LDS (EmitLaunch.ldsPad): it pays where emit shares the GPU
// with an ingest chain, and costs where emit has it to itself (§4 DESIGN.md).
template <int PRE>
__global__ void __launch_bounds__(EMIT_T) k_emit(EmitArgs A) {
  __shared__ __attribute__((aligned(16))) u8 pre[EMIT_G][PRE];
  __shared__ u64 sSrc[EMIT_G];  // arena offset of the record's first payload byte after the prefix
  __shared__ u32 sCs[EMIT_G];   // first chunk of the record, relative to the group
  __shared__ u32 sLen[EMIT_G];
  __shared__ u32 sPre[EMIT_G];  // prefix length | (LDS region length << 16)
  const u32 lane = threadIdx.x;
  const u64 total = A.totals[0];
  const u64 ngroups = (total + EMIT_G - 1) / EMIT_G;
  if (total > A.outCap || A.totals[1] > A.outByteCap) {
    if (blockIdx.x == 0 && lane == 0) atomicOr(A.err, 4u);
    return;
  }
  // XCD-aware partition: workgroups are dispatched round-robin over the 8
  // XCDs, so blockIdx % 8 names the XCD.  Each XCD walks its own contiguous
  // eighth of the (track-major) output in order: the records that re-read a
  // track's payloads (one per subscribing DownTrack) are adjacent, so the
  // re-reads hit that XCD's 4 MiB L2 instead of going to HBM.  (Falls back to
  // a plain grid-stride when the grid is not a multiple of 8.)
  const u32 nx = (LKF_EMIT_XCD && gridDim.x % 8 == 0) ? 8u : 1u;
  const u32 xcd = blockIdx.x % nx, slotInX = blockIdx.x / nx, perX = gridDim.x / nx;
  const u64 gpx = (ngroups + nx - 1) / nx;
  const u64 gBeg = u64(xcd) * gpx, gEnd = min(ngroups, gBeg + gpx);
  for (u64 g = gBeg + slotInX; g < gEnd; g += perX) {
    const u64 r0 = g * EMIT_G;
    const u32 nrec = u32(min(u64(EMIT_G), total - r0));
    // ---- prefix phase: lane = record
    CHK(g + 1 < A.gCap, CK_EMIT_GROUP, g + 1, A.gCap);
    const u32 pLo = A.gFirst[g];
    const u32 pHi = (g + 1 < ngroups) ? A.gFirst[g + 1] + 1 : A.ndts;
    u64 outOff = 0;
    if (lane < nrec) {
      const u64 r = r0 + lane;
      // position owning record r: last p in [pLo, pHi) with recBase[p] <= r
      u32 lo = pLo, hi = pHi;
      while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (A.recBase[mid] <= r)
          lo = mid;
        else
          hi = mid;
      }
      CHK(lo < A.ndts, CK_EMIT_POS, lo, A.ndts);
      const u32 d = A.perm[lo];
      CHK(d < A.maxDts, CK_EMIT_DT, d, A.maxDts);
      CHK(A.slotBase[d] + (r - A.recBase[lo]) < A.tupleCap, CK_EMIT_TUPLE, A.slotBase[d] + (r - A.recBase[lo]),
          A.tupleCap);
      const FwdRec *rp = A.recs + (A.slotBase[d] + (r - A.recBase[lo]));
      const U4x8 ra = *reinterpret_cast<const U4x8 *>(rp);  // sn, ts, pkt, rel16
      const uint2 rb = reinterpret_cast<const uint2 *>(rp)[2];  // outLen | flags | ddLen, aux
      const u32 tPkt = ra.z, tLen = rb.x & 0xffffu, tFlags = (rb.x >> 16) & 0xffu, tDDLen = rb.x >> 24, tAux = rb.y;
      CHK(tPkt < A.npkts, CK_EMIT_PKT, tPkt, A.npkts);
      const PktV p = load_pkt(A.pkts + tPkt);
      const DevDT dt = A.dts[d];
      const FwdBase fb = A.fbase[d];
      outOff = A.byteBase[lo] + (u64(ra.w) << 4);
      CHK(r < A.outCap, CK_EMIT_OUT, r, A.outCap);
      CHK(outOff + tLen <= A.outByteCap, CK_EMIT_BYTES, outOff + tLen, A.outByteCap);
      CHK(u64(p.arenaOff) + p.poff + p.plen <= A.arenaLen, CK_EMIT_ARENA, u64(p.arenaOff) + p.poff + p.plen,
          A.arenaLen);
      CHK(!(tFlags & T_DD) || u64(tAux) + tDDLen <= A.ddCap, CK_EMIT_DD, u64(tAux) + tDDLen, A.ddCap);
      u64 extSN = widen32(fb.sn, ra.x), extTS = widen32(fb.ts, ra.y);
      if (tFlags & T_WIDE) {
        const FwdBase wv = A.wide[A.slotBase[d] + (r - A.recBase[lo])];
        extSN = wv.sn;
        extTS = wv.ts;
      }
      lkf_out o;
      o.ext_sn = extSN;
      o.ext_ts = extTS;
      o.out_off = outOff;
      o.dt = d;
      o.pkt = tPkt;
      o.out_len = u16(tLen);
      o.flags = u8(tFlags & 0x0f);  // (the T_* bits stay internal)
      o.layer = p.layer;
      o.reserved = 0;
      A.out[r] = o;
      // prefix: RTP header (getTranslatedRTPHeader downtrack.go:1714-1726)
      u8 *w = pre[lane];
      const int cc = p.hdr0 & 0xf;
      const bool playout = tFlags & T_PLAYOUT;
      const bool ddOn = (PRE == PRE_MAX_DD) && (tFlags & T_DD);
      const bool hasExt = playout || dt.extAbs || ddOn || dt.extTcc;
      // pion's TWCC HeaderExtensionInterceptor: the transport's next sequence
      // number in send order (this record's ordinal in its DownTrack's output
      // after the DownTrack's base)
      const u16 tcc = dt.extTcc ? u16(A.twccBase[d] + u32(r - A.recBase[lo])) : u16(0);
      w[0] = u8((p.hdr0 & 0xe0) | (hasExt ? 0x10 : 0) | cc);  // V, P copied; X per new extensions
      w[1] = u8(((tFlags & LKF_OUT_MARKER) ? 0x80 : 0) | (dt.pt & 0x7f));
      const u16 sn = u16(extSN);
      const u32 ts = u32(extTS);
      w[2] = u8(sn >> 8);
      w[3] = u8(sn);
      w[4] = u8(ts >> 24);
      w[5] = u8(ts >> 16);
      w[6] = u8(ts >> 8);
      w[7] = u8(ts);
      w[8] = u8(dt.ssrc >> 24);
      w[9] = u8(dt.ssrc >> 16);
      w[10] = u8(dt.ssrc >> 8);
      w[11] = u8(dt.ssrc);
      int n = 12;
      const u8 *raw = A.arena + p.arenaOff;
      for (int i = 0; i < 4 * cc; i++) w[n++] = raw[12 + i];
      if (hasExt && !(ddOn && tDDLen > 16)) {  // pion Header.MarshalTo one-byte profile (RFC 8285)
        const int eb = (ddOn ? 1 + tDDLen : 0) + (playout ? 4 : 0) + (dt.extAbs ? 4 : 0) + (dt.extTcc ? 3 : 0);
        const int words = (eb + 3) >> 2;
        w[n++] = 0xBE;
        w[n++] = 0xDE;
        w[n++] = u8(words >> 8);
        w[n++] = u8(words);
        if (ddOn) {  // the DD element first (pacer/base.go:77-83)
          w[n++] = u8((dt.extDD << 4) | (tDDLen - 1));
          for (int i = 0; i < tDDLen; i++) w[n++] = A.ddArena[tAux + i];
        }
        if (playout) {
          w[n++] = u8((dt.extPlayout << 4) | 2);
          w[n++] = dt.playout[0];
          w[n++] = dt.playout[1];
          w[n++] = dt.playout[2];
        }
        if (dt.extAbs) {
          w[n++] = u8((dt.extAbs << 4) | 2);
          w[n++] = 0;
          w[n++] = 0;
          w[n++] = 0;
        }
        if (dt.extTcc) {  // rtp.TransportCCExtension.Marshal: big-endian u16
          w[n++] = u8((dt.extTcc << 4) | 1);
          w[n++] = u8(tcc >> 8);
          w[n++] = u8(tcc);
        }
        for (int i = eb; i < 4 * words; i++) w[n++] = 0;
      } else if (hasExt) {  // two-byte profile 0x1000: a DD element above 16 B
        const int eb = 2 + tDDLen + (playout ? 5 : 0) + (dt.extAbs ? 5 : 0) + (dt.extTcc ? 4 : 0);
        const int words = (eb + 3) >> 2;
        w[n++] = 0x10;
        w[n++] = 0x00;
        w[n++] = u8(words >> 8);
        w[n++] = u8(words);
        w[n++] = dt.extDD;
        w[n++] = tDDLen;
        for (int i = 0; i < tDDLen; i++) w[n++] = A.ddArena[tAux + i];
        if (playout) {
          w[n++] = dt.extPlayout;
          w[n++] = 3;
          w[n++] = dt.playout[0];
          w[n++] = dt.playout[1];
          w[n++] = dt.playout[2];
        }
        if (dt.extAbs) {
          w[n++] = dt.extAbs;
          w[n++] = 3;
          w[n++] = 0;
          w[n++] = 0;
          w[n++] = 0;
        }
        if (dt.extTcc) {
          w[n++] = dt.extTcc;
          w[n++] = 2;
          w[n++] = u8(tcc >> 8);
          w[n++] = u8(tcc);
        }
        for (int i = eb; i < 4 * words; i++) w[n++] = 0;
      }
      u64 src = u64(p.arenaOff) + p.poff;
      if (tFlags & T_CODEC) {  // translateVP8PacketTo downtrack.go:1728-1736: the munged
                               // descriptor, re-marshalled from its munged fields as decide did
        const u16 mpid = u16(tAux & 0xffffu);
        const bool mM = mpid > 127, M = p.vbits & LKF_VP8_M;
        const int hs = int(p.vhs) + (mM == M ? 0 : (mM ? 1 : -1));
        u64 cb = 0;
        const int cl = vp8_marshal(p.vfirst, p.vbits & LKF_VP8_I, mM, mpid, p.vbits & LKF_VP8_L, u8(tAux >> 16),
                                   p.vbits & LKF_VP8_T, p.tid, p.vbits & LKF_VP8_Y, p.vbits & LKF_VP8_K,
                                   u8(tAux >> 24), hs, cb);
#pragma unroll
        for (int i = 0; i < 6; i++)
          if (i < cl) w[n + i] = u8(cb >> (8 * i));
        n += cl > 0 ? cl : 0;
        src += p.vhs;
      }
      // LDS region = prefix rounded up to 16 B, its tail filled from the
      // payload (so every 16-B chunk is either all-LDS or all-payload)
      const int R = (n + 15) & ~15;
      if (R > n) {
        const uint4 v = load_window(A.arena, src);
        const u32 vw[4] = {v.x, v.y, v.z, v.w};
        for (int i = n; i < R; i++) {
          const int b = i - n;
          w[i] = (i < int(tLen)) ? u8(vw[b >> 2] >> (8 * (b & 3))) : 0;
        }
      }
      sSrc[lane] = src;
      sLen[lane] = tLen;
      sPre[lane] = u32(n) | (u32(R) << 16);
    }
    // first chunk of each record relative to the group's first output byte
    const u64 gByte = rl64(outOff, 0);
    if (lane < nrec) sCs[lane] = u32((outOff - gByte) >> 4);
    __syncthreads();  // one wave: orders the LDS writes above before the cross-lane reads below
    // ---- copy phase: flat sweep of the group's 16-B chunks
    const u32 nchunks = sCs[nrec - 1] + ((sLen[nrec - 1] + 15) >> 4);
    u8 *const outG = A.outArena + gByte;
    u32 cur = 0;  // wave-uniform: a record whose first chunk is <= c0
    for (u32 c0 = 0; c0 < nchunks;) {
      u32 wEnd = min(c0 + EMIT_U * 64, nchunks);
      const u32 ji = cur + 1 + lane;
      const u32 st = ji < nrec ? sCs[ji] : 0xffffffffu;
      u64 inW = __ballot(st < wEnd);
      if (inW == ~0ull) {  // more than 63 records start in the window: cut it
        wEnd = rl32(st, 63);
        inW = __ballot(st < wEnd);
      }
      const u32 k = u32(__popcll(inW));
      u32 c[EMIT_U], j[EMIT_U];
#pragma unroll
      for (int u = 0; u < EMIT_U; u++) {
        c[u] = c0 + 64u * u + lane;
        j[u] = cur;
      }
      for (u32 i = 0; i < k; i++) {
        const u32 sv = rl32(st, i);
#pragma unroll
        for (int u = 0; u < EMIT_U; u++) j[u] += c[u] >= sv ? 1u : 0u;
      }
      // sources of the lane's chunks, then all their loads in flight together
      bool act[EMIT_U], lds[EMIT_U];
      u32 o[EMIT_U];
      u64 src[EMIT_U];
      U4A qa[EMIT_U];
      u32 qb[EMIT_U];
      uint4 v[EMIT_U];
#pragma unroll
      for (int u = 0; u < EMIT_U; u++) {
        act[u] = c[u] < wEnd;
        o[u] = (c[u] - sCs[j[u]]) << 4;
        const u32 pr = sPre[j[u]];
        lds[u] = o[u] < (pr >> 16);
        src[u] = sSrc[j[u]] + (o[u] - (pr & 0xffff));
        qa[u] = U4A{0, 0, 0, 0};
        qb[u] = 0;
        if (act[u] && !lds[u]) {  // (issued together: the loads of all EMIT_U chunks in flight)
          CHK((src[u] & ~u64(3)) + 20 <= A.arenaLen + 32, CK_EMIT_ARENA, (src[u] & ~u64(3)) + 20, A.arenaLen + 32);
          const u8 *q = A.arena + (src[u] & ~u64(3));
          qa[u] = *reinterpret_cast<const U4A *>(q);
          qb[u] = *reinterpret_cast<const u32 *>(q + 16);
        }
      }
#pragma unroll
      for (int u = 0; u < EMIT_U; u++) {
        if (!act[u]) continue;
        if (lds[u])
          v[u] = *reinterpret_cast<const uint4 *>(&pre[j[u]][o[u]]);
        else  // the funnel shift, then the 16-B tail padding zeroed
          v[u] = keep_bytes(window_of(qa[u], qb[u], u32(src[u] & 3)), int(sLen[j[u]]) - int(o[u]));
        CHK(gByte + (u64(c[u]) << 4) + 16 <= A.outByteCap + 64, CK_EMIT_BYTES, gByte + (u64(c[u]) << 4) + 16,
            A.outByteCap + 64);
        store16(outG + (u64(c[u]) << 4), v[u]);
      }
      cur += k;
      c0 = wEnd;
    }
    __syncthreads();  // LDS reused by the next group
  }
}

// getExtPacketMetas sequencer.go:277-300: the ring slot of NACKed sn, or -1
// (out of order from the head, an excluded padding SN, or too old).  Without
// padding exclusions slot = extSN % size = seqHighSlot - (highest - extSN).
__device__ int seq_find(const DTHot &h, SeqRM *srm, u32 cap, u32 size, u16 sn, u64 &extSN) {
  const u16 highestSN = u16(h.seqExtHighestSN);
  if (u16(highestSN - sn) > (1 << 15)) return -1;
  extSN = u64(sn) + (h.seqExtHighestSN & 0xFFFFFFFFFFFF0000ull);
  if (sn > highestSN) extSN -= (1ull << 16);
  u64 off = 0, snOff = 0;
  if (h.flags & F_SEQ_RM) {
    if (!srm_get(srm, cap, extSN, off)) return -1;
    snOff = srm->snOffset;
  }
  const u64 dist = (h.seqExtHighestSN - snOff) - (extSN - off);
  if (dist >= u64(size)) return -1;
  const i32 sl = i32(h.seqHighSlot) - i32(dist);
  return sl < 0 ? sl + i32(size) : sl;
}

// ---------------------------------------------------------------------------
// sequencer.getExtPacketMetas sequencer.go:263-332 for one DownTrack (RTX
// lookup; one lane, serial over the NACKed sequence numbers).
// ---------------------------------------------------------------------------
__global__ void k_seq_lookup(DTHot *hot, SeqMeta *seqBase, u32 seqSize, u8 *srmBase, u64 srmStride, u32 srmCap, u32 d,
                             const u16 *sns, u32 n, i64 nowMs, lkf_seq_meta *out, u32 *nOut) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DTHot h = hot[d];
  SeqMeta *seq = seqBase + size_t(d) * seqSize;
  u32 cnt = 0;
  if (h.flags & F_SEQ_INIT) {
    const u32 rtt = 70;  // defaultRtt (setRTT is out of scope)
    const u32 refTime = u32(nowMs - h.seqStartMs);
    const u32 highestTS = u32(h.seqExtHighestTS);
    SeqRM *srm = reinterpret_cast<SeqRM *>(srmBase + size_t(d) * srmStride);
    for (u32 i = 0; i < n; i++) {
      const u16 sn = sns[i];
      u64 extSN = 0;
      const int slot = seq_find(h, srm, srmCap, seqSize, sn, extSN);
      if (slot < 0) continue;
      SeqMeta &m = seq[slot];
      const bool invalid = m.sourceSeqNo == 0 && m.targetSeqNo == 0 && m.lastNack == 0;
      if (m.targetSeqNo != sn || invalid) continue;
      const u32 lim = (2 * rtt < 100) ? 2 * rtt : 100;
      if (m.nacked < 3 && u32(refTime - m.lastNack) > lim) {
        m.nacked++;
        m.lastNack = refTime;
        u64 extTS = u64(m.timestamp) + (h.seqExtHighestTS & 0xFFFFFFFF00000000ull);
        if (m.timestamp > highestTS) extTS -= (1ull << 32);
        lkf_seq_meta o = {};
        o.ext_sn = extSN;
        o.ext_ts = extTS;
        o.source_sn = m.sourceSeqNo;
        o.target_sn = m.targetSeqNo;
        o.timestamp = m.timestamp;
        o.last_nack = m.lastNack;
        o.marker = m.marker;
        o.nacked = m.nacked;
        o.layer = m.layer;
        o.codec_len = m.codecLen;
        for (int k = 0; k < 8; k++) o.codec[k] = m.codec[k];
        out[cnt++] = o;
      }
    }
  }
  *nOut = cnt;
}

// ---------------------------------------------------------------------------
// k_seq_dd: the ddBytes of sequencer.push (sequencer.go:198-199) for the
// DownTracks that can forward a dependency descriptor (one wave each, after
// the batch's decide, on the decide stream, so the DownTrack's sequencer head
// is the batch's final one).  A tuple whose record is still in the ring —
// seq_find of its munged SN gives a slot holding that target and source SN —
// stores its descriptor bytes (or none) in the slot's 256-B DD entry (length
// byte + up to 255 bytes); a tuple pushed out later in the batch or never
// stored (too old) has no slot, as in the reference.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_seq_dd(const u32 *__restrict__ list, u32 n, const DTHot *__restrict__ hot,
                                               const SeqMeta *__restrict__ seqBase, u32 seqSize, u8 *srmBase,
                                               u64 srmStride, u32 srmCap, const u32 *__restrict__ ddIdx, u8 *seqDD,
                                               const FwdRec *__restrict__ recs, const FwdBase *__restrict__ fbase,
                                               const FwdBase *__restrict__ wide,
                                               const u64 *__restrict__ slotBase,
                                               const u32 *__restrict__ fwdCnt, const lkf_pkt *__restrict__ pkts,
                                               const u8 *__restrict__ ddArena) {
  const u32 w = blockIdx.x, lane = threadIdx.x;
  if (w >= n) return;
  const u32 d = list[w];
  const u32 cnt = fwdCnt[d];
  if (!cnt) return;
  const DTHot h = hot[d];
  if (!(h.flags & F_SEQ_INIT)) return;
  const SeqMeta *seq = seqBase + size_t(d) * seqSize;
  SeqRM *srm = reinterpret_cast<SeqRM *>(srmBase + size_t(d) * srmStride);
  u8 *ring = seqDD + size_t(ddIdx[d]) * seqSize * kSeqDDBytes;
  const FwdRec *tp = recs + slotBase[d];
  const u64 bSN = fbase[d].sn;
  for (u32 c0 = 0; c0 < cnt; c0 += 64) {
    const u32 k = c0 + lane;
    if (k < cnt) {
      const FwdRec t = tp[k];
      const u64 extSN = (t.flags & T_WIDE) ? wide[slotBase[d] + k].sn : widen32(bSN, t.sn);
      u64 ext = 0;
      const int slot = seq_find(h, srm, srmCap, seqSize, u16(extSN), ext);
      if (slot >= 0 && ext == extSN && seq[slot].targetSeqNo == u16(extSN) &&
          seq[slot].sourceSeqNo == u16(pkts[t.pkt].ext_sn)) {
        u8 *e = ring + size_t(slot) * kSeqDDBytes;
        const u32 len = (t.flags & T_DD) ? t.ddLen : 0u;
        e[0] = u8(len);
        for (u32 i = 0; i < len; i++) e[1 + i] = ddArena[t.aux + i];
      }
    }
  }
}

hipError_t launch_seq_dd(hipStream_t s, const SeqDDLaunch &a) {
  if (!a.n) return hipSuccess;
  hipLaunchKernelGGL(k_seq_dd, dim3(a.n), dim3(64), 0, s, a.list, a.n, a.hot, a.seq, a.seqSize, a.srm, a.srmStride,
                     a.srmCap, a.ddIdx, a.seqDD, a.recs, a.fbase, a.wide, a.slotBase, a.fwdCnt, a.pkts, a.ddArena);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_rtx_lookup: DownTrack.retransmitPackets up to Receiver.ReadRTP
// (downtrack.go:1596-1631) for many DownTracks at once — one lane per
// DownTrack NACK list (serial over it, as getExtPacketMetas mutates the
// records it returns).  FilterRTX layers (forwarder.go:1424-1432) from the
// DownTrack's state; out[k]/valid[k] per NACK entry (compacted on the host).
// ---------------------------------------------------------------------------
__global__ void k_rtx_lookup(const DTHot *__restrict__ hot, SeqMeta *seqBase, u32 seqSize, u8 *srmBase,
                             u64 srmStride, u32 srmCap, const lkf_nack *__restrict__ nacks, const u32 *__restrict__ gStart, u32 ngroups, i64 nowMs,
                             lkf_rtx *__restrict__ out, u32 *__restrict__ valid) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  const u32 b = gStart[g], e = gStart[g + 1];
  const u32 d = u32(nacks[b].dt);
  const DTHot h = hot[d];
  SeqMeta *seq = seqBase + size_t(d) * seqSize;
  // FlagFilterRTXLayers: disallowed while deficient and target < current, or above current
  const bool def = h.flags & F_DEFICIENT;
  const i32 curS = h.curS, tgtS = h.tgtS;
  const u32 rtt = 70;  // defaultRtt (setRTT is out of scope)
  const u32 refTime = u32(nowMs - h.seqStartMs);
  const u32 highestTS = u32(h.seqExtHighestTS);
  SeqRM *srm = reinterpret_cast<SeqRM *>(srmBase + size_t(d) * srmStride);
  for (u32 k = b; k < e; k++) {
    u32 ok = 0;
    const u16 sn = nacks[k].sn;
    u64 extSN = 0;
    const int slot = (h.flags & F_SEQ_INIT) ? seq_find(h, srm, srmCap, seqSize, sn, extSN) : -1;
    if (slot >= 0) {
      {
        SeqMeta &m = seq[slot];
        const bool invalid = m.sourceSeqNo == 0 && m.targetSeqNo == 0 && m.lastNack == 0;
        const u32 lim = (2 * rtt < 100) ? 2 * rtt : 100;
        if (m.targetSeqNo == sn && !invalid && m.nacked < 3 && u32(refTime - m.lastNack) > lim) {
          m.nacked++;
          m.lastNack = refTime;
          const i32 l = m.layer;
          const bool dis = def && (tgtS < curS || l > curS) && l >= 0 && l <= 2;
          if (!dis) {
            u64 extTS = u64(m.timestamp) + (h.seqExtHighestTS & 0xFFFFFFFF00000000ull);
            if (m.timestamp > highestTS) extTS -= (1ull << 32);
            lkf_rtx r = {};
            r.meta.ext_sn = extSN;
            r.meta.ext_ts = extTS;
            r.meta.source_sn = m.sourceSeqNo;
            r.meta.target_sn = m.targetSeqNo;
            r.meta.timestamp = m.timestamp;
            r.meta.last_nack = m.lastNack;
            r.meta.marker = m.marker;
            r.meta.nacked = m.nacked;
            r.meta.layer = m.layer;
            r.meta.codec_len = m.codecLen;
            for (int q = 0; q < 8; q++) r.meta.codec[q] = m.codec[q];
            r.dt = int32_t(d);
            r.reserved = u32(slot) + 1;  // the sequencer slot: lkf_rtx_emit reads its ddBytes there
            out[k] = r;
            ok = 1;
          }
        }
      }
    }
    valid[k] = ok;
  }
}

hipError_t launch_rtx_lookup(hipStream_t s, const DTHot *hot, SeqMeta *seq, u32 seqSize, u8 *srm, u64 srmStride,
                             u32 srmCap, const lkf_nack *nacks, const u32 *gStart, u32 ngroups, i64 nowMs, lkf_rtx *out,
                             u32 *valid) {
  if (!ngroups) return hipSuccess;
  hipLaunchKernelGGL(k_rtx_lookup, dim3((ngroups + 63) / 64), dim3(64), 0, s, hot, seq, seqSize, srm, srmStride, srmCap,
                     nacks, gStart, ngroups, nowMs, out, valid);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Padding and blank frames: DownTrack.WritePaddingRTP
// (downtrack.go:764-859) and one tick of writeBlankFrameRTP (:1307-1401) for
// many DownTracks at once, one wave per request (distinct DownTracks).  The
// DownTrack's state is staged in LDS like a decide wave's; the munger's
// RangeMap ring is used in place (a control-rate path).
// ---------------------------------------------------------------------------
__constant__ u8 kVP8KeyFrame8x8[31] = {0x10, 0x02, 0x00, 0x9d, 0x01, 0x2a, 0x08, 0x00, 0x08, 0x00, 0x00,
                                        0x47, 0x08, 0x85, 0x85, 0x88, 0x85, 0x84, 0x88, 0x02, 0x02, 0x00,
                                        0x0c, 0x0d, 0x60, 0x00, 0xfe, 0xff, 0xab, 0x50, 0x80};  // downtrack.go:91-96
// STAP-A of H264KeyFrame2x2 SPS, PPS, IDR (downtrack.go:98-110, getH264BlankFrame :1456-1472)
__constant__ u8 kH264Blank[47] = {0x18, 0x00, 0x18, 0x67, 0x42, 0xc0, 0x1f, 0x0f, 0xd9, 0x1f, 0x88, 0x88, 0x84,
                                  0x00, 0x00, 0x03, 0x00, 0x04, 0x00, 0x00, 0x03, 0x00, 0xc8, 0x3c, 0x60, 0xc9,
                                  0x20, 0x00, 0x06, 0x68, 0x87, 0xcb, 0x83, 0xcb, 0x20, 0x00, 0x0a, 0x65, 0x88,
                                  0x84, 0x0a, 0xf2, 0x62, 0x80, 0x00, 0xa7, 0xbe};
constexpr int kOpusSilenceLen = 80;  // OpusSilenceFrame downtrack.go:112-123: f8 ff fe, then zeros
constexpr u32 kPadPayload = 255;     // RTPPaddingMaxPayloadSize downtrack.go:63
constexpr u32 kPadEstHdr = 20;       // RTPPaddingEstimatedHeaderSize downtrack.go:64

// RangeMap.DecValue rangemap.go:70-88 (munger ring, prune as rm_exclude)
__device__ void rm_dec(Lane &L, u64 end, u64 dec) {
  if (L.h.rmOpenStart > end) {
    L.h.rmOpenValue -= dec;
    return;
  }
  RangeEntry c;
  c.start = L.h.rmOpenStart;
  c.end = end;
  c.value = L.h.rmOpenValue;
  if (L.h.rmCount < kRangeCap) {
    const int idx = (int(L.h.rmHead) + int(L.h.rmCount)) % kRangeCap;
    if (lane_id() == 0) L.rm[idx] = c;
    L.h.rmCount++;
  } else {
    if (lane_id() == 0) L.rm[L.h.rmHead] = c;
    L.h.rmHead = u16((L.h.rmHead + 1) % kRangeCap);
  }
  L.h.rmOpenStart = end + 1;
  L.h.rmOpenValue = c.value - dec;
}
// RTPMunger.UpdateAndGetPaddingSnTs rtpmunger.go:288-346.  ts[0..1]: the
// timestamps of the first two packets (frameRate != 0 only with num <= 2);
// every timestamp is extLastTS for frameRate 0.  false: not on a frame boundary.
__device__ bool mg_padding(Lane &L, u32 num, u32 clockRate, u32 frameRate, bool forceMarker, u64 extRtpTS,
                           u64 ts[2]) {
  if (num == 0) return true;
  bool useLast = false;
  u32 tsOff = 0;
  if (!hasf(L, F_LAST_MARKER)) {
    if (!forceMarker) return false;
    useLast = true;
    tsOff = 1;
  }
  const u64 lastTS = L.h.extLastTS;
  u64 eLastTS = lastTS;
  ts[0] = ts[1] = lastTS;
  if (frameRate != 0) {
    for (u32 i = 0; i < num && i < 2; i++) {
      if (useLast && i == 0) {
        ts[i] = lastTS;
      } else {
        u64 ets = extRtpTS + u64((u32(u32(i + 1 - tsOff) * clockRate) + frameRate - 1) / frameRate);
        if (i64(ets - eLastTS) <= 0) ets = eLastTS + 1;
        eLastTS = ets;
        ts[i] = ets;
      }
    }
  }
  const u64 eLastSN = L.h.extLastSN + num;
  L.h.extSecondLastSN = eLastSN - 1;
  L.h.extLastSN = eLastSN;
  rm_dec(L, L.h.extHighestIncomingSN, num);
  mg_updateSnOffset(L);
  L.h.extSecondLastTS = (num == 1 || frameRate == 0) ? lastTS : ts[num - 2];  // (frameRate 0: all lastTS)
  L.h.tsOffset -= eLastTS - lastTS;
  L.h.extLastTS = eLastTS;
  if (forceMarker) setf(L, F_LAST_MARKER, true);
  return true;
}
// Forwarder.maybeStart forwarder.go:1766-1796 (the random start comes with the request)
__device__ void fw_maybeStart(Lane &L, i64 now, u64 startSN, u64 startTS) {
  if (hasf(L, F_STARTED)) return;
  setf(L, F_STARTED, true);
  L.h.preStartTime = now;
  mg_setLastSnTs(L, startSN, startTS);
  L.h.extFirstTS = startTS;
}
// sequencer.pushPadding sequencer.go:211-261 (video DownTracks: the sequencer
// has its RangeMap).  One thread; the caller syncs the wave after it.
__device__ void seq_push_padding(Lane &L, u64 s, u64 e) {
  const u32 size = L.seqSize;
  const bool rmOn = hasf(L, F_SEQ_RM);
  const u64 snOff = rmOn ? L.srm->snOffset : 0;
  const u64 hi = L.h.seqExtHighestSN;
  if (s <= hi) {  // before what is already sequenced: invalidate those slots
    for (u64 sn = s; sn != e + 1; sn++) {
      const i64 diff = i64(sn - hi);
      if (diff >= 0 || diff < -i64(size)) continue;
      u64 off = 0;
      if (rmOn && !srm_get(L.srm, L.srmCap, sn, off)) continue;
      const u64 dist = (hi - snOff) - (sn - off);
      if (dist >= u64(size)) continue;
      i32 sl = i32(L.h.seqHighSlot) - i32(dist);
      if (sl < 0) sl += i32(size);
      L.seq[sl] = SeqMeta{};
    }
    return;
  }
  if (!rmOn) {  // first exclusion: the identity map (NewRangeMap: open range [0, inf) -> 0)
    L.srm->openStart = 0;
    L.srm->openValue = 0;
    L.srm->snOffset = 0;
    L.srm->head = L.srm->count = 0;
  }
  if (!srm_exclude(L.srm, L.srmCap, s, e + 1, true)) return;
  u64 nOff = snOff;
  if (srm_get(L.srm, L.srmCap, e + 1, nOff)) L.srm->snOffset = nOff;  // updateSNOffset
  nOff = L.srm->snOffset;
  if (hasf(L, F_SEQ_INIT)) {  // the slot of the (adjusted) highest SN moves with it
    const u64 mv = u64((e - nOff) - (hi - snOff)) % size;
    L.h.seqHighSlot = u16((u64(L.h.seqHighSlot) + mv) % size);
  }
  L.h.seqExtHighestSN = e;
  setf(L, F_SEQ_RM, true);
}
// codecmunger.VP8.UpdateAndGetPadding vp8.go:304-363 -> marshalled descriptor
__device__ int vp8_padding(Lane &L, bool newPicture, u64 &out) {
  const i32 offset = newPicture ? 1 : 0;
  const bool picUsed = hasf(L, F_PICID_USED), tl0Used = hasf(L, F_TL0_USED), tidUsed = hasf(L, F_TID_USED),
             keyUsed = hasf(L, F_KEYIDX_USED);
  int hs = 1;
  if (picUsed || tl0Used || tidUsed || keyUsed) hs += 1;
  i32 ext = L.h.extLastPictureId;
  if (picUsed) {
    ext = L.h.extLastPictureId + offset;
    L.h.extLastPictureId = ext;
    L.h.pictureIdOffset -= offset;
    hs += ((ext & 0x7fff) > 127) ? 2 : 1;
  }
  const u16 pid = u16(ext & 0x7fff);
  u8 tl0 = 0;
  if (tl0Used) {
    tl0 = u8(L.h.lastTl0 + offset);
    L.h.lastTl0 = tl0;
    L.h.tl0Off = u8(L.h.tl0Off - offset);
    hs += 1;
  }
  if (tidUsed || keyUsed) hs += 1;
  u8 key = 0;
  if (keyUsed) {
    key = u8((L.h.lastKeyIdx + offset) & 0x1f);
    L.h.lastKeyIdx = key;
    L.h.keyIdxOff = u8(L.h.keyIdxOff - offset);
  }
  return vp8_marshal(0x10, picUsed, pid > 127, pid, tl0Used, tl0, tidUsed, 0, true, keyUsed, key, hs, out);
}

struct PadArgs {
  int blank;
  u32 n;
  const lkf_pad_req *reqs;
  i64 nowNs;
  DTHot *hot;
  const DevDT *dts;
  const DevTrack *tracks;
  RangeEntry *rm;
  SeqMeta *seq;
  u32 seqSize;
  u8 *srm;
  u64 srmStride;
  u32 srmCap;
  DTCum *dtCum;
  const u64 *recOff, *byteOff;
  lkf_out *out;
  u8 *arena;
  u32 *cnt, *bytes;
};

// RTP header of a padding / blank packet (pion Header.MarshalTo; pacer
// writeRTPHeaderExtensions pacer/base.go:71-100: abs-send-time placeholder)
__device__ __forceinline__ u32 pad_hdr_len(const DevDT &dt) {
  const u32 eb = (dt.extAbs ? 4u : 0u) + (dt.extTcc ? 3u : 0u);
  return eb ? 16u + ((eb + 3) & ~3u) : 12u;
}
// (the transport-cc element, when negotiated, is written with 0 and stamped in
// send order by k_twcc_stamp after the kernel)
__device__ int pad_header(u8 *w, bool padding, bool marker, const DevDT &dt, u64 sn, u64 ts) {
  w[0] = u8(0x80 | (padding ? 0x20 : 0) | ((dt.extAbs || dt.extTcc) ? 0x10 : 0));
  w[1] = u8((marker ? 0x80 : 0) | (dt.pt & 0x7f));
  w[2] = u8(sn >> 8);
  w[3] = u8(sn);
  w[4] = u8(ts >> 24);
  w[5] = u8(ts >> 16);
  w[6] = u8(ts >> 8);
  w[7] = u8(ts);
  w[8] = u8(dt.ssrc >> 24);
  w[9] = u8(dt.ssrc >> 16);
  w[10] = u8(dt.ssrc >> 8);
  w[11] = u8(dt.ssrc);
  const int hl = int(pad_hdr_len(dt));
  if (hl == 12) return 12;
  w[12] = 0xBE;
  w[13] = 0xDE;
  w[14] = 0;
  w[15] = u8((hl - 16) / 4);
  int n = 16;
  if (dt.extAbs) {
    w[n++] = u8((dt.extAbs << 4) | 2);
    w[n++] = 0;
    w[n++] = 0;
    w[n++] = 0;
  }
  if (dt.extTcc) {
    w[n++] = u8((dt.extTcc << 4) | 1);
    w[n++] = 0;
    w[n++] = 0;
  }
  while (n < hl) w[n++] = 0;
  return hl;
}
__device__ void pad_record(const PadArgs &A, u32 r, u32 k, u32 d, u64 off, u32 len, u64 sn, u64 ts, bool marker) {
  lkf_out o;
  o.ext_sn = sn;
  o.ext_ts = ts;
  o.out_off = off;
  o.dt = d;
  o.pkt = r;
  o.out_len = u16(len);
  o.flags = marker ? LKF_OUT_MARKER : 0;
  o.layer = -1;
  o.reserved = 0;
  A.out[A.recOff[r] + k] = o;
}

__global__ void __launch_bounds__(64) k_pad(PadArgs A) {
  __shared__ __attribute__((aligned(16))) DTHot sHot;
  const u32 r = blockIdx.x, lane = threadIdx.x;
  if (r >= A.n) return;
  const lkf_pad_req q = A.reqs[r];
  const u32 d = u32(q.dt);
  reinterpret_cast<u32 *>(&sHot)[lane] = reinterpret_cast<const u32 *>(A.hot + d)[lane];
  __syncthreads();
  Lane L{sHot};
  L.rm = A.rm + size_t(d) * kRangeCap;  // (the ring in place: nothing to stage or write back)
  L.rmG = L.rm;
  L.rmNew = 0;
  L.rmLoaded = true;
  L.vcDirty = false;
  L.seq = A.seq + size_t(d) * A.seqSize;
  L.seqSize = A.seqSize;
  L.srm = reinterpret_cast<SeqRM *>(A.srm + size_t(d) * A.srmStride);
  L.srmCap = A.srmCap;
  const DevDT dt = A.dts[d];
  const DevTrack &tk = A.tracks[dt.track];
  L.kind = tk.kind;
  L.codec = tk.codec;
  L.clockRate = tk.clockRate;
  const bool onMute = q.flags & LKF_PAD_ON_MUTE;
  const bool active = hasf(L, F_STATS_INIT);  // rtpStats.IsActive (rtpstats_base.go:308)
  u32 nPk = 0, nBytes = 0;
  const u64 ob = A.byteOff[r];
  if (!A.blank) {
    bool ok = (q.flags & LKF_PAD_WRITABLE) != 0;
    if (!active && !onMute) ok = false;
    if (L.kind == LKF_KIND_AUDIO) ok = false;
    if (hasf(L, F_MUTED) && !onMute) ok = false;
    if (!(q.flags & LKF_PAD_RR_SEEN) && !onMute) ok = false;
    const u32 num = (q.bytes_to_send + kPadPayload + kPadEstHdr - 1) / (kPadPayload + kPadEstHdr);
    if (num == 0) ok = false;
    if (ok) {
      fw_maybeStart(L, A.nowNs, u16(q.start_sn), q.start_ts);  // GetSnTsForPadding forwarder.go:1798-1813
      const bool force = (q.flags & LKF_PAD_FORCE_MARKER) || L.h.tgtS == INVALID || L.h.tgtT == INVALID;
      const u64 first = L.h.extLastSN + 1;
      u64 ts[2];
      if (mg_padding(L, num, 0, 0, force, 0, ts)) {
        __syncthreads();
        if (lane == 0) seq_push_padding(L, first, first + num - 1);
        __syncthreads();
        const u32 len = pad_hdr_len(dt) + kPadPayload;
        const u32 stride = (len + 15) & ~15u;
        for (u32 k = lane; k < num; k += 64) {
          u8 *w = A.arena + ob + u64(k) * stride;
          const int h = pad_header(w, true, false, dt, first + k, ts[0]);
          for (u32 i = 0; i < kPadPayload - 1; i++) w[h + i] = 0;
          w[h + kPadPayload - 1] = u8(kPadPayload);  // the padding size, that byte included
          for (u32 i = len; i < stride; i++) w[i] = 0;
          pad_record(A, r, k, d, ob + u64(k) * stride, len, first + k, ts[0], false);
        }
        nPk = num;
        nBytes = num * (12 + kPadPayload);  // hdr.MarshalSize() + len(payload) (downtrack.go:854)
      }
    }
  } else {
    const u32 codec = L.codec;
    bool ok = (q.flags & LKF_PAD_WRITABLE) && active &&
              (codec == LKF_CODEC_OPUS || codec == LKF_CODEC_VP8 || codec == LKF_CODEC_H264);
    if (ok) {
      const u32 frameRate = codec == LKF_CODEC_OPUS ? 50 : 30;
      fw_maybeStart(L, A.nowNs, u16(q.start_sn), q.start_ts);  // GetSnTsForBlankFrames forwarder.go:1815-1839
      const bool fen = !hasf(L, F_LAST_MARKER);
      const u32 num = fen ? 2 : 1;
      const u64 lastTS = L.h.extLastTS;
      u64 expTS = lastTS;
      if (hasf(L, F_HAS_EXPECTED) && active) {  // getExpectedRTPTimestamp downtrack.go:1765
        const i64 diff = (A.nowNs - L.h.statsFirstTime) * i64(L.clockRate) / 1000000000LL;
        expTS = L.h.statsExtStartTS + u64(diff);
      }
      if (i64(expTS - lastTS) <= 0) expTS = lastTS + 1;
      const u64 first = L.h.extLastSN + 1;
      u64 ts[2];
      mg_padding(L, num, L.clockRate, frameRate, fen, expTS, ts);  // forceMarker = frameEndNeeded: no error
      u64 off = ob;
      for (u32 k = 0; k < num; k++) {
        u64 vd = 0;
        int vl = 0;
        if (codec == LKF_CODEC_VP8 && hasf(L, F_VP8)) vl = vp8_padding(L, !(k == 0 && fen), vd);
        const u32 pl = codec == LKF_CODEC_OPUS ? u32(kOpusSilenceLen) : codec == LKF_CODEC_H264 ? 47u : u32(vl) + 31u;
        const u32 len = pad_hdr_len(dt) + pl;
        if (lane == 0) {
          u8 *w = A.arena + off;
          const int h = pad_header(w, false, true, dt, first + k, ts[k]);
          for (u32 i = 0; i < pl; i++) {
            u8 b;
            if (codec == LKF_CODEC_OPUS)
              b = i == 0 ? 0xf8 : i == 1 ? 0xff : i == 2 ? 0xfe : 0;
            else if (codec == LKF_CODEC_H264)
              b = kH264Blank[i];
            else
              b = i < u32(vl) ? u8(vd >> (8 * i)) : kVP8KeyFrame8x8[i - u32(vl)];
            w[h + i] = b;
          }
          for (u32 i = len; i < ((len + 15) & ~15u); i++) w[i] = 0;
          pad_record(A, r, k, d, off, len, first + k, ts[k], true);
        }
        off += (len + 15) & ~15u;
        nBytes += 12 + pl;  // sendingPacket: hdr.MarshalSize() + len(payload) (downtrack.go:1931-1939)
      }
      nPk = num;
      if (lane == 0) {
        A.dtCum[d].packets += num;
        A.dtCum[d].bytes += nBytes;
      }
    }
  }
  __syncthreads();
  reinterpret_cast<u32 *>(A.hot + d)[lane] = reinterpret_cast<const u32 *>(&sHot)[lane];
  if (lane == 0) {
    A.cnt[r] = nPk;
    A.bytes[r] = nBytes;
  }
}

hipError_t launch_pad(hipStream_t s, const PadLaunch &a) {
  if (!a.n) return hipSuccess;
  PadArgs A;
  A.blank = a.blank;
  A.n = a.n;
  A.reqs = a.reqs;
  A.nowNs = a.nowNs;
  A.hot = a.hot;
  A.dts = a.dts;
  A.tracks = a.tracks;
  A.rm = a.rm;
  A.seq = a.seq;
  A.seqSize = a.seqSize;
  A.srm = a.srm;
  A.srmStride = a.srmStride;
  A.srmCap = a.srmCap;
  A.dtCum = a.dtCum;
  A.recOff = a.recOff;
  A.byteOff = a.byteOff;
  A.out = a.out;
  A.arena = a.arena;
  A.cnt = a.cnt;
  A.bytes = a.bytes;
  hipLaunchKernelGGL(k_pad, dim3(a.n), dim3(64), 0, s, A);
  return hipGetLastError();
}

// per-batch counters -> cumulative (stats[3] := arena bytes from the out scan)
// stats[0..kStatWords) = sum of the kStatCopies partial copies that follow it
__global__ void __launch_bounds__(256) k_stats_reduce(u64 *stats) {
  const u32 i = threadIdx.x;
  if (i < u32(kStatWords)) {
    u64 v = 0;
    for (int c = 0; c < kStatCopies; c++) v += stats[size_t(1 + c) * kStatWords + i];
    stats[i] = v;
  }
}

__global__ void k_ev_offsets(const u32 *__restrict__ laneOf, const RunDesc *__restrict__ desc, u32 nl,
                             u32 *__restrict__ off) {
  const u32 l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l > nl) return;
  const u32 nev = desc->nev;
  u32 lo = 0, hi = nev;  // lower_bound(laneOf, l)
  while (lo < hi) {
    const u32 mid = (lo + hi) >> 1;
    if (laneOf[mid] < l)
      lo = mid + 1;
    else
      hi = mid;
  }
  off[l] = lo;
}

hipError_t launch_ev_offsets(hipStream_t s, const u32 *laneOf, const RunDesc *desc, u32 nl, u32 *off) {
  hipLaunchKernelGGL(k_ev_offsets, dim3((nl + 1 + 255) / 256), dim3(256), 0, s, laneOf, desc, nl, off);
  return hipGetLastError();
}

hipError_t launch_stats_reduce(hipStream_t s, u64 *stats) {
  hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(256), 0, s, stats);
  return hipGetLastError();
}

__global__ void k_accumulate(const u64 *stats, const u64 *tot, u64 *cum, const u32 *err, u32 *sticky) {
  const int i = threadIdx.x;
  if (i < 4 + LKF_DROP_NREASONS) cum[i] += (i == 3) ? tot[3] : stats[i];
  if (i == 0 && err[0]) sticky[0] |= err[0] & 0xffu;  // one lane: no race within the launch
}

// ORs an error word into the engine's sticky word (shifted), stream-ordered
// after the kernels that set it
__global__ void k_err_fold(const u32 *err, u32 *sticky, u32 shift) {
  if (threadIdx.x == 0 && err[0]) sticky[0] |= (err[0] & 0xffu) << shift;
}

hipError_t launch_err_fold(hipStream_t s, const u32 *err, u32 *sticky, u32 shift) {
  hipLaunchKernelGGL(k_err_fold, dim3(1), dim3(64), 0, s, err, sticky, shift);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_dd_decode: the dependency descriptor of every LKF_PKT_DD packet, read from
// its extension bytes with the track's current FrameDependencyStructure (as
// the Go parser did at ingress, dependencydescriptorparser.go:86-97), into one
// DDPkt per packet for k_decide_dt.  A structure attached to a packet goes to
// the next slot of the track's ring and becomes current.  One wave per track
// (see the kernel); runs on the prep stream, so batch n+1's decode follows
// batch n's.
// ---------------------------------------------------------------------------
// StreamTrackerDependencyDescriptor.Observe (streamtracker_dd.go:133-212) of one
// packet, serial in the track's lane
__device__ void dd_tracker_observe(DDTrkState &T, const DDStruct &S, const DDPkt &o, u32 ddFlags, u32 pktSize,
                                   u32 payload) {
  if ((T.flags & (DT_PAUSED | DT_STOPPED)) || payload == 0) return;
  if ((o.flags & DP_ACTIVE) && (ddFlags & LKF_DD_ACTIVE_UPDATED)) {
    i32 ms = 0, mt = 0;
    for (u32 k = 0; k < S.numDT; k++)
      if (o.activeMask & (1u << S.dtTarget[k])) {
        ms = max(ms, i32(S.dtS[k]));
        mt = max(mt, i32(S.dtT[k]));
      }
    ms = min(ms, 2);
    mt = min(mt, 3);
    const i32 old = T.maxS;
    T.maxS = ms;
    T.maxT = mt;
    if (old == -1) T.flags |= DT_WORKER;  // go s.worker(generation)
    const i32 lo = old > ms ? ms + 1 : old + 1, hi = old > ms ? old : ms;
    for (i32 l = lo; l <= hi && old != ms; l++) {
      T.notif[l]++;
      T.lastNotified[l] = old > ms ? 0 : 1;  // StreamStatusStopped / Active
    }
  }
  for (u32 k = 0; k < S.numDT; k++) {
    const u32 tg = S.dtTarget[k];
    if (o.ndti <= tg || ((o.dtis >> (2 * tg)) & 3) == 0) continue;  // DecodeTargetNotPresent
    T.bytes[S.dtS[k]][S.dtT[k]] += pktSize;
  }
}

// One wave per track, 64 packets at a time: the descriptors of a run of
// packets that attach no structure are read lane-parallel against the
// structure in force; a packet that attaches one is read alone (its structure
// goes to the ring's next slot and is in force from then on).  The DD stream
// tracker (order-dependent) folds the chunk's packets on lane 0 in order.
__global__ void __launch_bounds__(64) k_dd_decode(const RunDesc *__restrict__ desc, const u32 *__restrict__ tBegin,
                                                  const u32 *__restrict__ tEnd, const DevTrack *__restrict__ tracks,
                                                  u32 ntracks, DDStruct *structs, DDTrack *ddTracks,
                                                  DDPkt *__restrict__ out, u32 *err,
                                                  const u32 *__restrict__ trackDDTrk, DDTrkState *ddTrk, u16 *spill,
                                                  u32 *spillUsed, u32 spillCap) {
  const lkf_pkt *__restrict__ pkts = reinterpret_cast<const lkf_pkt *>(desc->pkts);
  const lkf_pkt_dd *__restrict__ dds = reinterpret_cast<const lkf_pkt_dd *>(desc->dd);
  const u8 *__restrict__ arena = reinterpret_cast<const u8 *>(desc->arena);
  const u32 t = blockIdx.x, lane = threadIdx.x;
  if (t >= ntracks) return;
  const u32 ddIdx = tracks[t].ddIdx;
  if (ddIdx == 0xffffffffu) return;
  DDTrack st = ddTracks[ddIdx];  // (wave-uniform)
  DDStruct *ring = structs + size_t(ddIdx) * kDDSlots;
  u32 updates = 0;
  bool bad = false;  // per lane
  const u32 pb = tBegin[t], pe = tEnd[t];
  const u32 trk = trackDDTrk ? trackDDTrk[t] : 0xffffffffu;
  for (u32 j = pb; j < pe; j += 64) {
    const u32 i = j + lane;
    bool isDD = false;
    u32 aoff = 0, psize = 0, pay = 0;
    if (i < pe) {
      const lkf_pkt &pk = pkts[i];
      isDD = pk.flags & LKF_PKT_DD;
      aoff = pk.arena_off;
      psize = u32(pk.payload_off) + pk.payload_len;
      pay = pk.payload_len;
    }
    lkf_pkt_dd r = {};
    if (isDD && dds) r = dds[i];
    // template_dependency_structure_present_flag (the first extended-field bit)
    const bool attL = isDD && dds && r.dd_len > 3 && (arena[u64(aoff) + r.dd_off + 3] & 0x80);
    DDPkt o = {};
    u64 pend = __ballot(isDD);
    while (pend) {
      const u64 attM = __ballot(attL) & pend;
      const u32 a = attM ? u32(__ffsll(static_cast<long long>(attM)) - 1) : 64u;
      const u64 runM = pend & (a < 64 ? ((1ull << a) - 1) : ~0ull);  // decoded together
      const u32 cur = st.cur, next = st.valid ? (st.cur + 1) % kDDSlots : 0u;
      const DDStruct *curS = st.valid ? ring + cur : nullptr;
      bool attOK = false;
      if (((runM >> lane) & 1) || lane == a) {
        if (!dds) {  // LKF_PKT_DD packets without their lkf_pkt_dd side array
          bad = true;
        } else {
          o.extFN = r.ext_frame_num;
          o.extKFN = r.ext_key_frame_num;
          o.extFlags = r.flags;
          bool att = false;
          const int e =
              r.dd_len ? dd::dd_parse(arena + aoff + r.dd_off, r.dd_len, curS, ring + next, o, att, spill, spillUsed,
                                      spillCap)
                       : int(dd::INVALID);
          if (e) {
            bad = true;
            o.flags = 0;
          } else {
            attOK = att;
            if (att && LKF_DD_SER) dd::ser_structure(ring[next]);  // (the attaching packet's lane only)
            o.slot = u8(att ? next : cur);
            o.flags |= DP_VALID;
          }
        }
      }
      if (a < 64) {  // the attaching packet's structure is in force from here on
        if (__builtin_amdgcn_readlane(int(attOK), a)) {
          st.cur = next;
          st.valid = 1;
          updates++;
        }
        pend &= ~((2ull << a) - 1);
      } else {
        pend = 0;
      }
    }
    if (isDD) out[i] = o;
    if (trk != 0xffffffffu) {  // StreamTrackerDependencyDescriptor.Observe in packet order
      const u64 vM = __ballot(isDD && (o.flags & DP_VALID));
      const u32 w0 = u32(o.flags) | (u32(o.slot) << 8) | (u32(o.ndti) << 16) | (u32(r.flags) << 24);
      for (u64 w = vM; w; w &= w - 1) {  // (whole wave: every lane's operands exist)
        const u32 x = u32(__ffsll(static_cast<long long>(w)) - 1);
        const u32 fx = u32(__builtin_amdgcn_readlane(int(w0), x));
        const u32 amx = u32(__builtin_amdgcn_readlane(int(o.activeMask), x));
        const u64 dtx = (u64(u32(__builtin_amdgcn_readlane(int(u32(o.dtis >> 32)), x))) << 32) |
                        u32(__builtin_amdgcn_readlane(int(u32(o.dtis)), x));
        const u32 szx = u32(__builtin_amdgcn_readlane(int(psize), x));
        const u32 pyx = u32(__builtin_amdgcn_readlane(int(pay), x));
        if (lane == 0) {
          DDPkt q = {};
          q.flags = u8(fx);
          q.slot = u8(fx >> 8);
          q.ndti = u8(fx >> 16);
          q.activeMask = amx;
          q.dtis = dtx;
          dd_tracker_observe(ddTrk[trk], ring[q.slot], q, fx >> 24, szx, pyx);
        }
      }
    }
  }
  // batch n+1's decode may run while batch n decides: a ring slot is reused
  // only after kDDSlots structures, so at most half of them per batch
  if (updates > u32(kDDSlots / 2)) bad = true;
  if (__ballot(bad) && lane == 0) atomicOr(err, 16u);
  if (lane == 0) ddTracks[ddIdx] = st;
}

hipError_t launch_dd_decode(hipStream_t s, const RunDesc *desc, const uint32_t *tBegin, const uint32_t *tEnd,
                            const DevTrack *tracks, uint32_t ntracks, DDStruct *structs, DDTrack *ddTracks, DDPkt *out,
                            uint32_t *err, const uint32_t *trackDDTrk, DDTrkState *ddTrk, uint16_t *spill,
                            uint32_t *spillUsed, uint32_t spillCap) {
  if (!ntracks) return hipSuccess;
  hipLaunchKernelGGL(k_dd_decode, dim3(ntracks), dim3(64), 0, s, desc, tBegin, tEnd, tracks, ntracks, structs,
                     ddTracks, out, err, trackDDTrk, ddTrk, spill, spillUsed, spillCap);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launch wrappers (kernels.h)
// ---------------------------------------------------------------------------
static u32 nblk(u64 n, u32 t) { return u32((n + t - 1) / t); }

hipError_t read_svc_stats(unsigned long long out[48], int reset) {
#if LKF_SVC_STATS
  static unsigned long long v[64 * 48];
  hipError_t r = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_svc), sizeof(v));
  for (int k = 0; k < 48; k++) {
    out[k] = 0;
    for (int c = 0; c < 64; c++) out[k] += v[c * 48 + k];
  }
  if (r == hipSuccess && reset) {
    for (auto &x : v) x = 0;
    r = hipMemcpyToSymbol(HIP_SYMBOL(g_svc), v, sizeof(v));
  }
  return r;
#else
  for (int i = 0; i < 48; i++) out[i] = 0;
  (void)reset;
  return hipErrorNotSupported;
#endif
}

hipError_t read_check(unsigned long long out[4], int reset) {
#if LKF_CHECKED
  hipError_t r = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chk), sizeof(unsigned long long) * 4);
  if (r == hipSuccess && reset) {
    unsigned long long z[4] = {};
    r = hipMemcpyToSymbol(HIP_SYMBOL(g_chk), z, sizeof(z));
  }
  return r;
#else
  (void)reset;
  for (int i = 0; i < 4; i++) out[i] = 0;
  return hipErrorNotSupported;
#endif
}

hipError_t launch_batch_init(hipStream_t s, u32 ntracks, u32 ndts, u32 nstats, u32 *tBegin, u32 *tEnd, u32 *tRuns,
                             u32 *err, u64 *stats, u32 *fwdCnt, u64 *fwdBytes) {
  u32 n = ntracks > ndts ? ntracks : ndts;
  if (n < nstats) n = nstats;
  u32 g = nblk(n, 256);
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_batch_init, dim3(g), dim3(256), 0, s, ntracks, ndts, nstats, tBegin, tEnd, tRuns, err, stats,
                     fwdCnt, fwdBytes);
  return hipGetLastError();
}

hipError_t launch_track_ranges(hipStream_t s, const RunDesc *desc, u32 maxPkts, u32 ntracks, u32 *tBegin, u32 *tEnd,
                               u32 *tRuns, u32 *err) {
  // grid for the engine's batch capacity (the same launch every run: the
  // batch length is in the descriptor)
  if (maxPkts == 0) return hipSuccess;
  hipLaunchKernelGGL(k_track_ranges, dim3(nblk(maxPkts, 256)), dim3(256), 0, s, desc, ntracks, tBegin, tEnd, tRuns,
                     err);
  return hipGetLastError();
}

hipError_t launch_scan(hipStream_t s, int mode, const DevDT *dts, const u32 *tBegin, const u32 *tEnd, const u32 *cnt,
                       const u64 *bytes, u32 n, u64 *partA, u64 *partB, u64 *outA, u64 *outB, u64 *totA, u64 *totB,
                       const u32 *perm, u32 *gFirst, u64 gCap) {
  (void)partB;
  ScanIn in;
  in.gFirst = gFirst;
  in.gCap = gCap;
  in.mode = mode;
  in.perm = perm;
  in.dts = dts;
  in.tBegin = tBegin;
  in.tEnd = tEnd;
  in.cnt = cnt;
  in.bytes = bytes;
  const u32 nb = nblk(n ? n : 1, SCAN_TILE);
  hipLaunchKernelGGL(k_scan_1p, dim3(nb), dim3(SCAN_T), 0, s, in, n, nb, partA, outA, outB, totA, totB);
  return hipGetLastError();
}

size_t scan_state_words(uint32_t maxN) { return kScanStHead + 8 * size_t(nblk(maxN ? maxN : 1, SCAN_TILE)); }

hipError_t launch_decide(hipStream_t s, const DecideLaunch &a) {
  if (a.nlanes == 0) return hipSuccess;
  DecideArgs A;
  A.sched = a.sched;
  A.waveTrack = a.waveTrack;
  A.nlanes = a.nlanes;
  A.hot = a.hot;
  A.dts = a.dts;
  A.tracks = a.tracks;
  A.rm = a.rm;
  A.vc = a.vc;
  A.seq = a.seq;
  A.seqSize = a.seqSize;
  A.srm = a.srm;
  A.srmStride = a.srmStride;
  A.srmCap = a.srmCap;
  A.pkts = a.pkts;
  A.tBegin = a.tBegin;
  A.tEnd = a.tEnd;
  A.slotBase = a.slotBase;
  A.recs = a.recs;
  A.fbase = a.fbase;
  A.wide = a.wide;
  A.tupleCap = a.tupleCap;
  A.err = a.err;
  A.ss = a.ss;
  A.ssRing = a.ssRing;
  A.ssGap = a.ssGap;
  A.dtOffs = a.dtOffs;
  A.events = a.events;
  A.evOff = a.evOff;
  A.fwdCnt = a.fwdCnt;
  A.layerList = a.layerList;
  A.layerBefore = a.layerBefore;
  A.layerCnt = a.layerCnt;
  A.pktStride = a.pktStride;
  A.fwdBytes = a.fwdBytes;
  A.dtCum = a.dtCum;
  A.stats = a.stats;
  A.ddPkts = a.ddPkts;
  A.ddStructs = a.ddStructs;
  A.ddState = a.ddState;
  A.ddArena = a.ddArena;
  A.ddUsed = a.ddUsed;
  A.ddSpill = a.ddSpill;
  A.ddCap = a.ddCap;
  A.maxDts = a.maxDts;
  A.maxTracks = a.maxTracks;
  A.npkts = a.npkts;
  A.nev = a.nev;
  // DownTracks of the dependency-descriptor selector run in their own
  // instantiation (the last ddLanes waves of the schedule)
  // Each part is a multiple of 8 slots (per-XCD lists of equal length);
  // a workgroup takes perWave consecutive slots of one XCD's list.
  const u32 nPlain = a.nlanes - a.ddLanes;
  const u32 K = a.perWave ? (a.perWave < kDecideMaxK ? a.perWave : kDecideMaxK) : 1;
  A.perWave = K;
  auto blocks = [K](u32 lanes) { return (lanes / 8 + K - 1) / K * 8; };
  A.waveBase = 0;
  A.waveEnd = nPlain;
  if (nPlain) hipLaunchKernelGGL(k_decide_dt<false>, dim3(blocks(nPlain)), dim3(64), 0, s, A, a.pkts);
  A.waveBase = nPlain;
  A.waveEnd = a.nlanes;
  if (a.ddLanes) hipLaunchKernelGGL(k_decide_dt<true>, dim3(blocks(a.ddLanes)), dim3(64), 0, s, A, a.pkts);
  return hipGetLastError();
}

hipError_t launch_layer_index(hipStream_t s, const RunDesc *desc, const u32 *tBegin, const u32 *tEnd, u32 ntracks,
                              u32 stride, u32 *list, u32 *before, u32 *cnt, u64 *zero2) {
  if (!ntracks) return hipSuccess;
  hipLaunchKernelGGL(k_layer_index, dim3(ntracks), dim3(64), 0, s, desc, tBegin, tEnd, stride, list, before, cnt,
                     zero2);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Transport-wide sequence numbers (pion/interceptor v0.1.25 pkg/twcc
// HeaderExtensionInterceptor, added per subscriber PeerConnection with
// send-side BWE, pkg/rtc/transport.go:352-355): every RTP packet a
// PeerConnection writes on a stream that negotiated transport-cc gets
// uint16(n) of the PeerConnection's counter n (atomic.AddUint32 - 1) as a
// 2-byte extension element, in send order.  A batch's send order is its
// record order (track, DownTrack, packet): a transport's DownTracks take
// consecutive ranges in that order (k_twcc_base, after decide), the records
// their base plus their ordinal (k_emit); padding, blank frames and RTX are
// stamped in call order (k_twcc_stamp).
// ---------------------------------------------------------------------------
__global__ void k_twcc_base(const DevDT *__restrict__ dts, u32 ndts, const u32 *__restrict__ fwdCnt,
                            u32 *__restrict__ ctrD, u32 *__restrict__ ctrT, const u32 *__restrict__ tOff,
                            const u32 *__restrict__ tList, u32 ntr, u32 *__restrict__ base) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < ndts) {  // a DownTrack counting on its own (no transport bound)
    const DevDT dt = dts[i];
    if (dt.extTcc && !(dt.twccGroup & 0x80000000u)) {
      base[i] = ctrD[i];
      ctrD[i] += fwdCnt[i];
    }
  } else if (i - ndts < ntr) {  // a transport: its DownTracks in record order
    const u32 t = i - ndts;
    u32 c = ctrT[t];
    for (u32 k = tOff[t]; k < tOff[t + 1]; k++) {
      const u32 d = tList[k];
      base[d] = c;
      c += fwdCnt[d];
    }
    ctrT[t] = c;
  }
}
hipError_t launch_twcc_base(hipStream_t s, const DevDT *dts, uint32_t ndts, const uint32_t *fwdCnt, uint32_t *ctrD,
                            uint32_t *ctrT, const uint32_t *tOff, const uint32_t *tList, uint32_t ntr,
                            uint32_t *base) {
  const u32 n = ndts + ntr;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_twcc_base, dim3((n + 255) / 256), dim3(256), 0, s, dts, ndts, fwdCnt, ctrD, ctrT, tOff, tList,
                     ntr, base);
  return hipGetLastError();
}

// the 2-byte element with extension id `id` (RFC 8285 one- or two-byte block) <- seq
__device__ void twcc_put(u8 *pkt, u32 len, u8 id, u16 seq) {
  if (len < 12 || !(pkt[0] & 0x10)) return;
  u32 n = 12 + 4 * (pkt[0] & 15);
  if (n + 4 > len) return;
  const u32 prof = (u32(pkt[n]) << 8) | pkt[n + 1];
  const u32 end = n + 4 + 4 * ((u32(pkt[n + 2]) << 8) | pkt[n + 3]);
  n += 4;
  while (n < end && end <= len) {
    if (pkt[n] == 0) {
      n++;
      continue;
    }
    u8 eid;
    u32 el;
    if (prof == 0xBEDE) {
      eid = pkt[n] >> 4;
      el = (pkt[n] & 15) + 1;
      n++;
      if (eid == 15) return;
    } else {
      eid = pkt[n];
      el = pkt[n + 1];
      n += 2;
    }
    if (eid == id && el == 2 && n + 2 <= len) {
      pkt[n] = u8(seq >> 8);
      pkt[n + 1] = u8(seq);
      return;
    }
    n += el;
  }
}

// Control-rate packets in send order (one thread: a few packets per call).
// pad mode: requests r < n, packets k < cnt[r] at records recOff[r] + k;
// rtx mode: records r < n with len[r] > 0 at off[r], DownTrack rtx[r].dt.
__global__ void k_twcc_stamp(const DevDT *__restrict__ dts, u32 *ctrD, u32 *ctrT, u32 n, const lkf_out *recs,
                             const u64 *recOff, const u32 *cnt, const lkf_rtx *rtx, const u64 *off, const u32 *len,
                             u8 *arena) {
  if (threadIdx.x || blockIdx.x) return;
  auto next = [&](u32 d) -> u16 {
    const DevDT dt = dts[d];
    u32 &c = (dt.twccGroup & 0x80000000u) ? ctrT[dt.twccGroup & 0x7fffffffu] : ctrD[d];
    return u16(c++);
  };
  for (u32 r = 0; r < n; r++) {
    if (recs) {
      for (u32 k = 0; k < cnt[r]; k++) {
        const lkf_out &o = recs[recOff[r] + k];
        const u8 id = dts[o.dt].extTcc;
        if (id) twcc_put(arena + o.out_off, o.out_len, id, next(o.dt));
      }
    } else if (len[r]) {
      const u32 d = u32(rtx[r].dt);
      const u8 id = dts[d].extTcc;
      if (id) twcc_put(arena + off[r], len[r], id, next(d));
    }
  }
}
hipError_t launch_twcc_stamp(hipStream_t s, const DevDT *dts, uint32_t *ctrD, uint32_t *ctrT, uint32_t n,
                             const lkf_out *recs, const uint64_t *recOff, const uint32_t *cnt, const lkf_rtx *rtx,
                             const uint64_t *off, const uint32_t *len, uint8_t *arena) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_twcc_stamp, dim3(1), dim3(64), 0, s, dts, ctrD, ctrT, n, recs, recOff, cnt, rtx, off, len,
                     arena);
  return hipGetLastError();
}

hipError_t launch_emit(hipStream_t s, const EmitLaunch &a) {
  EmitArgs A;
  A.perm = a.perm;
  A.recBase = a.recBase;
  A.byteBase = a.byteBase;
  A.gFirst = a.gFirst;
  A.slotBase = a.slotBase;
  A.totals = a.totals;
  A.recs = a.recs;
  A.fbase = a.fbase;
  A.wide = a.wide;
  A.pkts = a.pkts;
  A.arena = a.arena;
  A.dts = a.dts;
  A.ndts = a.ndts;
  A.out = a.out;
  A.outArena = a.outArena;
  A.outCap = a.outCap;
  A.outByteCap = a.outByteCap;
  A.err = a.err;
  A.ddArena = a.ddArena;
  A.twccBase = a.twccBase;
  A.maxDts = a.maxDts;
  A.npkts = a.npkts;
  A.tupleCap = a.tupleCap;
  A.arenaLen = a.arenaLen;
  A.ddCap = a.ddCap;
  A.gCap = a.gCap;
  if (a.ddArena)
    hipLaunchKernelGGL(k_emit<PRE_MAX_DD>, dim3(a.grid), dim3(EMIT_T), 0, s, A);
  else
    hipLaunchKernelGGL(k_emit<PRE_MAX>, dim3(a.grid), dim3(EMIT_T), a.ldsPad, s, A);
  return hipGetLastError();
}

// The run's first kernel: pulls the page-locked staging buffer (the host's
// RunDesc, then the control ops and their lanes) into device memory through
// the device mapping.  Sizes come from the staged descriptor, so the launch
// is the same every run (grid-stride).
__global__ void k_h2d(const u8 *__restrict__ stage, RunDesc *__restrict__ dDesc, DevEvent *__restrict__ dEv,
                      u32 *__restrict__ dLane) {
  const RunDesc *h = reinterpret_cast<const RunDesc *>(stage);
  const u32 nev = h->nev, cap = h->evCap;
  const u64 nA = u64(nev) * (sizeof(DevEvent) / 4), nB = nev;
  const u32 *sA = reinterpret_cast<const u32 *>(stage + sizeof(RunDesc));
  const u32 *sB = reinterpret_cast<const u32 *>(stage + sizeof(RunDesc) + u64(cap) * sizeof(DevEvent));
  u32 *dA = reinterpret_cast<u32 *>(dEv);
  const u64 stride = u64(gridDim.x) * blockDim.x;
  const u64 t = u64(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t < sizeof(RunDesc) / 4) reinterpret_cast<u32 *>(dDesc)[t] = reinterpret_cast<const u32 *>(h)[t];
  for (u64 i = t; i < nA + nB; i += stride) {
    if (i < nA)
      dA[i] = sA[i];
    else
      dLane[i - nA] = sB[i - nA];
  }
}

hipError_t launch_h2d(hipStream_t s, const uint8_t *stage, RunDesc *dDesc, DevEvent *dEv, uint32_t *dLane) {
  hipLaunchKernelGGL(k_h2d, dim3(256), dim3(256), 0, s, stage, dDesc, dEv, dLane);
  return hipGetLastError();
}

hipError_t launch_accumulate(hipStream_t s, const u64 *stats, const u64 *tot, u64 *cum, const u32 *err, u32 *sticky) {
  hipLaunchKernelGGL(k_accumulate, dim3(1), dim3(64), 0, s, stats, tot, cum, err, sticky);
  return hipGetLastError();
}

hipError_t launch_seq_lookup(hipStream_t s, DTHot *hot, SeqMeta *seq, u32 seqSize, u8 *srm, u64 srmStride, u32 srmCap,
                             u32 d, const u16 *sns, u32 n, i64 nowMs, lkf_seq_meta *out, u32 *nOut) {
  hipLaunchKernelGGL(k_seq_lookup, dim3(1), dim3(64), 0, s, hot, seq, seqSize, srm, srmStride, srmCap, d, sns, n, nowMs,
                     out, nOut);
  return hipGetLastError();
}

}  // namespace lkf
