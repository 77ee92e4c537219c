// =============================================================================
//  dd_select_oracle.h — TEST INFRASTRUCTURE ONLY (CPU restatement, not shipped).
//
//  The dependency-descriptor half of SVC forwarding (§8(a) rows a9 and a16):
//    pkg/sfu/videolayerselector/selectordecisioncache.go  SelectorDecisionCache
//    pkg/sfu/videolayerselector/framechain.go             FrameChain
//    pkg/sfu/videolayerselector/decodetarget.go           DecodeTarget
//    pkg/sfu/videolayerselector/dependencydescriptor.go   DependencyDescriptor
//        (Select :65-355, Rollback :357, updateDependencyStructure :363,
//         updateActiveDecodeTargets :394, invalidateKeyFrame :410, CheckSync :418)
//    pkg/sfu/buffer/dependencydescriptorparser.go         DependencyDescriptorParser.Parse
//        :75-163, ProcessFrameDependencyStructure :178-201,
//        GetActiveDecodeTargetBitmask :203-212
//    pkg/sfu/buffer/frameintegrity.go                     FrameIntegrityChecker,
//        PacketHistory, FrameEntity
//  Included by lkf_oracle.h (namespace orc), after VideoLayer and WrapAround.
//  Pinned by oracle/kat_ddsel.inc: videolayerselector/dependencydescriptor_test.go
//  (TestDecodeTarget, TestFrameChain, TestDependencyDescriptor) and
//  buffer/frameintegrity_test.go (TestFrameIntegrityChecker).
// =============================================================================
#pragma once
#include <map>
#include <memory>

#include "dd_oracle.h"

namespace orc {

// ---- selectordecisioncache.go ----------------------------------------------
enum SelectorDecision : int { SDMissing = 0, SDDropped = 1, SDForwarded = 2, SDUnknown = 3 };

struct FrameChain;

struct SelectorDecisionCache {
  bool initialized = false;
  u64 base = 0, last = 0;
  std::vector<u64> masks;
  u64 numEntries = 0, numNackEntries = 0;
  // onExpectEntityChanged: the only callback registered on the hot path is
  // FrameChain.OnExpectFrameChanged (framechain.go:81)
  std::map<u64, std::vector<std::shared_ptr<FrameChain>>> onExpect;

  SelectorDecisionCache(u64 maxNumElements, u64 nack) {  // :60-68
    const u64 numElements = (maxNumElements * 2 + 63) / 64;
    masks.assign(numElements, 0);
    numEntries = numElements * 32;
    numNackEntries = nack;
  }
  void AddForwarded(u64 e) { addEntity(e, SDForwarded); }
  void AddDropped(u64 e) { addEntity(e, SDDropped); }
  // GetDecision :78-94 (err: "too old")
  SelectorDecision GetDecision(u64 e, bool *err = nullptr) const {
    if (err) *err = false;
    if (!initialized || e < base) return SDMissing;
    if (e > last) return SDUnknown;
    if (last - e >= numEntries) {
      if (err) *err = true;
      return SDMissing;
    }
    return getEntity(e);
  }
  // ExpectDecision :96-110
  bool ExpectDecision(u64 e, const std::shared_ptr<FrameChain> &fc) {
    if (!initialized || e < base) return false;
    if (e < last && last - e >= numEntries) return false;
    onExpect[e].push_back(fc);
    return true;
  }
  void addEntity(u64 entity, SelectorDecision sd);  // :112-165 (below FrameChain)
  void setEntityIfUnknown(u64 e, SelectorDecision sd) {
    if (getEntity(e) == SDUnknown) setEntity(e, sd);
  }
  void setEntity(u64 e, SelectorDecision sd);  // :173-186
  SelectorDecision getEntity(u64 e) const {
    u64 off = (e - base) % numEntries;
    return SelectorDecision((masks[off >> 5] >> ((off & 0x1f) * 2)) & 3);
  }
};

// ---- framechain.go -----------------------------------------------------------
struct FrameChain : std::enable_shared_from_this<FrameChain> {
  SelectorDecisionCache *decisions;
  bool broken = true;
  int chainIdx;
  bool active = false;
  bool updatingActive = false;
  std::vector<u64> expectFrames;

  FrameChain(SelectorDecisionCache *d, int idx) : decisions(d), chainIdx(idx) {}

  // OnFrame :43-92
  bool OnFrame(u64 extFrameNum, const orc_dd::Template &fd) {
    if (!active) return false;
    if (int(fd.ChainDiffs.size()) <= chainIdx) return broken;
    if (fd.ChainDiffs[chainIdx] == 0) {
      broken = false;
      expectFrames.clear();
      return true;
    }
    if (broken) return false;
    const u64 prev = extFrameNum - u64(fd.ChainDiffs[chainIdx]);
    const SelectorDecision sd = decisions->GetDecision(prev);
    bool intact = false;
    if (sd == SDForwarded) {
      intact = true;
    } else if (sd == SDUnknown) {
      if (decisions->ExpectDecision(prev, shared_from_this())) {
        intact = true;
        expectFrames.push_back(prev);
      }
    }
    if (!intact) broken = true;
    return intact;
  }
  // OnExpectFrameChanged :94-110
  void OnExpectFrameChanged(u64 frameNum, SelectorDecision d) {
    if (broken) return;
    for (size_t i = 0; i < expectFrames.size(); i++) {
      if (expectFrames[i] == frameNum) {
        if (d != SDForwarded) broken = true;
        expectFrames[i] = expectFrames.back();
        expectFrames.pop_back();
        break;
      }
    }
  }
  bool Broken() const { return broken; }
  void BeginUpdateActive() { updatingActive = false; }
  void UpdateActive(bool a) { updatingActive = updatingActive || a; }
  void EndUpdateActive() {  // :124-138
    const bool a = updatingActive;
    updatingActive = false;
    if (a == active) return;
    if (!active) broken = true;
    active = a;
  }
};

inline void SelectorDecisionCache::setEntity(u64 e, SelectorDecision sd) {
  const u64 off = (e - base) % numEntries;
  u64 &m = masks[off >> 5];
  const int bp = int(off & 0x1f) * 2;
  m &= ~(u64(3) << bp);
  m |= (u64(sd) & 3) << bp;
  if (sd != SDUnknown) {
    auto it = onExpect.find(e);
    if (it != onExpect.end()) {
      auto fns = std::move(it->second);
      onExpect.erase(it);
      for (auto &f : fns) f->OnExpectFrameChanged(e, sd);
    }
  }
}

inline void SelectorDecisionCache::addEntity(u64 entity, SelectorDecision sd) {
  if (!initialized) {
    initialized = true;
    base = entity;
    last = entity;
    setEntity(entity, sd);
    return;
  }
  if (entity <= base) return;
  if (entity <= last) {
    setEntity(entity, sd);
    return;
  }
  for (u64 e = last + 1; e != entity; e++) setEntity(e, SDUnknown);
  u64 missingStart = last;
  if (missingStart > numNackEntries + base)
    missingStart -= numNackEntries;
  else
    missingStart = base;
  u64 missingEnd = entity;
  if (missingEnd > numNackEntries + base)
    missingEnd -= numNackEntries;
  else
    missingEnd = base;
  if (missingEnd > missingStart)
    for (u64 e = missingStart; e != missingEnd; e++) setEntityIfUnknown(e, SDMissing);
  setEntity(entity, sd);
  last = entity;
  // Go ranges over the map in random order; the callbacks only set `broken`
  // and drop a frame from a not-yet-broken chain, so the order cannot change
  // any later decision (a broken chain only recovers through a clearing frame)
  for (auto it = onExpect.begin(); it != onExpect.end();) {
    if (it->first + numEntries < last) {
      const u64 e = it->first;
      auto fns = std::move(it->second);
      it = onExpect.erase(it);
      for (auto &f : fns) f->OnExpectFrameChanged(e, SDMissing);
    } else {
      ++it;
    }
  }
}

// ---- buffer.DependencyDescriptorDecodeTarget / decodetarget.go ----------------
struct DDDecodeTarget {  // buffer/dependencydescriptorparser.go:167-170
  int Target = 0;
  VideoLayer Layer;
};

struct DecodeTarget {
  DDDecodeTarget dt;
  std::shared_ptr<FrameChain> chain;
  bool active = false;
  bool Valid() const { return !chain || !chain->Broken(); }
  bool Active() const { return active; }
  void UpdateActive(u32 mask) {  // :50-56
    active = (mask & (1u << dt.Target)) != 0;
    if (chain) chain->UpdateActive(active);
  }
  // OnFrame :58-70 -> false on error
  bool OnFrame(u64, const orc_dd::Template &fd, bool &targetValid, int &dti) const {
    targetValid = false;
    dti = 0;
    if (int(fd.DTIs.size()) <= dt.Target) return false;
    dti = fd.DTIs[dt.Target];
    targetValid = Valid();
    return true;
  }
};

// ProcessFrameDependencyStructure dependencydescriptorparser.go:178-201.
// sort.Slice with GreaterThan: Go's pdqsort runs insertion sort below 12
// elements (stable); larger structures only differ on tied layers.
inline std::vector<DDDecodeTarget> ProcessFrameDependencyStructure(const orc_dd::Structure &s) {
  std::vector<DDDecodeTarget> v;
  for (int t = 0; t < s.NumDecodeTargets; t++) {
    DDDecodeTarget d;
    d.Target = t;
    d.Layer = VideoLayer{0, 0};
    for (auto &tp : s.Templates) {
      if (t < int(tp.DTIs.size()) && tp.DTIs[t] != 0) {
        if (d.Layer.Spatial < tp.SpatialId) d.Layer.Spatial = tp.SpatialId;
        if (d.Layer.Temporal < tp.TemporalId) d.Layer.Temporal = tp.TemporalId;
      }
    }
    v.push_back(d);
  }
  std::stable_sort(v.begin(), v.end(),
                   [](const DDDecodeTarget &a, const DDDecodeTarget &b) { return a.Layer.GreaterThan(b.Layer); });
  return v;
}
// GetActiveDecodeTargetBitmask :203-212
inline u32 GetActiveDecodeTargetBitmask(VideoLayer l, const std::vector<DDDecodeTarget> &dts) {
  u32 m = 0;
  for (auto &d : dts)
    if (d.Layer.Spatial <= l.Spatial && d.Layer.Temporal <= l.Temporal) m |= 1u << d.Target;
  return m;
}

// buffer.ExtDependencyDescriptor dependencydescriptorparser.go:63-73
struct ExtDD {
  std::shared_ptr<orc_dd::Descriptor> Descriptor;
  std::vector<DDDecodeTarget> DecodeTargets;
  bool StructureUpdated = false;
  bool ActiveDecodeTargetsUpdated = false;
  bool Integrity = false;
  u64 ExtFrameNum = 0;
  u64 ExtKeyFrameNum = 0;
};

// ---- videolayerselector.DependencyDescriptor (selector state; the Base
// layers live in the VLS that owns it) ----------------------------------------
struct DDSelectorState {
  SelectorDecisionCache decisions{256, 80};
  bool hasPrevMask = false, hasMask = false;  // *uint32 nil-ness
  u32 prevMask = 0, mask = 0;
  std::shared_ptr<orc_dd::Structure> structure;
  u64 extKeyFrameNum = 0;
  bool keyFrameValid = false;
  std::vector<std::shared_ptr<FrameChain>> chains;
  std::vector<DecodeTarget> decodeTargets;
  orc_dd::FrameNumberWrapper fnWrapper;

  // updateDependencyStructure :363-392
  void updateDependencyStructure(const std::shared_ptr<orc_dd::Structure> &s, const std::vector<DDDecodeTarget> &dts,
                                 u64 extFrameNum) {
    structure = s;
    extKeyFrameNum = extFrameNum;
    keyFrameValid = true;
    chains.clear();
    for (int c = 0; c < s->NumChains; c++) chains.push_back(std::make_shared<FrameChain>(&decisions, c));
    std::vector<DecodeTarget> nt;
    for (auto &d : dts) {
      DecodeTarget t;
      t.dt = d;
      if (s->NumChains > 0) {
        const int ci = s->DecodeTargetProtectedByChain[d.Target];
        if (ci < int(chains.size())) t.chain = chains[ci];
      }
      nt.push_back(t);
    }
    decodeTargets = nt;
  }
  // updateActiveDecodeTargets :394-408
  void updateActiveDecodeTargets(u32 m) {
    for (auto &c : chains) c->BeginUpdateActive();
    for (auto &d : decodeTargets) d.UpdateActive(m);
    for (auto &c : chains) c->EndUpdateActive();
  }
  // invalidateKeyFrame :410-416
  void invalidateKeyFrame() {
    keyFrameValid = false;
    chains.clear();
    decodeTargets.clear();
  }
};

// ---- buffer/frameintegrity.go -------------------------------------------------
struct PacketHistory {  // :46-146
  u64 base = 0, last = 0;
  std::vector<u64> bits;
  int packetCount;
  bool inited = false;
  explicit PacketHistory(int n) {
    packetCount = (n + 63) / 64 * 64;
    bits.assign(size_t(packetCount / 64), 0);
  }
  void AddPacket(u64 s) {
    if (!inited) {
      inited = true;
      base = s;
      if (base > 100)
        base -= 100;
      else
        base = 0;
      last = s;
      set(s, true);
      return;
    }
    if (s <= base) return;
    if (s <= last) {
      if (last - s < u64(packetCount)) set(s, true);
      return;
    }
    for (u64 i = last + 1; i < s; i++) set(i, false);
    set(s, true);
    last = s;
  }
  void pos(u64 s, int &idx, int &off) const {
    const u64 i = (s - base) % u64(packetCount);
    idx = int(i >> 6);
    off = int(i % 64);
  }
  void set(u64 s, bool r) {
    int idx, off;
    pos(s, idx, off);
    if (!r)
      bits[idx] &= ~(u64(1) << off);
    else
      bits[idx] |= u64(1) << off;
  }
  bool PacketsConsecutive(u64 start, u64 end) const {
    if (start > end) return false;
    if (end - start >= u64(packetCount)) return false;
    int si, so, ei, eo;
    pos(start, si, so);
    pos(end, ei, eo);
    if (si == ei && end - start <= 64) {
      // Go: (1<<(eo-so+1))-1 with a 64-bit shift of 64 yields 0 - 1 = all ones
      const int w = eo - so + 1;
      const u64 tb = (w >= 64 ? ~u64(0) : ((u64(1) << w) - 1)) << so;
      return (bits[si] & tb) == tb;
    }
    // Go: (bits >> so) + 1 != 1 << (64 - so)  (1 << 64 == 0 for a uint64)
    const u64 lhs = (bits[si] >> so) + 1;
    const u64 rhs = (64 - so) >= 64 ? 0 : (u64(1) << (64 - so));
    if (lhs != rhs) return false;
    for (int i = si + 1; i != ei; i++) {
      if (i == int(bits.size())) {
        i = 0;
        if (i == ei) break;
      }
      if (bits[i] + 1 != 0) return false;
    }
    const u64 tb = eo + 1 >= 64 ? ~u64(0) : ((u64(1) << (eo + 1)) - 1);
    return (bits[ei] & tb) == tb;
  }
};

struct FrameEntity {  // :7-42
  bool hasStart = false, hasEnd = false;
  u64 startSeq = 0, endSeq = 0;
  bool integrity = false;
  void AddPacket(u64 s, bool first, bool lastPkt, const PacketHistory &ph) {
    if (integrity) return;
    if (!hasStart && first) {
      hasStart = true;
      startSeq = s;
    }
    if (!hasEnd && lastPkt) {
      hasEnd = true;
      endSeq = s;
    }
    if (hasStart && hasEnd && ph.PacketsConsecutive(startSeq, endSeq)) integrity = true;
  }
  void Reset() {
    integrity = false;
    hasStart = hasEnd = false;
  }
};

struct FrameIntegrityChecker {  // :150-211
  int frameCount;
  std::vector<FrameEntity> frames;
  u64 base = 0, last = 0;
  PacketHistory ph;
  bool inited = false;
  FrameIntegrityChecker(int fc, int pc) : frameCount(fc), frames(size_t(fc)), ph(pc) {}
  void AddPacket(u64 extSeq, u64 extFN, bool first, bool lastPkt) {
    ph.AddPacket(extSeq);
    if (!inited) {
      inited = true;
      base = extFN;
      last = extFN;
    }
    if (extFN < base) return;
    if (extFN <= last) {
      if (last - extFN >= u64(frameCount)) return;
      frames[size_t((extFN - base) % u64(frameCount))].AddPacket(extSeq, first, lastPkt, ph);
      return;
    }
    for (u64 i = last + 1; i <= extFN; i++) frames[size_t((i - base) % u64(frameCount))].Reset();
    frames[size_t((extFN - base) % u64(frameCount))].AddPacket(extSeq, first, lastPkt, ph);
    last = extFN;
  }
  bool FrameIntegrity(u64 extFN) const {
    if (extFN < base || extFN > last || last - extFN >= u64(frameCount)) return false;
    return frames[size_t((extFN - base) % u64(frameCount))].integrity;
  }
};

// ---- buffer/dependencydescriptorparser.go -------------------------------------
enum DDParseErr : int { DDP_OK = 0, DDP_UNMARSHAL = 1, DDP_EARLIER_THAN_KEYFRAME = 2, DDP_STRUCTURE_NOT_FIRST = 3 };

struct DependencyDescriptorParser {
  std::shared_ptr<orc_dd::Structure> structure;
  std::vector<DDDecodeTarget> decodeTargets;
  WrapAround<u16, u64> seqWrapAround{false};
  WrapAround<u16, u64> frameWrapAround{false};
  u64 structureExtFrameNum = 0;
  u64 activeDecodeTargetsExtSeq = 0;
  u32 activeDecodeTargetsMask = 0;
  FrameIntegrityChecker frameChecker{180, 1024};

  // Parse :75-163 on the DD extension payload (ddBuf = pkt.GetExtension(id);
  // absent -> (nil, nil)).  Returns DDP_OK with out == nullptr when absent.
  DDParseErr Parse(const u8 *ddBuf, int ddLen, u16 sn, std::shared_ptr<ExtDD> &out, VideoLayer &vl) {
    out.reset();
    vl = VideoLayer{0, 0};  // var videoLayer VideoLayer (zero value)
    if (!ddBuf) return DDP_OK;
    auto dv = std::make_shared<orc_dd::Descriptor>();
    int nread = 0;
    if (orc_dd::Unmarshal(ddBuf, ddLen, structure.get(), *dv, nread) != orc_dd::DD_OK) return DDP_UNMARSHAL;
    const u64 extSeq = seqWrapAround.Update(sn).ExtendedVal;
    if (dv->hasDeps) vl = VideoLayer{dv->FrameDependencies.SpatialId, dv->FrameDependencies.TemporalId};
    const u64 extFN = frameWrapAround.Update(dv->FrameNumber).ExtendedVal;
    if (extFN < structureExtFrameNum) return DDP_EARLIER_THAN_KEYFRAME;
    frameChecker.AddPacket(extSeq, extFN, dv->FirstPacketInFrame, dv->LastPacketInFrame);
    auto e = std::make_shared<ExtDD>();
    e->Descriptor = dv;
    e->ExtFrameNum = extFN;
    e->Integrity = frameChecker.FrameIntegrity(extFN);
    if (dv->AttachedStructure) {
      if (!dv->FirstPacketInFrame) return DDP_STRUCTURE_NOT_FIRST;
      structure = dv->AttachedStructure;
      decodeTargets = ProcessFrameDependencyStructure(*structure);
      structureExtFrameNum = extFN;
      e->StructureUpdated = true;
      e->ActiveDecodeTargetsUpdated = true;
    }
    if (dv->hasActiveMask && extSeq > activeDecodeTargetsExtSeq) {
      activeDecodeTargetsExtSeq = extSeq;
      if (dv->ActiveDecodeTargetsBitmask != activeDecodeTargetsMask) {
        activeDecodeTargetsMask = dv->ActiveDecodeTargetsBitmask;
        e->ActiveDecodeTargetsUpdated = true;  // onMaxLayerChanged: frame-rate calculator only (out of scope)
      }
    }
    e->DecodeTargets = decodeTargets;
    e->ExtKeyFrameNum = structureExtFrameNum;
    out = e;
    return DDP_OK;
  }
};

}  // namespace orc
