// =============================================================================
//  dd_oracle.h — TEST INFRASTRUCTURE ONLY (CPU restatement, not shipped).
//
//  The AV1 dependency-descriptor RTP header extension (§8(a) row a9), as the
//  reference reads and writes it:
//    pkg/sfu/dependencydescriptor/bitstreamreader.go   BitStreamReader
//    pkg/sfu/dependencydescriptor/bitstreamwriter.go   BitStreamWriter
//    pkg/sfu/dependencydescriptor/dependencydescriptorreader.go  Parse
//    pkg/sfu/dependencydescriptor/dependencydescriptorwriter.go  Write /
//        findBestTemplate / calculateMatch / ValueSizeBits
//    pkg/sfu/dependencydescriptor/dependencydescriptorextension.go  types,
//        Marshal(WithActiveChains) / Unmarshal
//    pkg/sfu/videolayerselector/framenumberwrapper.go  FrameNumberWrapper
//  Pinned by oracle/kat_dd.inc: the 14 hex captures of
//  dependencydescriptorextension_test.go:25-41 (parse, plus the reader->writer
//  round trip SURVEY.md §8(c) asks for) and the properties of
//  framenumberwrapper_test.go.  The GPU side of a9 (selector, per-tuple
//  re-marshal) is the next step; this is its checker.
// =============================================================================
#pragma once
#include <cmath>
#include <cstdint>
#include <memory>
#include <vector>

namespace orc_dd {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;

constexpr int MaxSpatialIds = 4;
constexpr int MaxTemporalIds = 8;
constexpr int MaxDecodeTargets = 32;
constexpr int MaxTemplates = 64;

enum DDErr {
  DD_OK = 0,
  DD_EOF,
  DD_NO_STRUCTURE,
  DD_TEMPLATE_WITHOUT_STRUCTURE,
  DD_TOO_MANY_TEMPLATES,
  DD_TOO_MANY_TEMPORAL,
  DD_TOO_MANY_SPATIAL,
  DD_INVALID_TEMPLATE_INDEX,
  DD_INVALID_SPATIAL_LAYER,
  DD_DTI_MISMATCH,
  DD_CHAIN_MISMATCH,
  DD_NO_TEMPLATE,
  DD_INVALID,
  DD_NO_SPACE,
};

inline int bitwidth(u32 n) {
  int w = 0;
  while (n) {
    n >>= 1;
    w++;
  }
  return w;
}

// bitstreamreader.go
struct BitReader {
  const u8 *buf;
  int len, pos = 0, remaining;
  BitReader(const u8 *b, int n) : buf(b), len(n), remaining(n * 8) {}
  DDErr bits(int n, u64 &out) {
    out = 0;
    if (n < 0 || n > 64) return DD_INVALID;
    if (remaining < n) {
      remaining -= n;
      return DD_EOF;
    }
    int inFirst = remaining % 8;
    remaining -= n;
    if (n < inFirst) {
      out = u64((buf[pos] >> (inFirst - n)) & ((1u << n) - 1));
      return DD_OK;
    }
    u64 r = 0;
    if (inFirst > 0) {
      n -= inFirst;
      r = u64(buf[pos] & u8((1u << inFirst) - 1)) << n;
      pos++;
    }
    while (n >= 8) {
      n -= 8;
      r |= u64(buf[pos]) << n;
      pos++;
    }
    if (n > 0) r |= u64(buf[pos] >> (8 - n));
    out = r;
    return DD_OK;
  }
  DDErr flag(bool &b) {
    u64 v;
    DDErr e = bits(1, v);
    b = v != 0;
    return e;
  }
  bool ok() const { return remaining >= 0; }
  void invalidate() { remaining = -1; }
  // ReadNonSymmetric (av1 ns(n))
  DDErr nonSymmetric(u32 numValues, u32 &out) {
    out = 0;
    if (numValues >= (1u << 31)) return DD_INVALID;
    const int w = bitwidth(numValues);
    const u32 numMin = (1u << w) - numValues;
    u64 v;
    DDErr e = bits(w - 1, v);
    if (e) return e;
    if (v < numMin) {
      out = u32(v);
      return DD_OK;
    }
    u64 b;
    e = bits(1, b);
    if (e) return e;
    out = u32((v << 1) + b - numMin);
    return DD_OK;
  }
  int bytesRead() const { return remaining % 8 > 0 ? pos + 1 : pos; }
};

// bitstreamwriter.go
struct BitWriter {
  std::vector<u8> *buf;
  int pos = 0, bitOffset = 0;
  explicit BitWriter(std::vector<u8> *b) : buf(b) {}
  int remainingBits() const { return int(buf->size() - pos) * 8 - bitOffset; }
  static u8 partial(u8 src, int srcBits, u8 target, int targetOff) {
    const u8 mask = u8(u8(0xff << (8 - srcBits)) >> targetOff);
    return u8((target & ~mask) | (src >> targetOff));
  }
  DDErr write(u64 val, int n) {
    if (n > remainingBits()) return DD_NO_SPACE;
    const int total = n;
    if (n == 0) return consume(0);
    val <<= (64 - n);
    u8 *b = buf->data() + pos;
    const int inCur = 8 - bitOffset;
    const int first = n < inCur ? n : inCur;
    b[0] = partial(u8(val >> 56), first, b[0], bitOffset);
    if (n <= inCur) return consume(total);
    val <<= first;
    b++;
    n -= first;
    while (n >= 8) {
      *b++ = u8(val >> 56);
      val <<= 8;
      n -= 8;
    }
    if (n > 0) b[0] = partial(u8(val >> 56), n, b[0], 0);
    return consume(total);
  }
  DDErr consume(int n) {
    if (n > remainingBits()) return DD_NO_SPACE;
    pos += (bitOffset + n) / 8;
    bitOffset = (bitOffset + n) % 8;
    return DD_OK;
  }
  DDErr nonSymmetric(u32 val, u32 numValues) {
    if (!(val < numValues && numValues <= (1u << 31))) return DD_INVALID;
    if (numValues == 1) return DD_OK;
    const int w = bitwidth(numValues);
    const u32 numMin = (1u << w) - numValues;
    return val < numMin ? write(val, w - 1) : write(u64(val + numMin), w);
  }
};
inline int sizeNonSymmetricBits(u32 val, u32 numValues) {
  const int w = bitwidth(numValues);
  const u32 numMin = (1u << w) - numValues;
  return val < numMin ? w - 1 : w;
}

// dependencydescriptorextension.go types
struct Template {
  int SpatialId = 0, TemporalId = 0;
  std::vector<int> DTIs;  // DecodeTargetIndication: 0 '-', 1 'D', 2 'S', 3 'R'
  std::vector<int> FrameDiffs;
  std::vector<int> ChainDiffs;
  bool hasDTIs = false, hasFdiffs = false;  // Go nil-vs-empty slices (DeepEqual, nil checks)
};
struct Resolution {
  int Width = 0, Height = 0;
};
struct Structure {
  int StructureId = 0, NumDecodeTargets = 0, NumChains = 0;
  std::vector<int> DecodeTargetProtectedByChain;
  std::vector<Resolution> Resolutions;
  std::vector<Template> Templates;
};
struct Descriptor {
  bool FirstPacketInFrame = false, LastPacketInFrame = false;
  u16 FrameNumber = 0;
  bool hasDeps = false;
  Template FrameDependencies;
  bool hasResolution = false;
  Resolution Res;
  bool hasActiveMask = false;
  u32 ActiveDecodeTargetsBitmask = 0;
  std::shared_ptr<Structure> AttachedStructure;
};

// dependencydescriptorreader.go
struct Reader {
  BitReader b;
  Descriptor *d;
  const Structure *structure;
  int templateId = 0;
  bool activePresent = false, customDtis = false, customFdiffs = false, customChains = false;
  Reader(const u8 *buf, int n, const Structure *s, Descriptor *desc) : b(buf, n), d(desc), structure(s) {}

  DDErr Parse(int &nread) {
    nread = 0;
    DDErr e = mandatory();
    if (e) return e;
    if (b.len > 3) {
      e = extended();
      if (e) return e;
    }
    if (d->AttachedStructure) structure = d->AttachedStructure.get();
    if (!structure) {
      b.invalidate();
      return DD_NO_STRUCTURE;
    }
    if (activePresent) {
      u64 m;
      e = b.bits(structure->NumDecodeTargets, m);
      if (e) return e;
      d->hasActiveMask = true;
      d->ActiveDecodeTargetsBitmask = u32(m);
    }
    e = frameDependencyDefinition();
    if (e) return e;
    nread = b.bytesRead();
    return DD_OK;
  }
  DDErr mandatory() {
    DDErr e;
    if ((e = b.flag(d->FirstPacketInFrame))) return e;
    if ((e = b.flag(d->LastPacketInFrame))) return e;
    u64 v;
    if ((e = b.bits(6, v))) return e;
    templateId = int(v);
    if ((e = b.bits(16, v))) return e;
    d->FrameNumber = u16(v);
    return DD_OK;
  }
  DDErr extended() {
    bool structPresent;
    DDErr e;
    if ((e = b.flag(structPresent))) return e;
    if ((e = b.flag(activePresent))) return e;
    if ((e = b.flag(customDtis))) return e;
    if ((e = b.flag(customFdiffs))) return e;
    if ((e = b.flag(customChains))) return e;
    if (structPresent) {
      if ((e = templateStructure())) return e;
      if (!d->AttachedStructure) return DD_TEMPLATE_WITHOUT_STRUCTURE;
      d->hasActiveMask = true;
      d->ActiveDecodeTargetsBitmask = u32((u64(1) << d->AttachedStructure->NumDecodeTargets) - 1);
    }
    return DD_OK;
  }
  DDErr templateStructure() {
    d->AttachedStructure = std::make_shared<Structure>();
    Structure &s = *d->AttachedStructure;
    u64 v;
    DDErr e;
    if ((e = b.bits(6, v))) return e;
    s.StructureId = int(v);
    if ((e = b.bits(5, v))) return e;
    s.NumDecodeTargets = int(v) + 1;
    // readTemplateLayers
    int tid = 0, sid = 0;
    for (;;) {
      if (int(s.Templates.size()) == MaxTemplates) return DD_TOO_MANY_TEMPLATES;
      Template t;
      t.TemporalId = tid;
      t.SpatialId = sid;
      s.Templates.push_back(t);
      if ((e = b.bits(2, v))) return e;
      const int idc = int(v);
      if (idc == 1) {
        if (++tid >= MaxTemporalIds) return DD_TOO_MANY_TEMPORAL;
      } else if (idc == 2) {
        sid++;
        tid = 0;
        if (sid >= MaxSpatialIds) return DD_TOO_MANY_SPATIAL;
      }
      if (!(idc != 3 && b.ok())) break;
    }
    // readTemplateDtis
    for (auto &t : s.Templates) {
      t.DTIs.assign(s.NumDecodeTargets, 0);
      t.hasDTIs = true;
      for (auto &x : t.DTIs) {
        if ((e = b.bits(2, v))) return e;
        x = int(v);
      }
    }
    // readTemplateFdiffs
    for (auto &t : s.Templates) {
      for (;;) {
        bool follow;
        if ((e = b.flag(follow))) return e;
        if (!follow) break;
        if ((e = b.bits(4, v))) return e;
        t.FrameDiffs.push_back(int(v) + 1);
        t.hasFdiffs = true;
      }
    }
    // readTemplateChains
    u32 nc;
    if ((e = b.nonSymmetric(u32(s.NumDecodeTargets) + 1, nc))) return e;
    s.NumChains = int(nc);
    if (s.NumChains) {
      for (int i = 0; i < s.NumDecodeTargets; i++) {
        u32 pb;
        if ((e = b.nonSymmetric(u32(s.NumChains), pb))) return e;
        s.DecodeTargetProtectedByChain.push_back(int(pb));
      }
      for (auto &t : s.Templates)
        for (int c = 0; c < s.NumChains; c++) {
          if ((e = b.bits(4, v))) return e;
          t.ChainDiffs.push_back(int(v));
        }
    }
    bool hasRes;
    if ((e = b.flag(hasRes))) return e;
    if (hasRes) {
      const int layers = s.Templates.back().SpatialId + 1;
      for (int i = 0; i < layers; i++) {
        u64 w, h;
        if ((e = b.bits(16, w))) return e;
        if ((e = b.bits(16, h))) return e;
        s.Resolutions.push_back({int(w) + 1, int(h) + 1});
      }
    }
    return DD_OK;
  }
  DDErr frameDependencyDefinition() {
    const int idx = (templateId + MaxTemplates - structure->StructureId) % MaxTemplates;
    if (idx >= int(structure->Templates.size())) {
      b.invalidate();
      return DD_INVALID_TEMPLATE_INDEX;
    }
    d->hasDeps = true;
    d->FrameDependencies = structure->Templates[idx];  // Clone: copies are never nil slices
    d->FrameDependencies.hasDTIs = d->FrameDependencies.hasFdiffs = true;
    u64 v;
    DDErr e;
    if (customDtis) {
      if (int(d->FrameDependencies.DTIs.size()) != structure->NumDecodeTargets) return DD_DTI_MISMATCH;
      for (auto &x : d->FrameDependencies.DTIs) {
        if ((e = b.bits(2, v))) return e;
        x = int(v);
      }
    }
    if (customFdiffs) {
      d->FrameDependencies.FrameDiffs.clear();
      for (;;) {
        if ((e = b.bits(2, v))) return e;
        if (v == 0) break;
        u64 f;
        if ((e = b.bits(int(v) * 4, f))) return e;
        d->FrameDependencies.FrameDiffs.push_back(int(f) + 1);
      }
    }
    if (customChains) {
      if (int(d->FrameDependencies.ChainDiffs.size()) != structure->NumChains) return DD_CHAIN_MISMATCH;
      for (auto &x : d->FrameDependencies.ChainDiffs) {
        if ((e = b.bits(8, v))) return e;
        x = int(v);
      }
    }
    if (structure->Resolutions.empty()) {
      d->hasResolution = false;
    } else {
      if (d->FrameDependencies.SpatialId >= int(structure->Resolutions.size())) {
        b.invalidate();
        return DD_INVALID_SPATIAL_LAYER;
      }
      d->hasResolution = true;
      d->Res = structure->Resolutions[d->FrameDependencies.SpatialId];
    }
    return DD_OK;
  }
};

// dependencydescriptorwriter.go
struct TemplateMatch {
  int TemplateIdx = 0;
  bool NeedCustomDtis = false, NeedCustomFdiffs = false, NeedCustomChains = false;
  int ExtraSizeBits = 0;
};

struct Writer {
  const Descriptor *d;
  const Structure *s;
  u32 activeChains;
  TemplateMatch best;
  Writer(const Structure *st, u32 chains, const Descriptor *desc) : d(desc), s(st), activeChains(chains) {}

  TemplateMatch match(int idx, const Template &t) const {
    TemplateMatch r;
    r.TemplateIdx = idx;
    const Template &f = d->FrameDependencies;
    // reflect.DeepEqual on []int: equal iff both nil, or both non-nil with equal elements
    auto deq = [](const std::vector<int> &a, bool aSet, const std::vector<int> &b, bool bSet) {
      if (aSet != bSet) return false;
      return a == b;
    };
    r.NeedCustomFdiffs = f.hasFdiffs && !deq(f.FrameDiffs, f.hasFdiffs, t.FrameDiffs, t.hasFdiffs);
    r.NeedCustomDtis = f.hasDTIs && !deq(f.DTIs, f.hasDTIs, t.DTIs, t.hasDTIs);
    for (int i = 0; i < s->NumChains; i++) {
      if ((activeChains & (1u << i)) &&
          (int(f.ChainDiffs.size()) <= i || int(t.ChainDiffs.size()) <= i || f.ChainDiffs[i] != t.ChainDiffs[i])) {
        r.NeedCustomChains = true;
        break;
      }
    }
    if (r.NeedCustomFdiffs) {
      r.ExtraSizeBits = 2 * (1 + int(f.FrameDiffs.size()));
      for (int fd : f.FrameDiffs) r.ExtraSizeBits += fd <= (1 << 4) ? 4 : fd <= (1 << 8) ? 8 : 12;
    }
    if (r.NeedCustomDtis) r.ExtraSizeBits += 2 * int(f.DTIs.size());
    if (r.NeedCustomChains) r.ExtraSizeBits += 8 * s->NumChains;
    return r;
  }
  DDErr findBestTemplate() {
    int first = -1;
    const Template &f = d->FrameDependencies;
    for (int i = 0; i < int(s->Templates.size()); i++)
      if (s->Templates[i].SpatialId == f.SpatialId && s->Templates[i].TemporalId == f.TemporalId) {
        first = i;
        break;
      }
    if (first < 0) return DD_NO_TEMPLATE;
    // lastSameLayerIdx: the reference records the last index whose layer
    // DIFFERS (writer.go findBestTemplate), restated as written
    int last = 0;
    for (int i = first; i < int(s->Templates.size()); i++)
      if (s->Templates[i].SpatialId != f.SpatialId || s->Templates[i].TemporalId != f.TemporalId) last = i;
    best = match(first, s->Templates[first]);
    for (int i = first + 1; i <= last; i++) {
      TemplateMatch m = match(i, s->Templates[i]);
      if (m.ExtraSizeBits < best.ExtraSizeBits) best = m;
    }
    return DD_OK;
  }
  bool shouldWriteActive() const {
    if (!d->hasActiveMask) return false;
    const u64 all = (u64(1) << s->NumDecodeTargets) - 1;
    if (d->AttachedStructure && u64(d->ActiveDecodeTargetsBitmask) == all) return false;
    return true;
  }
  bool hasExtended() const { return best.ExtraSizeBits > 0 || d->AttachedStructure || d->hasActiveMask; }
  int structureSizeBits() const {
    int bits = 11;
    const int nt = int(s->Templates.size());
    bits += 2 * nt + 2 * nt * s->NumDecodeTargets + nt;
    for (auto &t : s->Templates) bits += 5 * int(t.FrameDiffs.size());
    bits += sizeNonSymmetricBits(u32(s->NumChains), u32(s->NumDecodeTargets + 1));
    if (s->NumChains > 0) {
      for (int pb : s->DecodeTargetProtectedByChain) bits += sizeNonSymmetricBits(u32(pb), u32(s->NumChains));
      bits += 4 * nt * s->NumChains;
    }
    bits += 1 + 32 * int(s->Resolutions.size());
    return bits;
  }
  int valueSizeBits() const {
    int v = 1 + 1 + 6 + 16 + best.ExtraSizeBits;
    if (hasExtended()) {
      v += 5;
      if (d->AttachedStructure) v += structureSizeBits();
      if (shouldWriteActive()) v += s->NumDecodeTargets;
    }
    return v;
  }
  DDErr write(std::vector<u8> &out) {
    DDErr e = findBestTemplate();
    if (e) return e;
    BitWriter w(&out);
    const Template &f = d->FrameDependencies;
    if ((e = w.write(d->FirstPacketInFrame, 1)) || (e = w.write(d->LastPacketInFrame, 1))) return e;
    if ((e = w.write(u64((best.TemplateIdx + s->StructureId) % MaxTemplates), 6))) return e;
    if ((e = w.write(d->FrameNumber, 16))) return e;
    if (hasExtended()) {
      const bool act = shouldWriteActive();
      if ((e = w.write(d->AttachedStructure ? 1 : 0, 1)) || (e = w.write(act, 1)) ||
          (e = w.write(best.NeedCustomDtis, 1)) || (e = w.write(best.NeedCustomFdiffs, 1)) ||
          (e = w.write(best.NeedCustomChains, 1)))
        return e;
      if (d->AttachedStructure) {
        if (!(s->StructureId >= 0 && s->StructureId < MaxTemplates && s->NumDecodeTargets > 0 &&
              s->NumDecodeTargets <= MaxDecodeTargets))
          return DD_INVALID;
        if ((e = w.write(u64(s->StructureId), 6)) || (e = w.write(u64(s->NumDecodeTargets - 1), 5))) return e;
        // writeTemplateLayers
        if (!(!s->Templates.empty() && int(s->Templates.size()) <= MaxTemplates && s->Templates[0].SpatialId == 0 &&
              s->Templates[0].TemporalId == 0))
          return DD_INVALID;
        for (size_t i = 1; i < s->Templates.size(); i++) {
          const Template &p = s->Templates[i - 1], &n = s->Templates[i];
          int idc;
          if (n.SpatialId == p.SpatialId && n.TemporalId == p.TemporalId)
            idc = 0;
          else if (n.SpatialId == p.SpatialId && n.TemporalId == p.TemporalId + 1)
            idc = 1;
          else if (n.SpatialId == p.SpatialId + 1 && n.TemporalId == 0)
            idc = 2;
          else
            idc = 4;
          if (idc >= 3) return DD_INVALID;
          if ((e = w.write(u64(idc), 2))) return e;
        }
        if ((e = w.write(3, 2))) return e;
        for (auto &t : s->Templates)
          for (int x : t.DTIs)
            if ((e = w.write(u64(x), 2))) return e;
        for (auto &t : s->Templates) {
          for (int fd : t.FrameDiffs)
            if ((e = w.write((u64(1) << 4) | u64(fd - 1), 5))) return e;
          if ((e = w.write(0, 1))) return e;
        }
        if ((e = w.nonSymmetric(u32(s->NumChains), u32(s->NumDecodeTargets + 1)))) return e;
        if (s->NumChains) {
          for (int pb : s->DecodeTargetProtectedByChain)
            if ((e = w.nonSymmetric(u32(pb), u32(s->NumChains)))) return e;
          for (auto &t : s->Templates)
            for (int cd : t.ChainDiffs)
              if ((e = w.write(u64(cd), 4))) return e;
        }
        if ((e = w.write(s->Resolutions.empty() ? 0 : 1, 1))) return e;
        for (auto &r : s->Resolutions)
          if ((e = w.write(u64(r.Width) - 1, 16)) || (e = w.write(u64(r.Height) - 1, 16))) return e;
      }
      if (act && (e = w.write(u64(d->ActiveDecodeTargetsBitmask), s->NumDecodeTargets))) return e;
      // writeFrameDependencyDefinition
      if (best.NeedCustomDtis)
        for (int x : f.DTIs)
          if ((e = w.write(u64(x), 2))) return e;
      if (best.NeedCustomFdiffs) {
        for (int fd : f.FrameDiffs) {
          if (fd <= (1 << 4))
            e = w.write((u64(1) << 4) | u64(fd - 1), 6);
          else if (fd <= (1 << 8))
            e = w.write((u64(2) << 8) | u64(fd - 1), 10);
          else
            e = w.write((u64(3) << 12) | u64(fd - 1), 14);
          if (e) return e;
        }
        if ((e = w.write(0, 2))) return e;
      }
      if (best.NeedCustomChains)
        for (int i = 0; i < s->NumChains; i++) {
          const int cd = (activeChains & (1u << i)) ? f.ChainDiffs[i] : 0;
          if ((e = w.write(u64(cd), 8))) return e;
        }
    }
    const int rem = w.remainingBits();  // zero the padding
    if (rem % 64) {
      if ((e = w.write(0, rem % 64))) return e;
    }
    for (int i = 0; i < rem / 64; i++)
      if ((e = w.write(0, 64))) return e;
    return DD_OK;
  }
};

// DependencyDescriptorExtension.MarshalWithActiveChains / Unmarshal
inline DDErr Marshal(const Structure *s, const Descriptor &d, u32 activeChains, std::vector<u8> &out) {
  Writer w(s, activeChains, &d);
  DDErr e = w.findBestTemplate();
  if (e) return e;
  out.assign(size_t((w.valueSizeBits() + 7) / 8), 0);
  return w.write(out);
}
inline DDErr Unmarshal(const u8 *buf, int n, const Structure *s, Descriptor &d, int &nread) {
  Reader r(buf, n, s, &d);
  return r.Parse(nread);
}

// videolayerselector/framenumberwrapper.go UpdateAndGet
struct FrameNumberWrapper {
  bool inited = false;
  u64 last = 0, offset = 0;
  u64 UpdateAndGet(u64 nw, bool updateOffset) {
    if (!inited) {
      last = nw;
      inited = true;
      return nw;
    }
    if (nw <= last) return nw + offset;
    if (updateOffset) {
      const u16 n16 = u16(nw + offset), l16 = u16(last + offset);
      const u16 diff = u16(n16 - l16);
      if (diff > 0x8000 || (diff == 0x8000 && n16 <= l16)) offset += u64(65535 - diff + 6000);
    }
    last = nw;
    return nw + offset;
  }
};

}  // namespace orc_dd
