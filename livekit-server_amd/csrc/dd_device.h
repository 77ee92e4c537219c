// dd_device.h — gfx950 device code of the dependency-descriptor path
// (SURVEY.md §8(a) a9 + a16), included by forward_kernels.hip and
// ingress_kernels.hip.
//
//   dd_parse        DependencyDescriptorExtension.Unmarshal
//                   (dependencydescriptor/dependencydescriptorreader.go) into a
//                   DDPkt, with the structure ring of the track; an attached
//                   FrameDependencyStructure is written to a ring slot and its
//                   decode targets sorted (ProcessFrameDependencyStructure,
//                   buffer/dependencydescriptorparser.go:178-201)
//   dd_marshal      DependencyDescriptorExtension.Marshal
//                   (dependencydescriptor/dependencydescriptorwriter.go:40-515)
//   dd_select       videolayerselector.DependencyDescriptor.Select
//                   (videolayerselector/dependencydescriptor.go:65-355) with the
//                   SelectorDecisionCache (selectordecisioncache.go), FrameChain
//                   (framechain.go), DecodeTarget (decodetarget.go) and
//                   FrameNumberWrapper (framenumberwrapper.go) as one DDState.
//
// Everything here is wave-uniform scalar code on one descriptor: the decide
// kernel runs it on the broadcast packet with the DownTrack's DDState staged in
// LDS (every lane computes the same values; same-value LDS writes).
//
// FrameChain callbacks: the reference registers FrameChain.OnExpectFrameChanged
// in the decision cache for every unknown previous-in-chain frame and appends
// the frame to the chain's expectFrames.  All registrations of one frame fire
// together (on its first non-unknown decision, or when it ages out), and a
// registration whose frame has left expectFrames (cleared on a chain-intact
// frame) does nothing; a chain that is broken ignores them until a clearing
// frame.  So each chain keeps the SET of frames it waits on: a decision for a
// member removes it, and a non-forwarded decision breaks the chain.
#pragma once
#include "fwd_state.h"

namespace lkf {
namespace dd {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i32 = int32_t;

enum Err { OK = 0, EOFB, NO_STRUCTURE, TEMPLATE_WITHOUT_STRUCTURE, TOO_MANY, INVALID, LIMIT };

__device__ __forceinline__ int bitwidth(u32 n) { return n ? 32 - __clz(int(n)) : 0; }

// bitstreamreader.go
struct BitR {
  const u8 *buf;
  int len, pos, remaining;
  __device__ BitR(const u8 *b, int n) : buf(b), len(n), pos(0), remaining(n * 8) {}
  __device__ int bits(int n, u64 &out) {
    out = 0;
    if (n < 0 || n > 64) return INVALID;
    if (remaining < n) {
      remaining -= n;
      return EOFB;
    }
    int inFirst = remaining % 8;
    remaining -= n;
    if (n < inFirst) {
      out = u64((buf[pos] >> (inFirst - n)) & ((1u << n) - 1));
      return OK;
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
    return OK;
  }
  __device__ int flag(bool &b) {
    u64 v;
    const int e = bits(1, v);
    b = v != 0;
    return e;
  }
  __device__ bool ok() const { return remaining >= 0; }
  __device__ int nonSymmetric(u32 numValues, u32 &out) {  // av1 ns(n)
    out = 0;
    if (numValues >= (1u << 31)) return INVALID;
    const int w = bitwidth(numValues);
    const u32 numMin = (1u << w) - numValues;
    u64 v;
    int e = bits(w - 1, v);
    if (e) return e;
    if (v < numMin) {
      out = u32(v);
      return OK;
    }
    u64 b;
    e = bits(1, b);
    if (e) return e;
    out = u32((v << 1) + b - numMin);
    return OK;
  }
};

__device__ __forceinline__ u32 dti_at(u64 dtis, int i) { return u32(dtis >> (2 * i)) & 3u; }

// ProcessFrameDependencyStructure: decode-target layers = max (S, T) over the
// templates that are present in the target; sorted high -> low by
// VideoLayer.GreaterThan (insertion sort: Go's pdqsort below 12 elements)
struct Match {
  int idx;
  bool cDtis, cFdiffs, cChains;
  int extra;
};

// calculateMatch of template j for a packet that uses template k without
// custom fields (its frame diffs, DTIs and chain diffs are template k's)
#ifndef LKF_DD_PACK
#define LKF_DD_PACK 1  // SVC runs: a custom-field-free descriptor packed in a register (dd_marshal_tmpl)
#endif
#ifndef LKF_DD_SER
#define LKF_DD_SER 1  // marshal: an attached structure copied from its serialization (ser_structure)
#endif
#ifndef LKF_DD_FASTBEST
#define LKF_DD_FASTBEST 1  // marshal: the structure's precomputed best template (tmpl_best)
#endif

__device__ inline Match tmpl_match(const DDStruct &s, int j, int k) {
  const DDTmpl &t = s.t[j], &q = s.t[k];
  Match m;
  m.idx = j;
  bool fdEq = t.nfd != 0 && t.nfd == q.nfd;
  for (int i = 0; fdEq && i < q.nfd; i++) fdEq = s.fdPool[q.fdOff + i] == s.fdPool[t.fdOff + i];
  m.cFdiffs = !fdEq;
  const u64 dm = s.numDT >= 32 ? ~u64(0) : ((u64(1) << (2 * s.numDT)) - 1);
  m.cDtis = (q.dtis & dm) != (t.dtis & dm);
  m.cChains = false;
  for (int i = 0; i < s.numChains; i++)
    if (dd_tmpl_chain(q, i) != dd_tmpl_chain(t, i)) {
      m.cChains = true;
      break;
    }
  m.extra = 0;
  if (m.cFdiffs) m.extra = 2 * (1 + q.nfd) + 4 * q.nfd;  // (template frame diffs are 1-16: 4 bits each)
  if (m.cDtis) m.extra += 2 * s.numDT;
  if (m.cChains) m.extra += 8 * s.numChains;
  return m;
}

// findBestTemplate (dependencydescriptorwriter.go) for every template's
// custom-field-free packets, as dd_marshal_inl runs it
__device__ inline void tmpl_best(DDStruct &s) {
  for (int k = 0; k < s.numTmpl; k++) {
    const DDTmpl &q = s.t[k];
    int first = 0;
    while (first < s.numTmpl && !(s.t[first].sid == q.sid && s.t[first].tid == q.tid)) first++;
    int lastIdx = 0;  // as written: the last index whose layer differs
    for (int i = first; i < s.numTmpl; i++)
      if (s.t[i].sid != q.sid || s.t[i].tid != q.tid) lastIdx = i;
    Match best = tmpl_match(s, first, k);
    for (int i = first + 1; i <= lastIdx; i++) {
      const Match m = tmpl_match(s, i, k);
      if (m.extra < best.extra) best = m;
    }
    s.t[k].best = u8(best.idx);
    s.t[k].bestC = u8((best.cDtis ? 1 : 0) | (best.cFdiffs ? 2 : 0) | (best.cChains ? 4 : 0));
  }
}

__device__ inline void process_structure(DDStruct &s) {
  for (int t = 0; t < s.numDT; t++) {
    int ls = 0, lt = 0;
    for (int k = 0; k < s.numTmpl; k++)
      if (dti_at(s.t[k].dtis, t) != 0) {
        if (ls < s.t[k].sid) ls = s.t[k].sid;
        if (lt < s.t[k].tid) lt = s.t[k].tid;
      }
    s.dtTarget[t] = u8(t);
    s.dtS[t] = u8(ls);
    s.dtT[t] = u8(lt);
  }
  for (int i = 1; i < s.numDT; i++)
    for (int j = i; j > 0; j--) {
      const bool gt = s.dtS[j] > s.dtS[j - 1] || (s.dtS[j] == s.dtS[j - 1] && s.dtT[j] > s.dtT[j - 1]);
      if (!gt) break;
      u8 a = s.dtTarget[j], b = s.dtS[j], c = s.dtT[j];
      s.dtTarget[j] = s.dtTarget[j - 1];
      s.dtS[j] = s.dtS[j - 1];
      s.dtT[j] = s.dtT[j - 1];
      s.dtTarget[j - 1] = a;
      s.dtS[j - 1] = b;
      s.dtT[j - 1] = c;
    }
}

// templateStructure (dependencydescriptorreader.go readTemplateDependencyStructure)
__device__ inline int read_structure(BitR &b, DDStruct &s) {
  u64 v;
  int e;
  if ((e = b.bits(6, v))) return e;
  s.structureId = u8(v);
  if ((e = b.bits(5, v))) return e;
  s.numDT = u8(v + 1);
  s.numTmpl = 0;
  s.numRes = 0;
  s.nfdPool = 0;
  int tid = 0, sid = 0;
  for (;;) {
    if (s.numTmpl == 64) return TOO_MANY;
    DDTmpl &t = s.t[s.numTmpl++];
    t.sid = u8(sid);
    t.tid = u8(tid);
    t.nfd = 0;
    t.fdOff = 0;
    t.best = t.bestC = 0;
    t.chains[0] = t.chains[1] = t.chains[2] = t.chains[3] = 0;
    t.dtis = 0;
    if ((e = b.bits(2, v))) return e;
    const int idc = int(v);
    if (idc == 1) {
      if (++tid >= 8) return TOO_MANY;
    } else if (idc == 2) {
      sid++;
      tid = 0;
      if (sid >= 4) return TOO_MANY;
    }
    if (!(idc != 3 && b.ok())) break;
  }
  for (int k = 0; k < s.numTmpl; k++)
    for (int i = 0; i < s.numDT; i++) {
      if ((e = b.bits(2, v))) return e;
      s.t[k].dtis |= v << (2 * i);
    }
  for (int k = 0; k < s.numTmpl; k++) {  // the templates' frame diffs, one pool in template order
    s.t[k].fdOff = s.nfdPool;
    for (;;) {
      bool follow;
      if ((e = b.flag(follow))) return e;
      if (!follow) break;
      if ((e = b.bits(4, v))) return e;
      if (s.nfdPool >= kDDFdPool) return LIMIT;  // (more than 255 bytes hold)
      s.fdPool[s.nfdPool++] = u8(v + 1);
      s.t[k].nfd++;
    }
  }
  u32 nc;
  if ((e = b.nonSymmetric(u32(s.numDT) + 1, nc))) return e;
  if (nc > u32(kDDChains)) return LIMIT;  // (nc <= NumDecodeTargets <= 32: never)
  s.numChains = u8(nc);
  if (nc) {
    for (int i = 0; i < s.numDT; i++) {
      u32 pb;
      if ((e = b.nonSymmetric(nc, pb))) return e;
      s.protectedBy[i] = u8(pb);
    }
    for (int k = 0; k < s.numTmpl; k++)
      for (u32 c = 0; c < nc; c++) {
        if ((e = b.bits(4, v))) return e;
        s.t[k].chains[c >> 3] |= u32(v) << (4 * (c & 7));
      }
  }
  bool hasRes;
  if ((e = b.flag(hasRes))) return e;
  if (hasRes) {
    const int layers = s.t[s.numTmpl - 1].sid + 1;
    for (int i = 0; i < layers; i++) {
      u64 w, h;
      if ((e = b.bits(16, w))) return e;
      if ((e = b.bits(16, h))) return e;
      s.resW[i] = u16(w + 1);
      s.resH[i] = u16(h + 1);
    }
    s.numRes = u8(layers);
  }
  process_structure(s);
  tmpl_best(s);
  return OK;
}

// Parse: buf/len = the DD extension payload; cur = the track's current
// structure (nullptr before any); att = the ring slot an attached structure is
// written to.  On success o holds the descriptor and *usedAttached tells
// whether att became the structure.  A frame's custom frame diffs beyond
// kDDFdInline go to spill (bump-allocated at *spillUsed, spillCap entries);
// spill == nullptr keeps only their count (FD_NONE).
__device__ inline int dd_parse(const u8 *buf, int len, const DDStruct *cur, DDStruct *att, DDPkt &o,
                               bool &usedAttached, u16 *spill = nullptr, u32 *spillUsed = nullptr,
                               u32 spillCap = 0) {
  usedAttached = false;
  BitR b(buf, len);
  u64 v;
  int e;
  bool first, last;
  if ((e = b.flag(first)) || (e = b.flag(last))) return e;
  if ((e = b.bits(6, v))) return e;
  const int templateId = int(v);
  if ((e = b.bits(16, v))) return e;
  o.frameNumber = u16(v);
  o.flags = u8((first ? DP_FIRST : 0) | (last ? DP_LAST : 0));
  bool structPresent = false, activePresent = false, customDtis = false, customFdiffs = false, customChains = false;
  if (b.len > 3) {
    if ((e = b.flag(structPresent)) || (e = b.flag(activePresent)) || (e = b.flag(customDtis)) ||
        (e = b.flag(customFdiffs)) || (e = b.flag(customChains)))
      return e;
    if (structPresent) {
      if ((e = read_structure(b, *att))) return e;
      usedAttached = true;
      o.flags |= DP_ATTACHED | DP_ACTIVE;
      o.activeMask = u32((u64(1) << att->numDT) - 1);
    }
  }
  const DDStruct *s = usedAttached ? att : cur;
  if (!s) return NO_STRUCTURE;
  if (activePresent) {
    if ((e = b.bits(s->numDT, v))) return e;
    o.flags |= DP_ACTIVE;
    o.activeMask = u32(v);
  }
  // frameDependencyDefinition: the template, then the custom fields
  const int idx = (templateId + 64 - s->structureId) % 64;
  if (idx >= s->numTmpl) return INVALID;
  const DDTmpl &t = s->t[idx];
  o.tmplIdx = u8(idx);
  o.custom = u8((customDtis ? 1 : 0) | (customFdiffs ? 2 : 0) | (customChains ? 4 : 0));
  o.sid = t.sid;
  o.tid = t.tid;
  o.dtis = t.dtis;
  o.ndti = s->numDT;
  // the inline frame diffs gather in four words by name (a run-time index
  // into o.fd put the whole descriptor on the private stack)
  u32 fw0 = 0, fw1 = 0, fw2 = 0, fw3 = 0;
  auto put_fd = [&](u32 k, u32 f) {
    const u32 x = f << (16 * (k & 1));
    fw0 |= (k >> 1) == 0 ? x : 0u;
    fw1 |= (k >> 1) == 1 ? x : 0u;
    fw2 |= (k >> 1) == 2 ? x : 0u;
    fw3 |= (k >> 1) == 3 ? x : 0u;
  };
  o.nfd = t.nfd;
  if (t.nfd <= kDDFdInline) {
    o.fdKind = FD_INLINE;
    for (int i = 0; i < t.nfd; i++) put_fd(u32(i), s->fdPool[t.fdOff + i]);
  } else {  // a long template list stays in the structure's pool
    o.fdKind = FD_POOL;
    o.fdRef = t.fdOff;
  }
  o.nchain = s->numChains;
  {  // (four words by name, not by a run-time index: that put o on the private stack)
    u64 w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    for (int c = 0; c < s->numChains; c++) {
      const u64 v = u64(dd_tmpl_chain(t, c)) << (8 * (c & 7));
      w0 |= (c >> 3) == 0 ? v : 0;
      w1 |= (c >> 3) == 1 ? v : 0;
      w2 |= (c >> 3) == 2 ? v : 0;
      w3 |= (c >> 3) == 3 ? v : 0;
    }
    o.chainDiffs[0] = w0, o.chainDiffs[1] = w1, o.chainDiffs[2] = w2, o.chainDiffs[3] = w3;
  }
  if (customDtis) {
    o.dtis = 0;
    for (int i = 0; i < s->numDT; i++) {
      if ((e = b.bits(2, v))) return e;
      o.dtis |= v << (2 * i);
    }
  }
  if (customFdiffs) {
    const BitR at = b;  // (a list longer than kDDFdInline is read again into the spill)
    u32 n = 0;
    fw0 = fw1 = fw2 = fw3 = 0;
    for (;;) {
      if ((e = b.bits(2, v))) return e;
      if (v == 0) break;
      u64 f;
      if ((e = b.bits(int(v) * 4, f))) return e;
      if (n < u32(kDDFdInline)) put_fd(n, u32(u16(f + 1)));
      n++;
    }
    o.nfd = u16(n);
    o.fdKind = FD_INLINE;
    if (n > u32(kDDFdInline)) {
      if (!spill) {
        o.fdKind = FD_NONE;
      } else {
        const u32 off = atomicAdd(spillUsed, n);
        if (off + n > spillCap) return LIMIT;  // (the batch's spill capacity)
        BitR r = at;
        for (u32 k = 0; k < n; k++) {
          r.bits(2, v);
          u64 f;
          r.bits(int(v) * 4, f);
          spill[off + k] = u16(f + 1);
        }
        o.fdKind = FD_SPILL;
        o.fdRef = off;
      }
    }
  }
  if (customChains) {
    u64 w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    for (int c = 0; c < s->numChains; c++) {
      if ((e = b.bits(8, v))) return e;
      const u64 x = v << (8 * (c & 7));
      w0 |= (c >> 3) == 0 ? x : 0;
      w1 |= (c >> 3) == 1 ? x : 0;
      w2 |= (c >> 3) == 2 ? x : 0;
      w3 |= (c >> 3) == 3 ? x : 0;
    }
    o.chainDiffs[0] = w0, o.chainDiffs[1] = w1, o.chainDiffs[2] = w2, o.chainDiffs[3] = w3;
  }
  o.fd[0] = u16(fw0), o.fd[1] = u16(fw0 >> 16), o.fd[2] = u16(fw1), o.fd[3] = u16(fw1 >> 16);
  o.fd[4] = u16(fw2), o.fd[5] = u16(fw2 >> 16), o.fd[6] = u16(fw3), o.fd[7] = u16(fw3 >> 16);
  if (s->numRes && o.sid >= s->numRes) return INVALID;
  return OK;
}

// ---- writer (dependencydescriptorwriter.go) ------------------------------------
struct BitW {
  // bits gather in a register and leave as whole bytes (one byte store per 8
  // bits instead of a read-modify-write per bit); finish() writes the last
  // partial byte, zero-padded
  u8 *buf;  // cap bytes
  int cap, bitPos;
  u64 acc;
  int accBits, bytePos;
  __device__ BitW(u8 *b, int c) : buf(b), cap(c), bitPos(0), acc(0), accBits(0), bytePos(0) {}
  __device__ int write(u64 val, int n) {  // MSB first, n <= 32
    if (bitPos + n > cap * 8) return INVALID;
    acc = (acc << n) | (n >= 64 ? val : (val & ((u64(1) << n) - 1)));
    accBits += n;
    bitPos += n;
    while (accBits >= 8) {
      accBits -= 8;
      buf[bytePos++] = u8(acc >> accBits);
    }
    return OK;
  }
  __device__ void finish() {
    if (accBits > 0) buf[bytePos++] = u8(acc << (8 - accBits));
    accBits = 0;
  }
  __device__ int nonSymmetric(u32 val, u32 numValues) {
    if (!(val < numValues && numValues <= (1u << 31))) return INVALID;
    if (numValues == 1) return OK;
    const int w = bitwidth(numValues);
    const u32 numMin = (1u << w) - numValues;
    return val < numMin ? write(val, w - 1) : write(u64(val + numMin), w);
  }
};
__device__ __forceinline__ int ns_bits(u32 val, u32 numValues) {
  const int w = bitwidth(numValues);
  const u32 numMin = (1u << w) - numValues;
  return val < numMin ? w - 1 : w;
}

// FrameDependencies.FrameDiffs[i] of a parsed packet: in the DDPkt, in the
// parse-time structure's pool (pool = its fdPool), or in the batch's spill
__device__ __forceinline__ u32 fd_at(const DDPkt &p, const u8 *pool, const u16 *spill, int i) {
  if (p.fdKind == FD_INLINE) return p.fd[i];
  if (p.fdKind == FD_POOL) return pool[p.fdRef + u32(i)];
  return spill[p.fdRef + u32(i)];
}



// calculateMatch: frame DTIs / FrameDiffs are never nil after a parse (Clone);
// a template's FrameDiffs is nil iff it has none (reflect.DeepEqual(nil, []) = false)
__device__ inline Match dd_match(const DDStruct &s, int idx, const DDPkt &p, const u8 *ppool, const u16 *spill) {
  const DDTmpl &t = s.t[idx];
  Match m;
  m.idx = idx;
  bool fdEq = t.nfd != 0 && t.nfd == p.nfd;
  for (int i = 0; fdEq && i < p.nfd; i++) fdEq = fd_at(p, ppool, spill, i) == s.fdPool[t.fdOff + i];
  m.cFdiffs = !fdEq;
  const u64 dm = p.ndti >= 32 ? ~u64(0) : ((u64(1) << (2 * p.ndti)) - 1);
  m.cDtis = !(p.ndti == s.numDT && (p.dtis & dm) == (t.dtis & dm));
  m.cChains = false;
  for (int i = 0; i < s.numChains; i++)
    if (p.nchain <= i || dd_chain_diff(p, i) != dd_tmpl_chain(t, i)) {
      m.cChains = true;
      break;
    }
  m.extra = 0;
  if (m.cFdiffs) {
    m.extra = 2 * (1 + p.nfd);
    for (int i = 0; i < p.nfd; i++) {
      const u32 f = fd_at(p, ppool, spill, i);
      m.extra += f <= 16 ? 4 : f <= 256 ? 8 : 12;
    }
  }
  if (m.cDtis) m.extra += 2 * p.ndti;
  if (m.cChains) m.extra += 8 * s.numChains;
  return m;
}

__device__ inline int structure_bits(const DDStruct &s) {
  int bits = 11;
  const int nt = s.numTmpl;
  bits += 2 * nt + 2 * nt * s.numDT + nt;
  for (int k = 0; k < nt; k++) bits += 5 * s.t[k].nfd;
  bits += ns_bits(s.numChains, u32(s.numDT) + 1);
  if (s.numChains > 0) {
    for (int i = 0; i < s.numDT; i++) bits += ns_bits(s.protectedBy[i], s.numChains);
    bits += 4 * nt * s.numChains;
  }
  bits += 1 + 32 * s.numRes;
  return bits;
}

// Marshal (activeChains = all): writes the descriptor to out (zeroed here),
// returns its length in bytes, or -1 (error: the selector drops the frame).
// (ppool/spill: where p's frame diffs are, see fd_at)
__device__ __forceinline__ int dd_marshal_inl(const DDStruct &s, const DDPkt &p, u16 frameNumber, bool hasActive,
                                              u32 active, u8 *out, int cap, const u8 *ppool, const u16 *spill,
                                              bool sameStruct, const DDStruct *serS = nullptr) {
  // findBestTemplate.  A packet read with this structure (the one it
  // attaches, or the one in force) and with no custom field carries exactly
  // its template's fields: the search's result was computed with the
  // structure (tmpl_best)
  Match best;
  if (LKF_DD_FASTBEST && sameStruct && p.custom == 0 && p.tmplIdx < s.numTmpl) {
    const DDTmpl &q = s.t[p.tmplIdx];
    best.idx = q.best;
    best.cDtis = q.bestC & 1;
    best.cFdiffs = (q.bestC >> 1) & 1;
    best.cChains = (q.bestC >> 2) & 1;
    best.extra = 0;
    if (best.cFdiffs) {
      best.extra = 2 * (1 + p.nfd);
      for (int i = 0; i < p.nfd; i++) {
        const u32 f = fd_at(p, ppool, spill, i);
        best.extra += f <= 16 ? 4 : f <= 256 ? 8 : 12;
      }
    }
    if (best.cDtis) best.extra += 2 * p.ndti;
    if (best.cChains) best.extra += 8 * s.numChains;
  } else {
    int first = -1;
    for (int i = 0; i < s.numTmpl; i++)
      if (s.t[i].sid == p.sid && s.t[i].tid == p.tid) {
        first = i;
        break;
      }
    if (first < 0) return -1;
    int lastIdx = 0;  // as written: the last index whose layer differs
    for (int i = first; i < s.numTmpl; i++)
      if (s.t[i].sid != p.sid || s.t[i].tid != p.tid) lastIdx = i;
    best = dd_match(s, first, p, ppool, spill);
    for (int i = first + 1; i <= lastIdx; i++) {
      const Match m = dd_match(s, i, p, ppool, spill);
      if (m.extra < best.extra) best = m;
    }
  }
  const bool attached = p.flags & DP_ATTACHED;
  const u64 all = (u64(1) << s.numDT) - 1;
  const bool writeActive = hasActive && !(attached && u64(active) == all);
  const bool extended = best.extra > 0 || attached || hasActive;
  int vbits = 1 + 1 + 6 + 16 + best.extra;
  // an attached structure: its serialization (ser_structure) when given
  const u32 serBits = (attached && serS) ? u32(serS->serBits) : 0u;
  if (attached && serS && serBits == 0xffffu) return -1;
  if (extended) {
    vbits += 5;
    if (attached) vbits += serS ? int(serBits) : structure_bits(s);
    if (writeActive) vbits += s.numDT;
  }
  const int nbytes = (vbits + 7) / 8;
  if (nbytes > kDDMaxBytes || nbytes > cap) return -1;  // (cap: the caller's buffer; see svc_run)
  for (int i = 0; i < nbytes; i++) out[i] = 0;
  BitW w(out, nbytes);
  int e = 0;
  e |= w.write(p.flags & DP_FIRST ? 1 : 0, 1);
  e |= w.write(p.flags & DP_LAST ? 1 : 0, 1);
  e |= w.write(u64((best.idx + s.structureId) % 64), 6);
  e |= w.write(frameNumber, 16);
  if (extended) {
    e |= w.write(attached ? 1 : 0, 1);
    e |= w.write(writeActive ? 1 : 0, 1);
    e |= w.write(best.cDtis ? 1 : 0, 1);
    e |= w.write(best.cFdiffs ? 1 : 0, 1);
    e |= w.write(best.cChains ? 1 : 0, 1);
    if (attached && serS) {  // 32 bits at a time from the serialized structure
      const u8 *q = serS->ser;
      u32 k = 0;
      for (; k + 32 <= serBits; k += 32) {
        const u32 j = k >> 3;
        e |= w.write((u32(q[j]) << 24) | (u32(q[j + 1]) << 16) | (u32(q[j + 2]) << 8) | u32(q[j + 3]), 32);
      }
      for (; k < serBits; k += 8) {
        const u32 r = serBits - k < 8 ? serBits - k : 8u;
        e |= w.write(u32(q[k >> 3]) >> (8 - r), int(r));
      }
    } else if (attached) {
      if (!(s.structureId < 64 && s.numDT > 0 && s.numDT <= 32)) return -1;
      e |= w.write(s.structureId, 6);
      e |= w.write(u64(s.numDT - 1), 5);
      if (!(s.numTmpl > 0 && s.t[0].sid == 0 && s.t[0].tid == 0)) return -1;
      for (int i = 1; i < s.numTmpl; i++) {
        const DDTmpl &a = s.t[i - 1], &n = s.t[i];
        int idc;
        if (n.sid == a.sid && n.tid == a.tid)
          idc = 0;
        else if (n.sid == a.sid && n.tid == a.tid + 1)
          idc = 1;
        else if (n.sid == a.sid + 1 && n.tid == 0)
          idc = 2;
        else
          return -1;
        e |= w.write(u64(idc), 2);
      }
      e |= w.write(3, 2);
      for (int k = 0; k < s.numTmpl; k++)
        for (int i = 0; i < s.numDT; i++) e |= w.write(dti_at(s.t[k].dtis, i), 2);
      for (int k = 0; k < s.numTmpl; k++) {
        for (int i = 0; i < s.t[k].nfd; i++) e |= w.write((u64(1) << 4) | u64(s.fdPool[s.t[k].fdOff + i] - 1), 5);
        e |= w.write(0, 1);
      }
      e |= w.nonSymmetric(s.numChains, u32(s.numDT) + 1);
      if (s.numChains) {
        for (int i = 0; i < s.numDT; i++) e |= w.nonSymmetric(s.protectedBy[i], s.numChains);
        for (int k = 0; k < s.numTmpl; k++)
          for (int c = 0; c < s.numChains; c++) e |= w.write(dd_tmpl_chain(s.t[k], c), 4);
      }
      e |= w.write(s.numRes ? 1 : 0, 1);
      for (int i = 0; i < s.numRes; i++) {
        e |= w.write(u64(s.resW[i]) - 1, 16);
        e |= w.write(u64(s.resH[i]) - 1, 16);
      }
    }
    if (writeActive) e |= w.write(active, s.numDT);
    if (best.cDtis)
      for (int i = 0; i < p.ndti; i++) e |= w.write(dti_at(p.dtis, i), 2);
    if (best.cFdiffs) {
      for (int i = 0; i < p.nfd; i++) {
        const u64 f = fd_at(p, ppool, spill, i);
        if (f <= 16)
          e |= w.write((u64(1) << 4) | (f - 1), 6);
        else if (f <= 256)
          e |= w.write((u64(2) << 8) | (f - 1), 10);
        else
          e |= w.write((u64(3) << 12) | (f - 1), 14);
      }
      e |= w.write(0, 2);
    }
    if (best.cChains) {
      // every chain is active (Marshal = MarshalWithActiveChains(^0)); a frame
      // with fewer chain diffs than chains would index out of range (a
      // recovered panic in the reference): the frame is dropped
      if (p.nchain < s.numChains) return -1;
      for (int c = 0; c < s.numChains; c++) e |= w.write(dd_chain_diff(p, c), 8);
    }
  }
  w.finish();
  return e ? -1 : nbytes;
}
// dd_marshal_inl for a packet read with s, with no custom field and no
// structure attached: its fields are template k's, so the descriptor is
// written from the structure alone (svc_run: no read of the packet's lists)
__device__ __forceinline__ int dd_marshal_tmpl(const DDStruct &s, int k, u8 pflags, u16 frameNumber, bool hasActive,
                                               u32 active, u8 *out, int cap) {
  const DDTmpl &q = s.t[k];
  if (LKF_DD_PACK && q.bestC == 0) {
    // no custom field: the mandatory fields (+ the extended flags and the
    // active mask) are at most 61 bits, packed MSB first in one register and
    // stored as two big-endian dwords (out is dword-aligned, cap >= 8)
    const u32 nd = s.numDT;
    u64 v = (u64((pflags & DP_FIRST) ? 1 : 0) << 63) | (u64((pflags & DP_LAST) ? 1 : 0) << 62) |
            (u64((q.best + s.structureId) % 64) << 56) | (u64(frameNumber) << 40);
    int bits = 24;
    if (hasActive) {  // extended: attached 0, active 1, custom DTIs / frame diffs / chains 0
      v |= u64(0x08) << 35;
      v |= (u64(active) & (nd >= 32 ? 0xffffffffull : ((1ull << nd) - 1))) << (35 - nd);
      bits = 29 + int(nd);
    }
    u32 *o = reinterpret_cast<u32 *>(out);
    o[0] = __builtin_bswap32(u32(v >> 32));
    o[1] = __builtin_bswap32(u32(v));
    return (bits + 7) / 8;
  }
  const bool cDtis = q.bestC & 1, cFdiffs = q.bestC & 2, cChains = q.bestC & 4;
  int extra = 0;
  if (cFdiffs) extra = 2 * (1 + q.nfd) + 4 * q.nfd;  // (template frame diffs are 1-16)
  if (cDtis) extra += 2 * s.numDT;
  if (cChains) extra += 8 * s.numChains;
  const bool extended = extra > 0 || hasActive;
  int vbits = 1 + 1 + 6 + 16 + extra;
  if (extended) vbits += 5 + (hasActive ? s.numDT : 0);
  const int nbytes = (vbits + 7) / 8;
  if (nbytes > kDDMaxBytes || nbytes > cap) return -1;
  BitW w(out, nbytes);
  int e = 0;
  e |= w.write(pflags & DP_FIRST ? 1 : 0, 1);
  e |= w.write(pflags & DP_LAST ? 1 : 0, 1);
  e |= w.write(u64((q.best + s.structureId) % 64), 6);
  e |= w.write(frameNumber, 16);
  if (extended) {
    e |= w.write((u64(hasActive) << 3) | (u64(cDtis) << 2) | (u64(cFdiffs) << 1) | u64(cChains), 5);
    if (hasActive) e |= w.write(active, s.numDT);
    if (cDtis)
      for (int i = 0; i < s.numDT; i++) e |= w.write(dti_at(q.dtis, i), 2);
    if (cFdiffs) {
      for (int i = 0; i < q.nfd; i++) e |= w.write((u64(1) << 4) | u64(s.fdPool[q.fdOff + i] - 1), 6);
      e |= w.write(0, 2);
    }
    if (cChains)
      for (int c = 0; c < s.numChains; c++) e |= w.write(dd_tmpl_chain(q, c), 8);
  }
  w.finish();
  return e ? -1 : nbytes;
}

__device__ __attribute__((noinline)) int dd_marshal(const DDStruct &s, const DDPkt &p, u16 frameNumber, bool hasActive,
                                                   u32 active, u8 *out, const u8 *ppool, const u16 *spill,
                                                   bool sameStruct, const DDStruct *serS) {
  return dd_marshal_inl(s, p, frameNumber, hasActive, active, out, kDDMaxBytes, ppool, spill, sameStruct, serS);
}

// The structure's part of an attaching descriptor (Marshal's
// writeTemplateDependencyStructure .. resolutions), as dd_marshal_inl writes
// it, into s.ser: every DownTrack that forwards the attaching packet copies it
__device__ inline void ser_structure(DDStruct &s) {
  for (int i = 0; i < kDDSerBytes; i++) s.ser[i] = 0;
  BitW w(s.ser, kDDSerBytes);
  int e = 0;
  s.serBits = 0xffffu;
  if (!(s.structureId < 64 && s.numDT > 0 && s.numDT <= 32)) return;
  e |= w.write(s.structureId, 6);
  e |= w.write(u64(s.numDT - 1), 5);
  if (!(s.numTmpl > 0 && s.t[0].sid == 0 && s.t[0].tid == 0)) return;
  for (int i = 1; i < s.numTmpl; i++) {
    const DDTmpl &a = s.t[i - 1], &n = s.t[i];
    int idc;
    if (n.sid == a.sid && n.tid == a.tid)
      idc = 0;
    else if (n.sid == a.sid && n.tid == a.tid + 1)
      idc = 1;
    else if (n.sid == a.sid + 1 && n.tid == 0)
      idc = 2;
    else
      return;
    e |= w.write(u64(idc), 2);
  }
  e |= w.write(3, 2);
  for (int k = 0; k < s.numTmpl; k++)
    for (int i = 0; i < s.numDT; i++) e |= w.write(dti_at(s.t[k].dtis, i), 2);
  for (int k = 0; k < s.numTmpl; k++) {
    for (int i = 0; i < s.t[k].nfd; i++) e |= w.write((u64(1) << 4) | u64(s.fdPool[s.t[k].fdOff + i] - 1), 5);
    e |= w.write(0, 1);
  }
  e |= w.nonSymmetric(s.numChains, u32(s.numDT) + 1);
  if (s.numChains) {
    for (int i = 0; i < s.numDT; i++) e |= w.nonSymmetric(s.protectedBy[i], s.numChains);
    for (int k = 0; k < s.numTmpl; k++)
      for (int c = 0; c < s.numChains; c++) e |= w.write(dd_tmpl_chain(s.t[k], c), 4);
  }
  e |= w.write(s.numRes ? 1 : 0, 1);
  for (int i = 0; i < s.numRes; i++) {
    e |= w.write(u64(s.resW[i]) - 1, 16);
    e |= w.write(u64(s.resH[i]) - 1, 16);
  }
  const int bits = w.bitPos;
  w.finish();
  if (!e) s.serBits = u16(bits);
}

// ---- selector ------------------------------------------------------------------
enum SD : u32 { SD_MISSING = 0, SD_DROPPED = 1, SD_FORWARDED = 2, SD_UNKNOWN = 3 };
constexpr u64 kEntries = 256, kNack = 80;

__device__ __forceinline__ u32 c_get(const DDState &d, u64 e) {
  const u64 off = (e - d.cBase) % kEntries;
  return u32(d.masks[off >> 5] >> ((off & 31) * 2)) & 3u;
}
__device__ __forceinline__ void c_put(DDState &d, u64 e, u32 sd) {
  const u64 off = (e - d.cBase) % kEntries;
  const int bp = int(off & 31) * 2;
  d.masks[off >> 5] = (d.masks[off >> 5] & ~(u64(3) << bp)) | (u64(sd & 3) << bp);
}
// ---- FrameChain.expectFrames as a set (round 6) ---------------------------------
// A chain waits only on frames ExpectDecision accepted: not older than
// cLast - 255 when registered, and gone (missing: the chain breaks) once older
// than cLast - 256; below cLast + 256 in every case but one: a packet whose
// frame number jumped ahead of cLast may register one frame beyond, and its own
// add then moves cLast past it.  So each chain keeps a ring of 512 bits, bit
// e % 512 for frame e in [cLast - 256, cLast + 256), and one frame beyond
// (exp[c][8], expFar[c]).  A broken chain's set is never read again (the
// reference skips its callbacks and clears it with the chain-intact frame that
// un-breaks it), so it is cleared when the chain breaks.
constexpr u64 kExpHalf = 256;
__device__ __forceinline__ bool x_in_win(const DDState &d, u64 e) {
  return e + kExpHalf >= d.cLast && e < d.cLast + kExpHalf;
}
__device__ __forceinline__ bool x_has(const DDState &d, int c, u64 e) {
  if (x_in_win(d, e)) return (d.exp[c][(e >> 6) & 7] >> (e & 63)) & 1u;
  return d.expFar[c] && d.exp[c][8] == e;
}
__device__ __forceinline__ void x_del(DDState &d, int c, u64 e) {
  if (x_in_win(d, e))
    d.exp[c][(e >> 6) & 7] &= ~(u64(1) << (e & 63));
  else if (d.expFar[c] && d.exp[c][8] == e)
    d.expFar[c] = 0;
}
__device__ __forceinline__ void x_clear(DDState &d, int c) {
  for (int w = 0; w < kDDExpWords; w++) d.exp[c][w] = 0;
  d.expFar[c] = 0;
}
__device__ __forceinline__ bool x_any(const DDState &d, int c) {
  u64 o = 0;
  for (int w = 0; w < kDDExpWords; w++) o |= d.exp[c][w];
  return o != 0 || d.expFar[c];
}
// any waited-on frame in [a, b) (frames outside the ring's window are not in it)
__device__ inline bool x_any_frames(const DDState &d, int c, u64 a, u64 b) {
  bool hit = d.expFar[c] && d.exp[c][8] >= a && d.exp[c][8] < b;
  const u64 lo = d.cLast >= kExpHalf ? d.cLast - kExpHalf : 0, hi = d.cLast + kExpHalf;
  a = a > lo ? a : lo;
  b = b < hi ? b : hi;
  while (!hit && a < b) {
    const u32 bit = u32(a & 63);
    const u64 n = (b - a) < u64(64 - bit) ? (b - a) : u64(64 - bit);
    const u64 m = (n >= 64 ? ~u64(0) : ((u64(1) << n) - 1)) << bit;
    hit = (d.exp[c][(a >> 6) & 7] & m) != 0;
    a += n;
  }
  return hit;
}
__device__ __forceinline__ u32 x_count(const DDState &d, int c) {
  u32 n = d.expFar[c] ? 1u : 0u;
  for (int w = 0; w < kDDExpWords; w++) n += u32(__popcll(d.exp[c][w]));
  return n;
}

// callbacks of frame e firing with decision sd (see the header comment)
__device__ inline void c_fire(DDState &d, u64 e, u32 sd) {
  for (int c = 0; c < d.numChains; c++) {
    if ((d.chBroken >> c) & 1) continue;
    if (!x_has(d, c, e)) continue;
    x_del(d, c, e);
    if (sd != SD_FORWARDED) {
      d.chBroken |= 1u << c;
      x_clear(d, c);
    }
  }
}
__device__ __forceinline__ void c_set(DDState &d, u64 e, u32 sd) {
  c_put(d, e, sd);
  if (sd != SD_UNKNOWN) c_fire(d, e, sd);
}
// GetDecision selectordecisioncache.go:78-94
__device__ inline u32 c_decision(const DDState &d, u64 e, bool &tooOld) {
  tooOld = false;
  if (!(d.flags & DS_CACHE_INIT) || e < d.cBase) return SD_MISSING;
  if (e > d.cLast) return SD_UNKNOWN;
  if (d.cLast - e >= kEntries) {
    tooOld = true;
    return SD_MISSING;
  }
  return c_get(d, e);
}
// addEntity :112-165
__device__ inline void c_add(DDState &d, u64 entity, u32 sd) {
  if (!(d.flags & DS_CACHE_INIT)) {
    d.flags |= DS_CACHE_INIT;
    d.cBase = d.cLast = entity;
    c_set(d, entity, sd);
    return;
  }
  if (entity <= d.cBase) return;
  if (entity <= d.cLast) {
    c_set(d, entity, sd);
    return;
  }
  // [last+1, entity) -> unknown (no callbacks); beyond 256 frames the ring is all unknown
  const u64 gap = entity - d.cLast - 1;
  if (gap >= kEntries) {
    for (int i = 0; i < 8; i++) d.masks[i] = ~u64(0);
  } else {
    for (u64 e = d.cLast + 1; e != entity; e++) c_put(d, e, SD_UNKNOWN);
  }
  u64 ms = d.cLast, me = entity;
  ms = ms > kNack + d.cBase ? ms - kNack : d.cBase;
  me = me > kNack + d.cBase ? me - kNack : d.cBase;
  if (me > ms) {
    // each ring slot is first visited within the first 256 frames of the
    // range; a later visit finds it missing already (not unknown)
    const u64 n = me - ms < kEntries ? me - ms : kEntries;
    for (u64 k = 0; k < n; k++)
      if (c_get(d, ms + k) == SD_UNKNOWN) c_set(d, ms + k, SD_MISSING);
  }
  c_set(d, entity, sd);
  const u64 l0 = d.cLast;
  // frames waited on that aged out of the window (e + 256 < cLast, i.e. the
  // frames [l0 - 256, entity - 256)): missing, which breaks the chain; then
  // the ring follows cLast and takes the frame registered beyond it
  const u64 a = l0 >= kExpHalf ? l0 - kExpHalf : 0, b = entity >= kExpHalf ? entity - kExpHalf : 0;
  for (int c = 0; c < d.numChains; c++) {
    if ((d.chBroken >> c) & 1) continue;
    bool hit = false;
    if (b > a) {
      if (b - a >= 2 * kExpHalf) {
        for (int w = 0; w < kDDExpWords; w++) hit = hit || d.exp[c][w] != 0;
      } else {
        u64 x = a;
        while (!hit && x < b) {
          const u32 bit = u32(x & 63);
          const u64 n = (b - x) < u64(64 - bit) ? (b - x) : u64(64 - bit);
          const u64 m = (n >= 64 ? ~u64(0) : ((u64(1) << n) - 1)) << bit;
          hit = (d.exp[c][(x >> 6) & 7] & m) != 0;
          x += n;
        }
      }
    }
    if (hit) {
      d.chBroken |= 1u << c;
      x_clear(d, c);
    }
  }
  d.cLast = entity;
  for (int c = 0; c < d.numChains; c++)
    if (d.expFar[c] && x_in_win(d, d.exp[c][8])) {
      const u64 e = d.exp[c][8];
      d.exp[c][(e >> 6) & 7] |= u64(1) << (e & 63);
      d.expFar[c] = 0;
    }
}
// ExpectDecision :96-110 + the chain's append
__device__ inline bool c_expect(DDState &d, int c, u64 e, bool &overflow) {
  if (!(d.flags & DS_CACHE_INIT) || e < d.cBase) return false;
  if (e < d.cLast && d.cLast - e >= kEntries) return false;
  if (x_in_win(d, e)) {
    d.exp[c][(e >> 6) & 7] |= u64(1) << (e & 63);
    return true;
  }
  // beyond the ring (this packet's frame number jumped ahead): one such frame
  // per chain until the packet's add moves cLast past it
  if (d.expFar[c] && d.exp[c][8] != e) {
    overflow = true;
    return true;
  }
  d.exp[c][8] = e;
  d.expFar[c] = 1;
  return true;
}

// FrameChain.OnFrame framechain.go:43-92
__device__ inline void chain_on_frame(DDState &d, int c, u64 efn, const DDPkt &p, bool &overflow) {
  if (!((d.chActive >> c) & 1)) return;
  if (p.nchain <= c) return;
  const u32 diff = dd_chain_diff(p, c);
  if (diff == 0) {
    d.chBroken &= ~(1u << c);
    x_clear(d, c);
    return;
  }
  if ((d.chBroken >> c) & 1) return;
  const u64 prev = efn - diff;
  bool tooOld;
  const u32 sd = c_decision(d, prev, tooOld);
  bool intact = false;
  if (sd == SD_FORWARDED)
    intact = true;
  else if (sd == SD_UNKNOWN)
    intact = c_expect(d, c, prev, overflow);
  if (!intact) d.chBroken |= 1u << c;
}

// updateDependencyStructure :363-392 (chains recreated: inactive, broken)
__device__ inline void update_structure(DDState &d, const DDStruct &s, u8 slot, u64 efn) {
  d.slot = slot;
  d.extKeyFrameNum = efn;
  d.flags |= DS_KF_VALID;
  d.numChains = s.numChains;
  d.chBroken = s.numChains >= 32 ? ~0u : (1u << s.numChains) - 1;
  d.chActive = 0;
  d.chUpdating = 0;
  for (int c = 0; c < kDDChains; c++) x_clear(d, c);
  d.numTargets = s.numDT;
  d.dtActive = 0;
}
// updateActiveDecodeTargets :394-408 (+ FrameChain.Begin/EndUpdateActive)
__device__ inline void update_active(DDState &d, const DDStruct &s, u32 mask) {
  d.chUpdating = 0;
  d.dtActive = 0;
  for (int i = 0; i < d.numTargets; i++) {
    const bool a = (mask >> s.dtTarget[i]) & 1;
    if (a) d.dtActive |= 1u << i;
    if (d.numChains > 0 && a) d.chUpdating |= 1u << s.protectedBy[s.dtTarget[i]];
  }
  for (int c = 0; c < d.numChains; c++) {
    const bool a = (d.chUpdating >> c) & 1, was = (d.chActive >> c) & 1;
    if (a == was) continue;
    if (!was) d.chBroken |= 1u << c;
    d.chActive = a ? d.chActive | (1u << c) : d.chActive & ~(1u << c);
  }
  d.chUpdating = 0;
}
// invalidateKeyFrame :410-416
__device__ inline void invalidate_keyframe(DDState &d) {
  d.flags &= ~u32(DS_KF_VALID);
  d.numChains = 0;
  d.numTargets = 0;
}
// FrameNumberWrapper.UpdateAndGet framenumberwrapper.go
__device__ inline u64 fn_update(DDState &d, u64 nw, bool updateOffset) {
  if (!(d.flags & DS_FN_INIT)) {
    d.fnLast = nw;
    d.flags |= DS_FN_INIT;
    return nw;
  }
  if (nw <= d.fnLast) return nw + d.fnOffset;
  if (updateOffset) {
    const u16 n16 = u16(nw + d.fnOffset), l16 = u16(d.fnLast + d.fnOffset);
    const u16 diff = u16(n16 - l16);
    if (diff > 0x8000 || (diff == 0x8000 && n16 <= l16)) d.fnOffset += u64(65535 - diff + 6000);
  }
  d.fnLast = nw;
  return nw + d.fnOffset;
}

struct SelResult {
  bool selected, relevant, switching, resuming, marker;
  int ddLen;  // marshalled bytes in the output buffer (selected only)
  bool limit;  // an engine limit was hit (a second frame beyond the expectation ring)
  u32 stagedSlot;  // the ring slot the LDS copy holds on return
};

// Select :65-355.  Layers are the DownTrack's Base layers (DTHot); structs is
// the track's structure ring; out receives the marshalled descriptor.
// (staged: an LDS copy of structure slot stagedSlot, read instead of the
// track's ring in HBM for that slot)
__device__ __attribute__((noinline)) SelResult dd_select(DDState &d, const DDStruct *structs, const DDPkt *pp, bool pktMarker,
                                      i32 &curS, i32 &curT, i32 &prevS, i32 &prevT, i32 tgtS, i32 tgtT, u8 *out,
                                      DDStruct *staged, u32 stagedSlot, const u16 *spill) {
  auto pick = [&](u32 slot) -> const DDStruct & { return slot == stagedSlot ? *staged : structs[slot]; };
  SelResult r = {false, false, false, false, false, 0, false, stagedSlot};
  if (curS != -1 && curT != -1) r.relevant = true;
  if (!pp) return r;  // (no descriptor)
  const DDPkt &p = *pp;
  const u64 efn = p.extFN;
  const bool attached = p.flags & DP_ATTACHED;
  if (!(d.flags & DS_KF_VALID) && !attached) return r;
  bool tooOld;
  const u32 sd = c_decision(d, efn, tooOld);
  if (tooOld || sd == SD_DROPPED) return r;
  if (p.extFlags & LKF_DD_STRUCTURE_UPDATED) update_structure(d, pick(p.slot), p.slot, efn);
  if (p.extKFN != d.extKeyFrameNum) {
    c_add(d, efn, SD_DROPPED);
    invalidate_keyframe(d);
    return r;
  }
  // the structure in force, in LDS: staged again when this descriptor moved
  // the DownTrack to another slot (so the selection and the marshal read LDS)
  if (u32(d.slot) != stagedSlot) {
    const u32 slot = d.slot, ln = threadIdx.x & 63u;
    const uint4 *gs = reinterpret_cast<const uint4 *>(structs + slot);
    uint4 *ls = reinterpret_cast<uint4 *>(staged);
    const u32 nT = structs[slot].numTmpl, nP = structs[slot].nfdPool;
    constexpr u32 kTOff = __builtin_offsetof(DDStruct, t) / 16, kPOff = __builtin_offsetof(DDStruct, fdPool) / 16;
    const u32 nHead = kTOff + nT * (sizeof(DDTmpl) / 16), nPool = (nP + 15) / 16;
    for (u32 i = ln; i < nHead + nPool; i += 64) {
      const u32 k = i < nHead ? i : kPOff + (i - nHead);
      ls[k] = gs[k];
    }
    stagedSlot = slot;
    r.stagedSlot = slot;
    __syncthreads();
  }
  const DDStruct &s = *staged;
  if (p.extFlags & LKF_DD_ACTIVE_UPDATED) update_active(d, s, p.activeMask);
  if (p.nchain != d.numChains) {
    c_add(d, efn, SD_DROPPED);
    return r;
  }
#if defined(LKF_SVC_STATS) && LKF_SVC_STATS
  const u64 tq0 = __builtin_amdgcn_s_memtime();
#endif
  for (int c = 0; c < d.numChains; c++) chain_on_frame(d, c, efn, p, r.limit);
#if defined(LKF_SVC_STATS) && LKF_SVC_STATS
  const u64 tq1 = __builtin_amdgcn_s_memtime();
#endif
  int hiPos = -1;
  u32 dti = 0;
  for (int i = 0; i < d.numTargets; i++) {
    if (!((d.dtActive >> i) & 1) || i32(s.dtS[i]) > tgtS || i32(s.dtT[i]) > tgtT) continue;
    const int target = s.dtTarget[i];
    if (p.ndti <= target) {  // DecodeTarget.OnFrame error
      c_add(d, efn, SD_DROPPED);
      return r;
    }
    const bool valid = d.numChains == 0 || !((d.chBroken >> s.protectedBy[target]) & 1);
    if (valid) {
      hiPos = i;
      dti = dti_at(p.dtis, target);
      break;
    }
  }
  if (hiPos < 0 || dti == 0) {
    c_add(d, efn, SD_DROPPED);
    return r;
  }
  const u8 *const ppool = pick(p.slot).fdPool;
  for (int i = 0; i < p.nfd; i++) {
    const u32 f = fd_at(p, ppool, spill, i);
    if (f == 0) continue;
    bool old;
    if (c_decision(d, efn - f, old) == SD_DROPPED) {
      c_add(d, efn, SD_DROPPED);
      return r;
    }
  }
  const i32 hs = s.dtS[hiPos], ht = s.dtT[hiPos];
  if (curS != hs || curT != ht) {
    r.switching = true;
    if (curS == -1 || curT == -1) r.resuming = true;
    prevS = curS;
    prevT = curT;
    curS = hs;
    curT = ht;
    if (d.flags & DS_HAS_MASK)
      d.flags |= DS_HAS_PREV_MASK;
    else
      d.flags &= ~u32(DS_HAS_PREV_MASK);
    d.prevMask = d.mask;
    d.flags |= DS_HAS_MASK;
    u32 m = 0;  // GetActiveDecodeTargetBitmask over ExtDependencyDescriptor.DecodeTargets (the parse-time structure)
    const DDStruct &ps = pick(p.slot);
    for (int i = 0; i < ps.numDT; i++)
      if (i32(ps.dtS[i]) <= curS && i32(ps.dtT[i]) <= curT) m |= 1u << ps.dtTarget[i];
    d.mask = m;
    r.relevant = true;
  }
  const u16 fn = u16(fn_update(d, efn, p.extFlags & LKF_DD_STRUCTURE_UPDATED));
  bool hasActive = p.flags & DP_ACTIVE;
  u32 active = p.activeMask;
  if (!attached && (d.flags & DS_HAS_MASK)) {
    hasActive = true;
    active = d.mask;
  }
#if defined(LKF_SVC_STATS) && LKF_SVC_STATS
  const u64 tq2 = __builtin_amdgcn_s_memtime();
#endif
  const int n = dd_marshal(s, p, fn, hasActive, active, out, ppool, spill, p.slot == d.slot,
                           LKF_DD_SER && attached ? structs + p.slot : nullptr);
#if defined(LKF_SVC_STATS) && LKF_SVC_STATS
  if ((threadIdx.x & 63) == 0) {  // g_svc[40..43]: chains, selection, marshal cycles, marshals
    SVC_ADD(40, tq1 - tq0);
    SVC_ADD(41, tq2 - tq1);
    SVC_ADD(42, __builtin_amdgcn_s_memtime() - tq2);
    SVC_ADD(43, 1ull);
    if (p.flags & DP_ATTACHED) {  // g_svc[44..45]: the marshals that write a structure
      SVC_ADD(44, __builtin_amdgcn_s_memtime() - tq2);
      SVC_ADD(45, 1ull);
    }
  }
#endif
  if (n < 0) {
    c_add(d, efn, SD_DROPPED);
    return r;
  }
  r.ddLen = n;
  if (p.extFlags & LKF_DD_INTEGRITY) c_add(d, efn, SD_FORWARDED);
  r.marker = pktMarker || ((p.flags & DP_LAST) && curS == i32(p.sid));
  r.selected = true;
  return r;
}

}  // namespace dd
}  // namespace lkf
