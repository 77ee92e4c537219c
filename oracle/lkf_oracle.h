// =============================================================================
//  lkf_oracle.h — TEST INFRASTRUCTURE ONLY.
//
//  Scalar C++17 restatement of the livekit-server v1.5.2 (reference at
//  /root/reference, Go) per-packet SFU hot path.  It is the CHECKER for the
//  MI355X engine (livekit-server_amd/csrc) and the CPU baseline of bench.py;
//  it is never linked into, loaded by, or called from the product path.
//
//  Every routine cites the Go function it restates (file:line relative to
//  /root/reference).  Deviations forced by the absence of the Go runtime:
//    * time.Now() is replaced by an explicit virtual clock (ns, int64): the
//      packet's arrival time wherever the reference reads the wall clock on
//      the forwarding path (processSourceSwitch, sequencer lastNack).
//    * logger calls are dropped (they have no effect on outputs).
//    * third-party code absent from /root/reference is restated from its
//      published behaviour and flagged "parity unpinned" where no reference
//      test pins it (pion/rtp header marshal, elliotchance/orderedmap v2.2.0
//      overwrite semantics, livekit/protocol utils.Bitmap).
//
//  Pinning: oracle/kat.cpp transcribes the reference's own unit tests for
//  these functions (rangemap_test.go, wraparound_test.go, rtpmunger_test.go,
//  codecmunger/vp8_test.go, buffer/helpers_test.go, forwarder_test.go
//  GetTranslationParams*, sequencer_test.go, audio/audiolevel_test.go,
//  buffer/rtpstats_receiver_test.go) as known-answer tests.
// =============================================================================
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <utility>
#include <array>
#include <vector>

namespace orc {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i8 = int8_t;
using i32 = int32_t;
using i64 = int64_t;

// Error values of the reference (pkg/sfu/downtrack.go:97-105,
// codecmunger/codecmunger.go:23-27, utils/rangemap.go:28-33,
// buffer/helpers.go:25-29).
enum Err : int {
  OK = 0,
  ErrUnknownKind,
  ErrOutOfOrderSequenceNumberCacheMiss,
  ErrPaddingOnlyPacket,
  ErrDuplicatePacket,
  ErrSequenceNumberOffsetNotFound,
  ErrPaddingNotOnFrameBoundary,
  ErrNotVP8,
  ErrOutOfOrderVP8PictureIdCacheMiss,
  ErrFilteredVP8TemporalLayer,
  ErrReversedOrder,
  ErrKeyNotFound,
  ErrKeyTooOld,
  ErrKeyExcluded,
  ErrShortPacket,
  ErrNilPacket,
  ErrInvalidPacket,
  ErrSwitchTooFarBehind,
  ErrRefLayerUnavailable,
  ErrExpectedTSUnavailable,
};

// -----------------------------------------------------------------------------
// utils.RangeMap — pkg/sfu/utils/rangemap.go:43-175
// -----------------------------------------------------------------------------
template <typename RT, typename VT>
struct RangeMap {
  struct RV {
    RT start;
    RT end;
    VT value;
  };
  RT halfRange;
  int size;
  std::vector<RV> ranges;

  // NewRangeMap rangemap.go:56-64
  explicit RangeMap(int sz = 1)
      : halfRange(RT(RT(1) << (sizeof(RT) * 8 - 1))), size(std::max(sz, 1)) {
    initRanges(0, 0);
  }
  // ClearAndResetValue rangemap.go:66-68
  void ClearAndResetValue(RT start, VT val) { initRanges(start, val); }
  // DecValue rangemap.go:70-88
  void DecValue(RT end, VT dec) {
    RV &lr = ranges.back();
    if (lr.start > end) {
      lr.value = VT(lr.value - dec);
      return;
    }
    lr.end = end;
    VT nv = VT(lr.value - dec);
    ranges.push_back(RV{RT(end + 1), RT(0), nv});
    prune();
  }
  // initRanges rangemap.go:90-98
  void initRanges(RT start, VT val) {
    ranges.clear();
    ranges.push_back(RV{start, RT(0), val});
  }
  // ExcludeRange rangemap.go:100-132
  Err ExcludeRange(RT s, RT e) {
    if (e == s || RT(e - s) > halfRange) return ErrReversedOrder;
    RV &lr = ranges.back();
    if (lr.start > s) return ErrReversedOrder;
    VT nv = VT(lr.value + VT(RT(e - s)));
    if (lr.start == s) {
      lr.start = e;
      lr.value = nv;
      return OK;
    }
    lr.end = RT(s - 1);
    ranges.push_back(RV{e, RT(0), nv});
    prune();
    return OK;
  }
  // GetValue rangemap.go:134-169
  Err GetValue(RT key, VT &out) const {
    out = 0;
    int n = (int)ranges.size();
    if (n != 0) {
      if (key >= ranges[n - 1].start) {
        out = ranges[n - 1].value;
        return OK;
      }
      if (key < ranges[0].start) return ErrKeyTooOld;
    }
    for (int idx = n - 1; idx >= 0; idx--) {
      const RV &rv = ranges[idx];
      if (idx != n - 1) {
        if (RT(key - rv.start) < halfRange && RT(rv.end - key) < halfRange) {
          out = rv.value;
          return OK;
        }
      }
      if (idx > 0) {
        const RV &prev = ranges[idx - 1];
        RT before = RT(key - prev.end);
        RT after = RT(rv.start - key);
        if (before > 0 && before < halfRange && after > 0 && after < halfRange) return ErrKeyExcluded;
      }
    }
    return ErrKeyNotFound;
  }
  // prune rangemap.go:171-175
  void prune() {
    if ((int)ranges.size() > size + 1) ranges.erase(ranges.begin(), ranges.end() - (size + 1));
  }
};

// -----------------------------------------------------------------------------
// utils.WrapAround — pkg/sfu/utils/wraparound.go:29-186
// -----------------------------------------------------------------------------
template <typename T, typename ET>
struct WrapAroundResult {
  bool IsUnhandled = false;
  bool IsRestart = false;
  ET PreExtendedStart = 0;
  ET PreExtendedHighest = 0;
  ET ExtendedVal = 0;
};

template <typename T, typename ET>
struct WrapAround {
  bool isRestartAllowed = false;
  ET fullRange = ET(ET(1) << (sizeof(T) * 8));
  bool initialized = false;
  T start = 0;
  T highest = 0;
  ET cycles = 0;
  ET extendedHighest = 0;

  explicit WrapAround(bool restartAllowed = false) : isRestartAllowed(restartAllowed) {}

  // Update wraparound.go:68-97
  WrapAroundResult<T, ET> Update(T val) {
    WrapAroundResult<T, ET> r;
    if (!initialized) {
      r.PreExtendedHighest = ET(ET(val) - 1);
      r.ExtendedVal = ET(val);
      start = val;
      highest = val;
      updateExtendedHighest();
      initialized = true;
      return r;
    }
    T gap = T(val - highest);
    if (gap > T(fullRange >> 1)) return maybeAdjustStart(val);
    r.PreExtendedHighest = extendedHighest;
    if (val < highest) cycles = ET(cycles + fullRange);
    highest = val;
    updateExtendedHighest();
    r.ExtendedVal = extendedHighest;
    return r;
  }
  // RollbackRestart wraparound.go:99-105
  void RollbackRestart(ET ev) {
    if (isWrapBack(start, T(ev))) {
      cycles = ET(cycles - fullRange);
      updateExtendedHighest();
    }
    start = T(ev);
  }
  // ResetHighest wraparound.go:107-111
  void ResetHighest(ET ev) {
    highest = T(ev);
    cycles = ET(ev & ~(fullRange - 1));
    updateExtendedHighest();
  }
  T GetStart() const { return start; }
  ET GetExtendedStart() const { return ET(start); }
  T GetHighest() const { return highest; }
  ET GetExtendedHighest() const { return extendedHighest; }
  void updateExtendedHighest() { extendedHighest = ET(cycles + ET(highest)); }

  // maybeAdjustStart wraparound.go:133-176
  WrapAroundResult<T, ET> maybeAdjustStart(T val) {
    WrapAroundResult<T, ET> r;
    ET cyc = cycles;
    ET totalNum = ET(GetExtendedHighest() - GetExtendedStart() + 1);
    if (totalNum > (fullRange >> 1)) {
      if (isWrapBack(val, highest)) cyc = ET(cyc - fullRange);
      r.PreExtendedHighest = extendedHighest;
      r.ExtendedVal = ET(cyc + ET(val));
      return r;
    }
    if (T(val - start) > T(fullRange >> 1)) {
      if (isRestartAllowed) {
        r.IsRestart = true;
        if (val > start)
          r.PreExtendedStart = ET(fullRange + ET(start));
        else
          r.PreExtendedStart = ET(start);
        if (isWrapBack(val, highest)) {
          cycles = fullRange;
          updateExtendedHighest();
          cyc = 0;
        }
        start = val;
      } else {
        r.IsUnhandled = true;
      }
    } else {
      if (isWrapBack(val, highest)) cyc = ET(cyc - fullRange);
    }
    r.PreExtendedHighest = extendedHighest;
    r.ExtendedVal = ET(cyc + ET(val));
    return r;
  }
  // isWrapBack wraparound.go:178-180
  bool isWrapBack(T earlier, T later) const {
    return ET(later) < (fullRange >> 1) && ET(earlier) >= (fullRange >> 1);
  }
};

// -----------------------------------------------------------------------------
// buffer.VideoLayer — pkg/sfu/buffer/videolayer.go:19-58
// -----------------------------------------------------------------------------
constexpr i32 InvalidLayerSpatial = -1;
constexpr i32 InvalidLayerTemporal = -1;
constexpr i32 DefaultMaxLayerSpatial = 2;
constexpr i32 DefaultMaxLayerTemporal = 3;

struct VideoLayer {
  i32 Spatial = InvalidLayerSpatial;
  i32 Temporal = InvalidLayerTemporal;
  bool operator==(const VideoLayer &o) const { return Spatial == o.Spatial && Temporal == o.Temporal; }
  bool operator!=(const VideoLayer &o) const { return !(*this == o); }
  bool GreaterThan(const VideoLayer &o) const {
    return Spatial > o.Spatial || (Spatial == o.Spatial && Temporal > o.Temporal);
  }
  bool IsValid() const { return Spatial != InvalidLayerSpatial && Temporal != InvalidLayerTemporal; }
};
inline VideoLayer InvalidLayer() { return VideoLayer{InvalidLayerSpatial, InvalidLayerTemporal}; }

}  // namespace orc
#include "dd_select_oracle.h"  // DD selector / parser (namespace orc; needs VideoLayer, WrapAround)
namespace orc {

// -----------------------------------------------------------------------------
// buffer.VP8 payload descriptor — pkg/sfu/buffer/helpers.go:49-241
// -----------------------------------------------------------------------------
struct VP8 {
  u8 FirstByte = 0;
  bool S = false;
  bool I = false;
  bool M = false;
  u16 PictureID = 0;
  bool L = false;
  u8 TL0PICIDX = 0;
  bool T = false;
  u8 TID = 0;
  bool Y = false;
  bool K = false;
  u8 KEYIDX = 0;
  int HeaderSize = 0;
  bool IsKeyFrame = false;

  bool operator==(const VP8 &o) const {
    return FirstByte == o.FirstByte && S == o.S && I == o.I && M == o.M && PictureID == o.PictureID &&
           L == o.L && TL0PICIDX == o.TL0PICIDX && T == o.T && TID == o.TID && Y == o.Y && K == o.K &&
           KEYIDX == o.KEYIDX && HeaderSize == o.HeaderSize && IsKeyFrame == o.IsKeyFrame;
  }

  // Unmarshal helpers.go:76-162
  Err Unmarshal(const u8 *payload, int payloadLen) {
    if (payload == nullptr) return ErrNilPacket;
    if (payloadLen < 1) return ErrShortPacket;
    int idx = 0;
    FirstByte = payload[idx];
    S = (payload[idx] & 0x10) > 0;
    if (payload[idx] & 0x80) {
      idx++;
      if (payloadLen < idx + 1) return ErrShortPacket;
      I = (payload[idx] & 0x80) > 0;
      L = (payload[idx] & 0x40) > 0;
      T = (payload[idx] & 0x20) > 0;
      K = (payload[idx] & 0x10) > 0;
      if (L && !T) return ErrInvalidPacket;
      if (I) {
        idx++;
        if (payloadLen < idx + 1) return ErrShortPacket;
        u8 pid = payload[idx] & 0x7f;
        M = (payload[idx] & 0x80) > 0;
        if (M) {
          idx++;
          if (payloadLen < idx + 1) return ErrShortPacket;
          PictureID = u16((u16(pid) << 8) | payload[idx]);
        } else {
          PictureID = pid;
        }
      }
      if (L) {
        idx++;
        if (payloadLen < idx + 1) return ErrShortPacket;
        TL0PICIDX = payload[idx];
      }
      if (T || K) {
        idx++;
        if (payloadLen < idx + 1) return ErrShortPacket;
        if (T) {
          TID = (payload[idx] & 0xc0) >> 6;
          Y = (payload[idx] & 0x20) > 0;
        }
        if (K) KEYIDX = payload[idx] & 0x1f;
      }
      idx++;
      if (payloadLen < idx + 1) return ErrShortPacket;
      IsKeyFrame = (payload[idx] & 0x01) == 0 && S;
    } else {
      idx++;
      if (payloadLen < idx + 1) return ErrShortPacket;
      IsKeyFrame = (payload[idx] & 0x01) == 0 && S;
    }
    HeaderSize = idx;
    return OK;
  }

  // Marshal / MarshalTo helpers.go:164-227.  Go panics on an index beyond
  // HeaderSize; we return ErrShortPacket instead (never reached on valid
  // munger output).
  Err Marshal(std::vector<u8> &out) const {
    out.assign(HeaderSize < 0 ? 0 : HeaderSize, 0);
    auto put = [&](int i, u8 v) -> bool {
      if (i >= (int)out.size()) return false;
      out[i] = v;
      return true;
    };
    auto orb = [&](int i, u8 v) -> bool {
      if (i >= (int)out.size()) return false;
      out[i] |= v;
      return true;
    };
    if (out.size() < 1) return ErrShortPacket;
    int idx = 0;
    out[idx] = FirstByte;
    if (I || L || T || K) {
      out[idx] |= 0x80;
      idx++;
      int xpos = idx;
      u8 xval = 0;
      idx++;
      if (I) {
        xval |= (1 << 7);
        if (M) {
          if (!put(idx, u8(0x80 | ((PictureID >> 8) & 0x7f)))) return ErrShortPacket;
          if (!put(idx + 1, u8(PictureID & 0xff))) return ErrShortPacket;
          idx += 2;
        } else {
          if (!put(idx, u8(PictureID))) return ErrShortPacket;
          idx++;
        }
      }
      if (L) {
        xval |= (1 << 6);
        if (!put(idx, TL0PICIDX)) return ErrShortPacket;
        idx++;
      }
      if (T || K) {
        if (!put(idx, 0)) return ErrShortPacket;
        if (T) {
          xval |= (1 << 5);
          out[idx] = u8(TID << 6);
          if (Y) out[idx] |= (1 << 5);
        }
        if (K) {
          xval |= (1 << 4);
          if (!orb(idx, KEYIDX & 0x1f)) return ErrShortPacket;
        }
        idx++;
      }
      if (!put(xpos, xval)) return ErrShortPacket;
    } else {
      out[idx] &= u8(~0x80);
      idx++;
    }
    return OK;
  }
};

// VPxPictureIdSizeDiff helpers.go:231-241
inline int VPxPictureIdSizeDiff(bool m1, bool m2) {
  if (m1 == m2) return 0;
  return m1 ? 1 : -1;
}

// -----------------------------------------------------------------------------
// rtp.Header (pion/rtp v1.8.3, go.mod:32) — the subset the hot path uses.
// Marshal restates pion's Header.MarshalTo (RFC 3550 / RFC 8285); no reference
// test pins wire bytes: PARITY UNPINNED for the extension block layout.
// -----------------------------------------------------------------------------
struct RtpExt {
  u8 id;
  std::vector<u8> payload;
};

struct RtpHeader {
  u8 Version = 2;
  bool Padding = false;
  bool Extension = false;
  bool Marker = false;
  u8 PayloadType = 0;
  u16 SequenceNumber = 0;
  u32 Timestamp = 0;
  u32 SSRC = 0;
  std::vector<u32> CSRC;
  u16 ExtensionProfile = 0;
  std::vector<RtpExt> Extensions;

  // pion Header.SetExtension (one-byte 0xBEDE for payload <= 16, two-byte
  // 0x1000 for 17..255) — used by pacer/base.go:82,93.
  Err SetExtension(u8 id, const std::vector<u8> &payload) {
    if (Extension) {
      if (ExtensionProfile == 0xBEDE) {
        if (id < 1 || id > 14) return ErrInvalidPacket;
        if (payload.size() > 16) return ErrInvalidPacket;
      } else if (ExtensionProfile == 0x1000) {
        if (id < 1) return ErrInvalidPacket;
        if (payload.size() > 255) return ErrInvalidPacket;
      }
      for (auto &e : Extensions)
        if (e.id == id) {
          e.payload = payload;
          return OK;
        }
      Extensions.push_back(RtpExt{id, payload});
      return OK;
    }
    Extension = true;
    size_t n = payload.size();
    if (n <= 16)
      ExtensionProfile = 0xBEDE;
    else if (n < 256)
      ExtensionProfile = 0x1000;
    Extensions.push_back(RtpExt{id, payload});
    return OK;
  }

  int MarshalSize() const {
    int n = 12 + 4 * (int)CSRC.size();
    if (Extension) {
      int ext = 0;
      if (ExtensionProfile == 0xBEDE) {
        for (auto &e : Extensions) ext += 1 + (int)e.payload.size();
      } else if (ExtensionProfile == 0x1000) {
        for (auto &e : Extensions) ext += 2 + (int)e.payload.size();
      } else if (!Extensions.empty()) {
        ext += (int)Extensions[0].payload.size();
      }
      n += 4 + ((ext + 3) / 4) * 4;
    }
    return n;
  }

  void Marshal(std::vector<u8> &out) const {
    out.clear();
    out.push_back(u8((Version << 6) | (Padding ? 0x20 : 0) | (Extension ? 0x10 : 0) | (CSRC.size() & 0xf)));
    out.push_back(u8((Marker ? 0x80 : 0) | (PayloadType & 0x7f)));
    out.push_back(u8(SequenceNumber >> 8));
    out.push_back(u8(SequenceNumber));
    for (int s = 24; s >= 0; s -= 8) out.push_back(u8(Timestamp >> s));
    for (int s = 24; s >= 0; s -= 8) out.push_back(u8(SSRC >> s));
    for (u32 c : CSRC)
      for (int s = 24; s >= 0; s -= 8) out.push_back(u8(c >> s));
    if (Extension) {
      size_t hpos = out.size();
      out.push_back(u8(ExtensionProfile >> 8));
      out.push_back(u8(ExtensionProfile));
      out.push_back(0);
      out.push_back(0);
      size_t start = out.size();
      if (ExtensionProfile == 0xBEDE) {
        for (auto &e : Extensions) {
          out.push_back(u8((e.id << 4) | u8(u8(e.payload.size()) - 1)));
          out.insert(out.end(), e.payload.begin(), e.payload.end());
        }
      } else if (ExtensionProfile == 0x1000) {
        for (auto &e : Extensions) {
          out.push_back(e.id);
          out.push_back(u8(e.payload.size()));
          out.insert(out.end(), e.payload.begin(), e.payload.end());
        }
      } else if (!Extensions.empty()) {
        out.insert(out.end(), Extensions[0].payload.begin(), Extensions[0].payload.end());
      }
      size_t ext = out.size() - start;
      size_t rounded = ((ext + 3) / 4) * 4;
      out[hpos + 2] = u8((rounded / 4) >> 8);
      out[hpos + 3] = u8(rounded / 4);
      while (out.size() - start < rounded) out.push_back(0);
    }
  }
};

// -----------------------------------------------------------------------------
// codecs.VP9Packet.Unmarshal — github.com/pion/rtp v1.8.3 codecs/vp9_packet.go
// (third-party, absent from the reference tree: restated from its published
// descriptor layout — parity unpinned) and buffer.IsVP9KeyFrame
// helpers.go:317-336.
// -----------------------------------------------------------------------------
struct VP9Packet {
  bool I = false, P = false, L = false, F = false, B = false, E = false, V = false, Z = false;
  u16 PictureID = 0;
  u8 TID = 0, SID = 0, TL0PICIDX = 0;
  bool U = false, D = false;
  std::vector<u8> PDiff;
  size_t PayloadOff = 0;  // Payload = packet[PayloadOff:]

  Err Unmarshal(const u8 *pk, size_t n) {
    if (n < 1) return ErrShortPacket;
    I = pk[0] & 0x80;
    P = pk[0] & 0x40;
    L = pk[0] & 0x20;
    F = pk[0] & 0x10;
    B = pk[0] & 0x08;
    E = pk[0] & 0x04;
    V = pk[0] & 0x02;
    Z = pk[0] & 0x01;
    size_t pos = 1;
    if (I) {  // parsePictureID
      if (n <= pos) return ErrShortPacket;
      PictureID = u16(pk[pos] & 0x7F);
      if (pk[pos] & 0x80) {
        pos++;
        if (n <= pos) return ErrShortPacket;
        PictureID = u16((PictureID << 8) | pk[pos]);
      }
      pos++;
    }
    if (L) {  // parseLayerInfo: common, then non-flexible TL0PICIDX
      if (n <= pos) return ErrShortPacket;
      TID = pk[pos] >> 5;
      U = pk[pos] & 0x10;
      SID = (pk[pos] >> 1) & 0x7;
      D = pk[pos] & 0x01;
      if (SID >= 5) return ErrShortPacket;  // errTooManySpatialLayers
      pos++;
      if (!F) {
        if (n <= pos) return ErrShortPacket;
        TL0PICIDX = pk[pos];
        pos++;
      }
    }
    if (F && P) {  // parseRefIndices
      for (;;) {
        if (n <= pos) return ErrShortPacket;
        PDiff.push_back(pk[pos] >> 1);
        if ((pk[pos] & 0x01) == 0) break;
        if (PDiff.size() >= 3) return ErrShortPacket;  // errTooManyPDiff
        pos++;
      }
      pos++;
    }
    if (V) {  // parseSSData
      if (n <= pos) return ErrShortPacket;
      const size_t ns = size_t(pk[pos] >> 5) + 1;
      const bool Y = pk[pos] & 0x10, G = pk[pos] & 0x08;
      pos++;
      if (Y) {
        if (n <= pos + ns * 4 - 1) return ErrShortPacket;
        pos += ns * 4;
      }
      size_t ng = 0;
      if (G) {
        if (n <= pos) return ErrShortPacket;
        ng = pk[pos];
        pos++;
      }
      for (size_t i = 0; i < ng; i++) {
        if (n <= pos) return ErrShortPacket;
        const size_t r = (pk[pos] >> 2) & 0x3;
        pos++;
        if (n <= pos + r - 1) return ErrShortPacket;
        pos += r;
      }
    }
    PayloadOff = pos;
    return OK;
  }
  // IsVP9KeyFrame helpers.go:317-336 (re-parses the same payload)
  static bool IsKeyFrame(const u8 *pk, size_t n) {
    VP9Packet v;
    if (v.Unmarshal(pk, n) != OK || n - v.PayloadOff < 1) return false;
    if (!v.B) return false;
    const u8 h = pk[v.PayloadOff];
    if ((h & 0xc0) != 0x80) return false;
    const u8 profile = (h >> 4) & 0x3;
    if (profile != 3) return (h & 0xC) == 0;
    return (h & 0x6) == 0;
  }
};

// -----------------------------------------------------------------------------
// buffer.ExtPacket — pkg/sfu/buffer/buffer.go:54-64
// -----------------------------------------------------------------------------
enum PayloadKind : u8 { PayloadNone = 0, PayloadVP8 = 1, PayloadVP9 = 2 };

// codecs.VP9Packet (pion/rtp v1.8.3 codecs/vp9_packet.go): the flags the
// VP9 selector reads (videolayerselector/vp9.go:44-108).  SID/TID arrive as
// ExtPacket.VideoLayer (buffer.go:645-655).
struct VP9Flags {
  bool I = false, P = false, L = false, F = false, B = false, E = false, V = false, U = false;
};

struct ExtPacket {
  VideoLayer layer;  // ExtPacket.VideoLayer
  i64 Arrival = 0;   // virtual ns
  u64 ExtSequenceNumber = 0;
  u64 ExtTimestamp = 0;
  RtpHeader Header;
  std::vector<u8> Payload;  // rtp.Packet.Payload (padding excluded)
  u8 PaddingSize = 0;
  PayloadKind kind = PayloadNone;
  VP8 vp8;  // valid when kind == PayloadVP8
  VP9Flags vp9;  // valid when kind == PayloadVP9
  bool KeyFrame = false;
  std::shared_ptr<ExtDD> dd;  // ExtPacket.DependencyDescriptor (nil: no DD extension)
};

// -----------------------------------------------------------------------------
// RTPMunger — pkg/sfu/rtpmunger.go:26-358
// -----------------------------------------------------------------------------
enum SequenceNumberOrdering : int {
  SequenceNumberOrderingContiguous = 0,
  SequenceNumberOrderingOutOfOrder = 1,
  SequenceNumberOrderingGap = 2,
  SequenceNumberOrderingDuplicate = 3,
};
constexpr u64 RtxGateWindow = 2000;

struct TranslationParamsRTP {
  SequenceNumberOrdering snOrdering = SequenceNumberOrderingContiguous;
  u64 extSequenceNumber = 0;
  u64 extTimestamp = 0;
  bool operator==(const TranslationParamsRTP &o) const {
    return snOrdering == o.snOrdering && extSequenceNumber == o.extSequenceNumber && extTimestamp == o.extTimestamp;
  }
};

struct SnTs {
  u64 extSequenceNumber = 0;
  u64 extTimestamp = 0;
};

struct RTPMungerState {
  u64 ExtLastSN = 0, ExtSecondLastSN = 0, ExtLastTS = 0, ExtSecondLastTS = 0;
  bool LastMarker = false, SecondLastMarker = false;
};

struct RTPMunger {
  u64 extHighestIncomingSN = 0;
  RangeMap<u64, u64> snRangeMap{100};  // NewRTPMunger rtpmunger.go:94-99
  u64 extLastSN = 0, extSecondLastSN = 0, snOffset = 0;
  u64 extLastTS = 0, extSecondLastTS = 0, tsOffset = 0;
  bool lastMarker = false, secondLastMarker = false;
  u64 extRtxGateSn = 0;
  bool isInRtxGateRegion = false;

  RTPMungerState GetLast() const {  // rtpmunger.go:115-124
    return RTPMungerState{extLastSN, extSecondLastSN, extLastTS, extSecondLastTS, lastMarker, secondLastMarker};
  }
  void SeedLast(const RTPMungerState &s) {  // rtpmunger.go:126-133
    extLastSN = s.ExtLastSN;
    extSecondLastSN = s.ExtSecondLastSN;
    extLastTS = s.ExtLastTS;
    extSecondLastTS = s.ExtSecondLastTS;
    lastMarker = s.LastMarker;
    secondLastMarker = s.SecondLastMarker;
  }
  // SetLastSnTs rtpmunger.go:135-145
  void SetLastSnTs(const ExtPacket &p) {
    extHighestIncomingSN = p.ExtSequenceNumber - 1;
    extLastSN = p.ExtSequenceNumber;
    extSecondLastSN = extLastSN - 1;
    snRangeMap.ClearAndResetValue(p.ExtSequenceNumber, 0);
    updateSnOffset();
    extLastTS = p.ExtTimestamp;
    extSecondLastTS = p.ExtTimestamp;
  }
  // UpdateSnTsOffsets rtpmunger.go:147-154
  void UpdateSnTsOffsets(const ExtPacket &p, u64 snAdjust, u64 tsAdjust) {
    extHighestIncomingSN = p.ExtSequenceNumber - 1;
    snRangeMap.ClearAndResetValue(p.ExtSequenceNumber, p.ExtSequenceNumber - extLastSN - snAdjust);
    updateSnOffset();
    tsOffset = p.ExtTimestamp - extLastTS - tsAdjust;
  }
  // PacketDropped rtpmunger.go:156-181
  void PacketDropped(const ExtPacket &p) {
    if (extHighestIncomingSN != p.ExtSequenceNumber) return;
    (void)snRangeMap.ExcludeRange(extHighestIncomingSN, extHighestIncomingSN + 1);
    extLastSN = extSecondLastSN;
    updateSnOffset();
    extLastTS = extSecondLastTS;
    lastMarker = secondLastMarker;
  }
  // UpdateAndGetSnTs rtpmunger.go:183-271
  Err UpdateAndGetSnTs(const ExtPacket &p, bool marker, TranslationParamsRTP &tp) {
    tp = TranslationParamsRTP{};
    i64 diff = i64(p.ExtSequenceNumber - extHighestIncomingSN);
    if ((diff == 1 && !p.Payload.empty()) || diff > 1) {
      extHighestIncomingSN = p.ExtSequenceNumber;
      SequenceNumberOrdering ordering = diff > 1 ? SequenceNumberOrderingGap : SequenceNumberOrderingContiguous;
      u64 extMungedSN = p.ExtSequenceNumber - snOffset;
      u64 extMungedTS = p.ExtTimestamp - tsOffset;
      extSecondLastSN = extLastSN;
      extLastSN = extMungedSN;
      extSecondLastTS = extLastTS;
      extLastTS = extMungedTS;
      secondLastMarker = lastMarker;
      lastMarker = marker;
      if (p.KeyFrame) {
        extRtxGateSn = extMungedSN;
        isInRtxGateRegion = true;
      }
      if (isInRtxGateRegion && (extMungedSN - extRtxGateSn) > RtxGateWindow) isInRtxGateRegion = false;
      tp.snOrdering = ordering;
      tp.extSequenceNumber = extMungedSN;
      tp.extTimestamp = extMungedTS;
      return OK;
    }
    if (diff < 0) {
      u64 off = 0;
      if (snRangeMap.GetValue(p.ExtSequenceNumber, off) != OK) {
        tp.snOrdering = SequenceNumberOrderingOutOfOrder;
        return ErrOutOfOrderSequenceNumberCacheMiss;
      }
      u64 esn = p.ExtSequenceNumber - off;
      if (esn >= extLastSN) {
        tp.snOrdering = SequenceNumberOrderingOutOfOrder;
        return ErrOutOfOrderSequenceNumberCacheMiss;
      }
      tp.snOrdering = SequenceNumberOrderingOutOfOrder;
      tp.extSequenceNumber = esn;
      tp.extTimestamp = p.ExtTimestamp - tsOffset;
      return OK;
    }
    if (diff == 1) {
      extHighestIncomingSN = p.ExtSequenceNumber;
      (void)snRangeMap.ExcludeRange(extHighestIncomingSN, extHighestIncomingSN + 1);
      updateSnOffset();
      tp.snOrdering = SequenceNumberOrderingContiguous;
      return ErrPaddingOnlyPacket;
    }
    tp.snOrdering = SequenceNumberOrderingDuplicate;
    return ErrDuplicatePacket;
  }
  // FilterRTX rtpmunger.go:273-286
  std::vector<u16> FilterRTX(const std::vector<u16> &nacks) const {
    if (!isInRtxGateRegion) return nacks;
    std::vector<u16> f;
    for (u16 sn : nacks)
      if (u16(sn - u16(extRtxGateSn)) < (1 << 15)) f.push_back(sn);
    return f;
  }
  // UpdateAndGetPaddingSnTs rtpmunger.go:288-346
  Err UpdateAndGetPaddingSnTs(int num, u32 clockRate, u32 frameRate, bool forceMarker, u64 extRtpTimestamp,
                              std::vector<SnTs> &vals) {
    vals.clear();
    if (num == 0) return OK;
    bool useLastTSForFirst = false;
    int tsOff = 0;
    if (!lastMarker) {
      if (!forceMarker) return ErrPaddingNotOnFrameBoundary;
      useLastTSForFirst = true;
      tsOff = 1;
    }
    u64 eLastSN = extLastSN;
    u64 eLastTS = extLastTS;
    vals.assign(num, SnTs{});
    for (int i = 0; i < num; i++) {
      eLastSN++;
      vals[i].extSequenceNumber = eLastSN;
      if (frameRate != 0) {
        if (useLastTSForFirst && i == 0) {
          vals[i].extTimestamp = extLastTS;
        } else {
          u64 ets = extRtpTimestamp + u64((u32(u32(i + 1 - tsOff) * clockRate) + frameRate - 1) / frameRate);
          if (i64(ets - eLastTS) <= 0) ets = eLastTS + 1;
          eLastTS = ets;
          vals[i].extTimestamp = ets;
        }
      } else {
        vals[i].extTimestamp = extLastTS;
      }
    }
    extSecondLastSN = eLastSN - 1;
    extLastSN = eLastSN;
    snRangeMap.DecValue(extHighestIncomingSN, u64(num));
    updateSnOffset();
    if (vals.size() == 1)
      extSecondLastTS = extLastTS;
    else
      extSecondLastTS = vals[vals.size() - 2].extTimestamp;
    tsOffset -= eLastTS - extLastTS;
    extLastTS = eLastTS;
    if (forceMarker) lastMarker = true;
    return OK;
  }
  bool IsOnFrameBoundary() const { return lastMarker; }
  // updateSnOffset rtpmunger.go:352-358 (error is logged; value stays 0)
  void updateSnOffset() {
    u64 v = 0;
    snRangeMap.GetValue(extHighestIncomingSN + 1, v);
    snOffset = v;
  }
};

// -----------------------------------------------------------------------------
// elliotchance/orderedmap/v2 v2.2.0 (go.mod:9), restated: insertion-ordered
// map; Set on an existing key replaces the value IN PLACE (position kept) —
// parity unpinned beyond vp8_test.go / forwarder_test.go sequences.
// -----------------------------------------------------------------------------
template <typename K, typename V>
struct OrderedMap {
  std::vector<std::pair<K, V>> kv;
  bool Get(K k, V &v) const {
    for (auto &e : kv)
      if (e.first == k) {
        v = e.second;
        return true;
      }
    return false;
  }
  bool Has(K k) const {
    for (auto &e : kv)
      if (e.first == k) return true;
    return false;
  }
  void Set(K k, V v) {
    for (auto &e : kv)
      if (e.first == k) {
        e.second = v;
        return;
      }
    kv.emplace_back(k, v);
  }
  int Len() const { return (int)kv.size(); }
  void PopFront() { kv.erase(kv.begin()); }
  void Clear() { kv.clear(); }
};

// -----------------------------------------------------------------------------
// codecmunger.VP8 — pkg/sfu/codecmunger/vp8.go:27-488
// -----------------------------------------------------------------------------
constexpr int missingPictureIdsThreshold = 50;
constexpr int droppedPictureIdsThreshold = 20;
constexpr int exemptedPictureIdsThreshold = 20;

struct VP8State {  // vp8.go:35-43
  i32 ExtLastPictureId = 0;
  bool PictureIdUsed = false;
  u8 LastTl0PicIdx = 0;
  bool Tl0PicIdxUsed = false;
  bool TidUsed = false;
  u8 LastKeyIdx = 0;
  bool KeyIdxUsed = false;
};

struct VP8PictureIdWrapHandler {  // vp8.go:373-488
  i32 maxPictureId = 0;
  bool maxMBit = false;
  i32 totalWrap = 0;
  i32 lastWrap = 0;
  static bool isWrapping7Bit(i32 v1, i32 v2) { return v2 < v1 && (v1 - v2) > (1 << 6); }
  static bool isWrapping15Bit(i32 v1, i32 v2) { return v2 < v1 && (v1 - v2) > (1 << 14); }
  void Init(i32 extPictureId, bool mBit) {
    maxPictureId = extPictureId;
    maxMBit = mBit;
    totalWrap = 0;
    lastWrap = 0;
  }
  i32 MaxPictureId() const { return maxPictureId; }
  // Unwrap vp8.go:400-483
  i32 Unwrap(u16 pictureId, bool mBit) {
    i32 mp = maxPictureId;
    if (mp > 0) mp = maxMBit ? (maxPictureId & 0x7fff) : (maxPictureId & 0x7f);
    i32 np = mBit ? i32(pictureId & 0x7fff) : i32(pictureId & 0x7f);
    if (totalWrap > 0) {
      if ((maxPictureId + (lastWrap >> 1)) < (np + totalWrap)) return np + totalWrap - lastWrap;
    }
    i32 wrap = 0;
    if (maxMBit) {
      if (isWrapping15Bit(mp, np)) wrap = 1 << 15;
    } else {
      if (isWrapping7Bit(mp, np)) wrap = 1 << 7;
    }
    totalWrap += wrap;
    if (wrap != 0) lastWrap = wrap;
    np += totalWrap;
    return np;
  }
  void UpdateMaxPictureId(i32 ext, bool mBit) {
    maxPictureId = ext;
    maxMBit = mBit;
  }
};

struct VP8Munger {
  VP8PictureIdWrapHandler pictureIdWrapHandler;
  i32 extLastPictureId = 0;
  i32 pictureIdOffset = 0;
  bool pictureIdUsed = false;
  u8 lastTl0PicIdx = 0;
  u8 tl0PicIdxOffset = 0;
  bool tl0PicIdxUsed = false;
  bool tidUsed = false;
  u8 lastKeyIdx = 0;
  u8 keyIdxOffset = 0;
  bool keyIdxUsed = false;
  OrderedMap<i32, i32> missingPictureIds;
  OrderedMap<i32, bool> droppedPictureIds;
  OrderedMap<i32, bool> exemptedPictureIds;

  VP8State GetState() const {  // vp8.go:87-97
    return VP8State{extLastPictureId, pictureIdUsed, lastTl0PicIdx, tl0PicIdxUsed, tidUsed, lastKeyIdx, keyIdxUsed};
  }
  void SeedState(const VP8State &s) {  // vp8.go:99-109
    extLastPictureId = s.ExtLastPictureId;
    pictureIdUsed = s.PictureIdUsed;
    lastTl0PicIdx = s.LastTl0PicIdx;
    tl0PicIdxUsed = s.Tl0PicIdxUsed;
    tidUsed = s.TidUsed;
    lastKeyIdx = s.LastKeyIdx;
    keyIdxUsed = s.KeyIdxUsed;
  }
  // SetLast vp8.go:111-134
  void SetLast(const ExtPacket &p) {
    if (p.kind != PayloadVP8) return;
    const VP8 &v = p.vp8;
    pictureIdUsed = v.I;
    if (pictureIdUsed) {
      pictureIdWrapHandler.Init(i32(v.PictureID) - 1, v.M);
      extLastPictureId = i32(v.PictureID);
    }
    tl0PicIdxUsed = v.L;
    if (tl0PicIdxUsed) lastTl0PicIdx = v.TL0PICIDX;
    tidUsed = v.T;
    keyIdxUsed = v.K;
    if (keyIdxUsed) lastKeyIdx = v.KEYIDX;
  }
  // UpdateOffsets vp8.go:136-159
  void UpdateOffsets(const ExtPacket &p) {
    if (p.kind != PayloadVP8) return;
    const VP8 &v = p.vp8;
    if (pictureIdUsed) {
      pictureIdWrapHandler.Init(i32(v.PictureID) - 1, v.M);
      pictureIdOffset = i32(v.PictureID) - extLastPictureId - 1;
    }
    if (tl0PicIdxUsed) tl0PicIdxOffset = u8(v.TL0PICIDX - lastTl0PicIdx - 1);
    if (keyIdxUsed) keyIdxOffset = u8((v.KEYIDX - lastKeyIdx - 1) & 0x1f);
    missingPictureIds.Clear();
    droppedPictureIds.Clear();
    exemptedPictureIds.Clear();
  }
  // UpdateAndGet vp8.go:161-302
  Err UpdateAndGet(const ExtPacket &p, bool snOutOfOrder, bool snHasGap, i32 maxTemporalLayer,
                   std::vector<u8> &out) {
    out.clear();
    if (p.kind != PayloadVP8) return ErrNotVP8;
    const VP8 &v = p.vp8;
    i32 extPictureId = pictureIdWrapHandler.Unwrap(v.PictureID, v.M);
    if (snOutOfOrder) {
      i32 off = 0;
      if (!missingPictureIds.Get(extPictureId, off)) return ErrOutOfOrderVP8PictureIdCacheMiss;
      u16 mpid = u16((extPictureId - off) & 0x7fff);
      VP8 o;
      o.FirstByte = v.FirstByte;
      o.I = v.I;
      o.M = mpid > 127;
      o.PictureID = mpid;
      o.L = v.L;
      o.TL0PICIDX = u8(v.TL0PICIDX - tl0PicIdxOffset);
      o.T = v.T;
      o.TID = v.TID;
      o.Y = v.Y;
      o.K = v.K;
      o.KEYIDX = u8(v.KEYIDX - keyIdxOffset);
      o.IsKeyFrame = v.IsKeyFrame;
      o.HeaderSize = v.HeaderSize + VPxPictureIdSizeDiff(mpid > 127, v.M);
      return o.Marshal(out);
    }
    i32 prevMaxPictureId = pictureIdWrapHandler.MaxPictureId();
    pictureIdWrapHandler.UpdateMaxPictureId(extPictureId, v.M);
    if (snHasGap) {
      for (i32 lost = prevMaxPictureId; lost <= extPictureId; lost++) {
        if (!droppedPictureIds.Has(lost)) missingPictureIds.Set(lost, pictureIdOffset);
      }
      while (missingPictureIds.Len() > missingPictureIdsThreshold) missingPictureIds.PopFront();
      if (v.T && v.TID > u8(maxTemporalLayer)) {
        exemptedPictureIds.Set(extPictureId, true);
        while (exemptedPictureIds.Len() > exemptedPictureIdsThreshold) exemptedPictureIds.PopFront();
      }
    } else {
      if (v.T && v.TID > u8(maxTemporalLayer)) {
        if (!exemptedPictureIds.Has(extPictureId)) {
          if (v.I && prevMaxPictureId != extPictureId) {
            droppedPictureIds.Set(extPictureId, true);
            while (droppedPictureIds.Len() > droppedPictureIdsThreshold) droppedPictureIds.PopFront();
            pictureIdOffset += 1;
          }
          return ErrFilteredVP8TemporalLayer;
        }
      }
    }
    i32 extMungedPictureId = extPictureId - pictureIdOffset;
    u16 mpid = u16(extMungedPictureId & 0x7fff);
    u8 mtl0 = u8(v.TL0PICIDX - tl0PicIdxOffset);
    u8 mkey = u8((v.KEYIDX - keyIdxOffset) & 0x1f);
    extLastPictureId = extMungedPictureId;
    lastTl0PicIdx = mtl0;
    lastKeyIdx = mkey;
    VP8 o;
    o.FirstByte = v.FirstByte;
    o.I = v.I;
    o.M = mpid > 127;
    o.PictureID = mpid;
    o.L = v.L;
    o.TL0PICIDX = mtl0;
    o.T = v.T;
    o.TID = v.TID;
    o.Y = v.Y;
    o.K = v.K;
    o.KEYIDX = mkey;
    o.IsKeyFrame = v.IsKeyFrame;
    o.HeaderSize = v.HeaderSize + VPxPictureIdSizeDiff(mpid > 127, v.M);
    return o.Marshal(out);
  }
  // UpdateAndGetPadding vp8.go:304-363
  Err UpdateAndGetPadding(bool newPicture, std::vector<u8> &out) {
    int offset = newPicture ? 1 : 0;
    int headerSize = 1;
    if (pictureIdUsed || tl0PicIdxUsed || tidUsed || keyIdxUsed) headerSize += 1;
    i32 extPictureId = extLastPictureId;
    if (pictureIdUsed) {
      extPictureId = extLastPictureId + offset;
      extLastPictureId = extPictureId;
      pictureIdOffset -= offset;
      headerSize += ((extPictureId & 0x7fff) > 127) ? 2 : 1;
    }
    u16 pictureId = u16(extPictureId & 0x7fff);
    u8 tl0 = 0;
    if (tl0PicIdxUsed) {
      tl0 = u8(lastTl0PicIdx + offset);
      lastTl0PicIdx = tl0;
      tl0PicIdxOffset = u8(tl0PicIdxOffset - offset);
      headerSize += 1;
    }
    if (tidUsed || keyIdxUsed) headerSize += 1;
    u8 keyIdx = 0;
    if (keyIdxUsed) {
      keyIdx = u8((lastKeyIdx + offset) & 0x1f);
      lastKeyIdx = keyIdx;
      keyIdxOffset = u8(keyIdxOffset - offset);
    }
    VP8 o;
    o.FirstByte = 0x10;
    o.I = pictureIdUsed;
    o.M = pictureId > 127;
    o.PictureID = pictureId;
    o.L = tl0PicIdxUsed;
    o.TL0PICIDX = tl0;
    o.T = tidUsed;
    o.TID = 0;
    o.Y = true;
    o.K = keyIdxUsed;
    o.KEYIDX = keyIdx;
    o.IsKeyFrame = true;
    o.HeaderSize = headerSize;
    return o.Marshal(out);
  }
};

// -----------------------------------------------------------------------------
// VideoLayerSelector — pkg/sfu/videolayerselector/{base,null,simulcast}.go,
// temporallayerselector/vp8.go.  (VP9 / dependency-descriptor selectors are a
// later round.)
// -----------------------------------------------------------------------------
struct VideoLayerSelectorResult {  // videolayerselector.go:8-15
  bool IsSelected = false;
  bool IsRelevant = false;
  bool IsSwitching = false;
  bool IsResuming = false;
  bool RTPMarker = false;
  std::vector<u8> DependencyDescriptorExtension;  // nil unless the DD selector marshalled one
};

enum VLSKind : u8 { VLSNull = 0, VLSSimulcast = 1, VLSVP9 = 2, VLSDD = 3 };

struct VLS {
  VLSKind kind = VLSNull;
  bool tlsVP8 = false;  // temporallayerselector.VP8 attached
  VideoLayer maxLayer, maxSeenLayer, targetLayer, previousTargetLayer;
  i32 requestSpatial = InvalidLayerSpatial;
  VideoLayer currentLayer, previousLayer;
  std::shared_ptr<DDSelectorState> dd;  // kind == VLSDD (videolayerselector/dependencydescriptor.go)

  void SetMax(VideoLayer l) { maxLayer = l; }
  void SetMaxSpatial(i32 l) { maxLayer.Spatial = l; }
  void SetMaxTemporal(i32 l) { maxLayer.Temporal = l; }
  VideoLayer GetMax() const { return maxLayer; }
  void SetTarget(VideoLayer l) {  // base.go SetTarget
    previousTargetLayer = l;
    targetLayer = l;
  }
  VideoLayer GetTarget() const { return targetLayer; }
  void SetRequestSpatial(i32 l) { requestSpatial = l; }
  void SetMaxSeen(VideoLayer l) { maxSeenLayer = l; }
  void SetMaxSeenSpatial(i32 l) { maxSeenLayer.Spatial = l; }
  void SetMaxSeenTemporal(i32 l) { maxSeenLayer.Temporal = l; }
  VideoLayer GetMaxSeen() const { return maxSeenLayer; }
  void SetCurrent(VideoLayer l) { currentLayer = l; }
  VideoLayer GetCurrent() const { return currentLayer; }
  void Rollback() {  // base.go Rollback; DependencyDescriptor.Rollback dependencydescriptor.go:357-361
    if (kind == VLSDD) {
      dd->hasMask = dd->hasPrevMask;
      dd->mask = dd->prevMask;
    }
    currentLayer = previousLayer;
    targetLayer = previousTargetLayer;
  }
  std::pair<bool, i32> CheckSync() const {
    if (kind == VLSDD) {  // dependencydescriptor.go:418-434
      const i32 layer = requestSpatial;
      if (!currentLayer.IsValid() || !dd->keyFrameValid) return {false, layer};
      for (auto &t : dd->decodeTargets)
        if (t.Active() && t.dt.Layer.Spatial == layer && t.Valid()) return {true, layer};
      return {false, layer};
    }
    return {requestSpatial == currentLayer.Spatial, requestSpatial};
  }

  // DependencyDescriptor.Select videolayerselector/dependencydescriptor.go:65-355
  VideoLayerSelectorResult SelectDD(const ExtPacket &p) {
    VideoLayerSelectorResult r;
    DDSelectorState &d = *dd;
    if (currentLayer.IsValid()) r.IsRelevant = true;
    if (!p.dd) return r;
    const ExtDD &w = *p.dd;
    const orc_dd::Descriptor &desc = *w.Descriptor;
    const u64 efn = w.ExtFrameNum;
    const orc_dd::Template &fd = desc.FrameDependencies;
    if (!d.keyFrameValid && !desc.AttachedStructure) return r;
    bool tooOld = false;
    const SelectorDecision sd = d.decisions.GetDecision(efn, &tooOld);
    if (tooOld) return r;
    if (sd == SDDropped) return r;
    if (w.StructureUpdated) d.updateDependencyStructure(desc.AttachedStructure, w.DecodeTargets, efn);
    if (w.ExtKeyFrameNum != d.extKeyFrameNum) {
      d.decisions.AddDropped(efn);
      d.invalidateKeyFrame();
      return r;
    }
    if (w.ActiveDecodeTargetsUpdated) d.updateActiveDecodeTargets(desc.ActiveDecodeTargetsBitmask);
    if (fd.ChainDiffs.size() != d.chains.size()) {
      d.decisions.AddDropped(efn);
      return r;
    }
    for (auto &c : d.chains) c->OnFrame(efn, fd);
    DDDecodeTarget hi;
    hi.Target = -1;
    int dti = 0;
    for (auto &t : d.decodeTargets) {
      if (!t.Active() || t.dt.Layer.Spatial > targetLayer.Spatial || t.dt.Layer.Temporal > targetLayer.Temporal)
        continue;
      bool tv = false;
      int x = 0;
      if (!t.OnFrame(efn, fd, tv, x)) {
        d.decisions.AddDropped(efn);
        return r;
      }
      if (tv) {
        hi = t.dt;
        dti = x;
        break;
      }
    }
    if (hi.Target < 0 || dti == 0) {  // no decode target / DecodeTargetNotPresent
      d.decisions.AddDropped(efn);
      return r;
    }
    for (int fdiff : fd.FrameDiffs) {
      if (fdiff == 0) continue;
      if (d.decisions.GetDecision(efn - u64(fdiff)) == SDDropped) {
        d.decisions.AddDropped(efn);
        return r;
      }
    }
    if (currentLayer != hi.Layer) {
      r.IsSwitching = true;
      if (!currentLayer.IsValid()) r.IsResuming = true;
      previousLayer = currentLayer;
      currentLayer = hi.Layer;
      d.hasPrevMask = d.hasMask;
      d.prevMask = d.mask;
      d.hasMask = true;
      d.mask = GetActiveDecodeTargetBitmask(currentLayer, w.DecodeTargets);
      r.IsRelevant = true;
    }
    orc_dd::Descriptor out = desc;  // the (shallow) clone of :301/:312
    const u16 unwrapFn = u16(d.fnWrapper.UpdateAndGet(efn, w.StructureUpdated));
    if (unwrapFn != desc.FrameNumber) out.FrameNumber = unwrapFn;
    if (!desc.AttachedStructure && d.hasMask) {
      out.hasActiveMask = true;
      out.ActiveDecodeTargetsBitmask = d.mask;
    }
    std::vector<u8> bytes;
    if (orc_dd::Marshal(d.structure.get(), out, ~0u, bytes) != orc_dd::DD_OK) {  // error or recovered panic
      d.decisions.AddDropped(efn);
      return r;
    }
    r.DependencyDescriptorExtension = bytes;
    if (w.Integrity) d.decisions.AddForwarded(efn);
    r.RTPMarker = p.Header.Marker || (desc.LastPacketInFrame && currentLayer.Spatial == fd.SpatialId);
    r.IsSelected = true;
    return r;
  }

  // VP9.Select videolayerselector/vp9.go:43-109 (SVC: every layer in one
  // stream; a packet is selected unless its layer is above the current one)
  VideoLayerSelectorResult SelectVP9(const ExtPacket &p) {
    VideoLayerSelectorResult r;
    if (p.kind != PayloadVP9) return r;
    const VP9Flags &v = p.vp9;
    VideoLayer cur = currentLayer;
    if (currentLayer != targetLayer) {
      VideoLayer upd = currentLayer;
      if (!currentLayer.IsValid()) {
        if (!p.KeyFrame) return r;
        upd = p.layer;
      } else {
        if (currentLayer.Temporal != targetLayer.Temporal) {
          if (currentLayer.Temporal < targetLayer.Temporal) {
            if (p.layer.Temporal > currentLayer.Temporal && p.layer.Temporal <= targetLayer.Temporal && v.U && v.B) {
              cur.Temporal = p.layer.Temporal;
              upd.Temporal = p.layer.Temporal;
            }
          } else if (v.E) {
            upd.Temporal = targetLayer.Temporal;
          }
        }
        if (currentLayer.Spatial != targetLayer.Spatial) {
          if (currentLayer.Spatial < targetLayer.Spatial) {
            if (p.layer.Spatial > currentLayer.Spatial && p.layer.Spatial <= targetLayer.Spatial && !v.P && v.B) {
              cur.Spatial = p.layer.Spatial;
              upd.Spatial = p.layer.Spatial;
            }
          } else if (v.E) {
            upd.Spatial = targetLayer.Spatial;
          }
        }
      }
      if (upd != currentLayer) {
        r.IsSwitching = true;
        if (!currentLayer.IsValid() && upd.IsValid()) r.IsResuming = true;
        previousLayer = currentLayer;
        currentLayer = upd;
      }
    }
    r.RTPMarker = p.Header.Marker;
    if (v.E && p.layer.Spatial == cur.Spatial && (v.P || targetLayer.Spatial <= currentLayer.Spatial))
      r.RTPMarker = true;
    r.IsSelected = !p.layer.GreaterThan(cur);
    r.IsRelevant = true;
    return r;
  }

  // Select: Base/Null base.go (zero result), Simulcast simulcast.go:42-122, VP9 vp9.go:43-109
  VideoLayerSelectorResult Select(const ExtPacket &p, i32 layer) {
    VideoLayerSelectorResult r;
    if (kind == VLSVP9) return SelectVP9(p);
    if (kind == VLSDD) return SelectDD(p);
    if (kind != VLSSimulcast) return r;
    if (currentLayer.Spatial != targetLayer.Spatial) {
      VideoLayer cur = currentLayer;
      bool isActive = currentLayer.IsValid();
      bool found = false;
      if (p.KeyFrame) {
        if (layer > currentLayer.Spatial && layer <= targetLayer.Spatial) found = true;
        if (layer < currentLayer.Spatial && layer >= targetLayer.Spatial) found = true;
        if (found) {
          cur.Spatial = layer;
          cur.Temporal = p.layer.Temporal;
        }
      }
      if (found) {
        previousLayer = currentLayer;
        currentLayer = cur;
        previousTargetLayer = targetLayer;
        if (currentLayer.Spatial >= maxLayer.Spatial || currentLayer.Spatial == maxSeenLayer.Spatial)
          targetLayer.Spatial = currentLayer.Spatial;
        r.IsSwitching = true;
        if (!isActive) r.IsResuming = true;
      }
    }
    if (currentLayer.Spatial > maxLayer.Spatial && layer <= maxLayer.Spatial && p.KeyFrame) {
      previousLayer = currentLayer;
      currentLayer.Spatial = layer;
      previousTargetLayer = targetLayer;
      if (currentLayer.Spatial >= maxLayer.Spatial || currentLayer.Spatial == maxSeenLayer.Spatial)
        targetLayer.Spatial = layer;
      r.IsSwitching = true;
    }
    r.RTPMarker = p.Header.Marker;
    r.IsSelected = layer == currentLayer.Spatial;
    r.IsRelevant = false;
    return r;
  }

  // SelectTemporal base.go:143-168 + temporallayerselector/vp8.go:32-56
  std::pair<i32, bool> SelectTemporal(const ExtPacket &p) {
    if (!tlsVP8) return {currentLayer.Temporal, false};
    i32 current = currentLayer.Temporal, target = targetLayer.Temporal;
    i32 thisL = current, next = current;
    if (current != target && p.kind == PayloadVP8 && p.vp8.T) {
      i32 tid = i32(p.vp8.TID);
      if (current < target) {
        if (tid > current && tid <= target && p.vp8.S && p.vp8.Y) {
          thisL = tid;
          next = tid;
        }
      } else {
        if (p.Header.Marker) next = target;
      }
    }
    bool isSwitching = false;
    if (next != currentLayer.Temporal) {
      isSwitching = true;
      previousLayer = currentLayer;
      currentLayer.Temporal = next;
    }
    return {thisL, isSwitching};
  }
};

// -----------------------------------------------------------------------------
// Forwarder (per-packet half) — pkg/sfu/forwarder.go
// -----------------------------------------------------------------------------
constexpr bool FlagPauseOnDowngrade = true;  // forwarder.go:40
constexpr double ResumeBehindThresholdSeconds = 0.2;
constexpr double ResumeBehindHighTresholdSeconds = 2.0;
constexpr double LayerSwitchBehindThresholdSeconds = 0.05;
constexpr double SwitchAheadThresholdSeconds = 0.025;

enum Kind : u8 { KindAudio = 0, KindVideo = 1 };
enum Mime : u8 { MimeNone = 0, MimeOpus = 1, MimeVP8 = 2, MimeH264 = 3, MimeVP9 = 4, MimeAV1 = 5 };

struct TranslationParams {  // forwarder.go:146-154
  bool shouldDrop = false;
  bool isResuming = false;
  bool isSwitching = false;
  bool hasRTP = false;
  TranslationParamsRTP rtp;
  std::vector<u8> codecBytes;
  std::vector<u8> ddBytes;  // tp.ddBytes forwarder.go:1706
  bool marker = false;
  int dropReason = -1;  // engine statistic only (lkf_drop); not part of equality
  bool operator==(const TranslationParams &o) const {
    return shouldDrop == o.shouldDrop && isResuming == o.isResuming && isSwitching == o.isSwitching &&
           hasRTP == o.hasRTP && (!hasRTP || rtp == o.rtp) && codecBytes == o.codecBytes && ddBytes == o.ddBytes &&
           marker == o.marker;
  }
};

struct ForwarderState {  // forwarder.go:158-166
  bool Started = false;
  i32 ReferenceLayerSpatial = 0;
  i64 PreStartTime = 0;  // ns, 0 == time.Time{}
  u64 ExtFirstTS = 0;
  u64 RefTSOffset = 0;
  RTPMungerState RTP;
  bool HasVP8 = false;
  VP8State Codec;
};

// VideoAllocation forwarder.go:82-93 (Bitrates [spatial][temporal], bps)
using Bitrates = std::array<std::array<i64, 4>, 3>;
enum VideoPauseReason : i32 { PauseNone = 0, PauseMuted, PausePubMuted, PauseFeedDry, PauseBandwidth };
constexpr i32 TransitionCostSpatial = 10;  // forwarder.go:43
struct VideoAllocation {
  i32 PauseReason = PauseNone;
  bool IsDeficient = false;
  i64 BandwidthRequested = 0, BandwidthDelta = 0, BandwidthNeeded = 0;
  Bitrates Brs{};
  VideoLayer TargetLayer{0, 0};
  i32 RequestLayerSpatial = 0;
  VideoLayer MaxLayer{0, 0};
  double DistanceToDesired = 0;
};
inline VideoAllocation VideoAllocationDefault() {  // forwarder.go:111-116
  VideoAllocation a;
  a.PauseReason = PauseFeedDry;
  a.TargetLayer = InvalidLayer();
  a.RequestLayerSpatial = InvalidLayerSpatial;
  a.MaxLayer = InvalidLayer();
  return a;
}
// getOptimalBandwidthNeeded forwarder.go:1857-1878
inline i64 getOptimalBandwidthNeeded(bool muted, bool pubMuted, i32 maxPublishedLayer, const Bitrates &brs,
                                     VideoLayer maxLayer) {
  if (muted || pubMuted || maxPublishedLayer == InvalidLayerSpatial) return 0;
  for (i32 i = maxLayer.Spatial; i >= 0; i--)
    for (i32 j = maxLayer.Temporal; j >= 0; j--)
      if (brs[i][j] != 0) return brs[i][j];
  return 0;
}
// getBandwidthNeeded forwarder.go:1880-1886
inline i64 getBandwidthNeeded(const Bitrates &brs, VideoLayer layer, i64 fallback) {
  if (layer.IsValid() && brs[layer.Spatial][layer.Temporal] > 0) return brs[layer.Spatial][layer.Temporal];
  return fallback;
}
// getDistanceToDesired forwarder.go:1888-1973
inline double getDistanceToDesired(bool muted, bool pubMuted, VideoLayer maxSeenLayer,
                                   const std::vector<i32> &availableLayers, const Bitrates &brs,
                                   VideoLayer targetLayer, VideoLayer maxLayer) {
  if (muted || pubMuted || !maxSeenLayer.IsValid() || !maxLayer.IsValid()) return 0.0;
  VideoLayer adj = maxLayer;
  i32 maxAvailS = InvalidLayerSpatial, maxAvailT = InvalidLayerTemporal;
  for (i32 s = 2; s >= 0 && maxAvailS == InvalidLayerSpatial; s--)
    for (i32 t = 3; t >= 0; t--)
      if (brs[s][t] != 0) {
        maxAvailS = s;
        break;
      }
  for (i32 l : availableLayers)
    if (l > maxAvailS) {
      maxAvailS = l;
      maxAvailT = maxSeenLayer.Temporal;
    }
  if (maxAvailS < adj.Spatial) adj.Spatial = maxAvailS;
  if (maxSeenLayer.Spatial < adj.Spatial) adj.Spatial = maxSeenLayer.Spatial;
  if (adj.Spatial != InvalidLayerSpatial)
    for (i32 t = 3; t >= 0; t--)
      if (brs[adj.Spatial][t] != 0) {
        maxAvailT = t;
        break;
      }
  if (maxAvailT < adj.Temporal) adj.Temporal = maxAvailT;
  if (maxSeenLayer.Temporal < adj.Temporal) adj.Temporal = maxSeenLayer.Temporal;
  if (!adj.IsValid()) adj = VideoLayer{0, 0};
  VideoLayer adjT = targetLayer;
  if (!targetLayer.IsValid()) adjT = VideoLayer{0, 0};
  i32 distance = ((adj.Spatial - adjT.Spatial) * (maxSeenLayer.Temporal + 1)) + (adj.Temporal - adjT.Temporal);
  if (!targetLayer.IsValid()) distance += (maxSeenLayer.Temporal + 1);
  return double(distance) / double(maxSeenLayer.Temporal + 1);
}

struct Forwarder {
  Kind kind;
  Mime mime = MimeNone;
  u32 clockRate = 0;
  // getReferenceLayerRTPTimestamp (forwarder.go:192): nullptr in the
  // reference tests; the engine harness feeds per-layer SR offsets
  // (streamtrackermanager.go:660-679).
  std::function<Err(u32 ts, i32 layer, i32 ref, u32 &out)> getReferenceLayerRTPTimestamp;
  // getExpectedRTPTimestamp (forwarder.go:193; downtrack.go:1765 ->
  // rtpstats_sender.go:581-594) evaluated on the virtual clock.
  std::function<Err(i64 at, u64 &out)> getExpectedRTPTimestamp;

  bool muted = false, pubMuted = false;
  double resumeBehindThreshold = 0.0;
  bool started = false;
  i64 preStartTime = 0;
  u64 extFirstTS = 0;
  u32 lastSSRC = 0;
  i32 referenceLayerSpatial = InvalidLayerSpatial;
  u64 refTSOffset = 0;
  bool lastAllocIsDeficient = false;  // lastAllocation.IsDeficient
  VideoAllocation lastAllocation = VideoAllocationDefault();  // (AllocateOptimal; IsDeficient above)
  RTPMunger rtpMunger;
  VLS vls;
  bool hasVP8Munger = false;
  VP8Munger vp8;

  // NewForwarder forwarder.go:217-239
  explicit Forwarder(Kind k) : kind(k) {
    if (kind == KindVideo) vls.SetMaxTemporal(DefaultMaxLayerTemporal);
  }
  // DetermineCodec forwarder.go:269-338; hasDD = the dependency-descriptor
  // extension is among the receiver's header extensions (ddAvailable :278-285)
  void DetermineCodec(Mime m, u32 cr, bool hasDD = false) {
    if (mime != MimeNone) return;
    mime = m;
    clockRate = cr;
    if ((m == MimeVP9 || m == MimeAV1) && hasDD) {  // NewDependencyDescriptor(FromNull)
      vls.kind = VLSDD;
      vls.dd = std::make_shared<DDSelectorState>();
      return;
    }
    if (m == MimeAV1) {  // AV1 without DD: Simulcast selector
      vls.kind = VLSSimulcast;
      return;
    }
    if (m == MimeVP8) {
      hasVP8Munger = true;  // NewVP8FromNull seeds from Null's (zero) state
      vls.kind = VLSSimulcast;
      vls.tlsVP8 = true;
    } else if (m == MimeH264) {
      vls.kind = VLSSimulcast;
    } else if (m == MimeVP9) {  // no dependency-descriptor extension negotiated: VP9 selector
      vls.kind = VLSVP9;
    }
  }
  // GetState / SeedState forwarder.go:340-375
  ForwarderState GetState() const {
    ForwarderState s;
    if (!started) return s;
    s.Started = started;
    s.ReferenceLayerSpatial = referenceLayerSpatial;
    s.PreStartTime = preStartTime;
    s.ExtFirstTS = extFirstTS;
    s.RefTSOffset = refTSOffset;
    s.RTP = rtpMunger.GetLast();
    s.HasVP8 = hasVP8Munger;
    if (hasVP8Munger) s.Codec = vp8.GetState();
    return s;
  }
  void SeedState(const ForwarderState &s) {
    if (!s.Started) return;
    rtpMunger.SeedLast(s.RTP);
    if (hasVP8Munger && s.HasVP8) vp8.SeedState(s.Codec);
    started = true;
    referenceLayerSpatial = s.ReferenceLayerSpatial;
    preStartTime = s.PreStartTime;
    extFirstTS = s.ExtFirstTS;
    refTSOffset = s.RefTSOffset;
  }
  // Mute forwarder.go:377-413
  bool Mute(bool m, bool isSubscribeMutable) {
    if (muted == m) return false;
    if (m && !isSubscribeMutable) return false;
    muted = m;
    if (muted) resyncLocked();
    return true;
  }
  // PubMute forwarder.go:422-438
  bool PubMute(bool m) {
    if (pubMuted == m) return false;
    pubMuted = m;
    if (pubMuted) resyncLocked();
    return true;
  }
  // SetMaxSpatialLayer / SetMaxTemporalLayer forwarder.go:454-488
  bool SetMaxSpatialLayer(i32 l) {
    if (kind == KindAudio) return false;
    if (l == vls.GetMax().Spatial) return false;
    vls.SetMaxSpatial(l);
    return true;
  }
  bool SetMaxTemporalLayer(i32 l) {
    if (kind == KindAudio) return false;
    if (l == vls.GetMax().Temporal) return false;
    vls.SetMaxTemporal(l);
    return true;
  }
  // SetMaxPublishedLayer / SetMaxTemporalLayerSeen forwarder.go:241-267
  bool SetMaxPublishedLayer(i32 l) {
    if (l <= vls.GetMaxSeen().Spatial) return false;
    vls.SetMaxSeenSpatial(l);
    return true;
  }
  bool SetMaxTemporalLayerSeen(i32 l) {
    if (l <= vls.GetMaxSeen().Temporal) return false;
    vls.SetMaxSeenTemporal(l);
    return true;
  }
  // updateAllocation + setTargetLayer forwarder.go:1353-1382 (the fields the
  // per-packet half reads: IsDeficient, TargetLayer, RequestLayerSpatial)
  void SetAllocation(VideoLayer target, i32 requestSpatial, bool isDeficient) {
    if (target.IsValid() && mime == MimeH264) target.Temporal = 0;
    lastAllocIsDeficient = isDeficient;
    vls.SetTarget(target);
    vls.SetRequestSpatial(target.IsValid() ? requestSpatial : InvalidLayerSpatial);
    if (!vls.GetTarget().IsValid()) resyncLocked();
  }
  // VideoLayerSelector.IsOvershootOkay: Simulcast true (simulcast.go:38), the
  // base / VP9 / dependency-descriptor selectors false
  bool IsOvershootOkay() const { return vls.kind == VLSSimulcast; }
  // AllocateOptimal forwarder.go:591-725 (+ updateAllocation :1353-1373)
  VideoAllocation AllocateOptimal(const std::vector<i32> &availableLayers, const Bitrates &brs, bool allowOvershoot) {
    if (kind == KindAudio) return LastAllocation();
    const VideoLayer maxLayer = vls.GetMax(), maxSeenLayer = vls.GetMaxSeen(), currentLayer = vls.GetCurrent();
    const i32 requestSpatial = vls.requestSpatial;
    VideoAllocation alloc;
    alloc.PauseReason = PauseNone;
    alloc.Brs = brs;
    alloc.TargetLayer = InvalidLayer();
    alloc.RequestLayerSpatial = requestSpatial;
    alloc.MaxLayer = maxLayer;
    const i64 optimal = getOptimalBandwidthNeeded(muted, pubMuted, maxSeenLayer.Spatial, brs, maxLayer);
    if (optimal == 0) alloc.PauseReason = PauseFeedDry;
    alloc.BandwidthNeeded = optimal;
    auto getMaxTemporal = [&]() {
      i32 mt = maxLayer.Temporal;
      if (maxSeenLayer.Temporal != InvalidLayerTemporal && maxSeenLayer.Temporal < mt) mt = maxSeenLayer.Temporal;
      return mt;
    };
    if (!maxLayer.IsValid() || maxSeenLayer.Spatial == InvalidLayerSpatial) {
    } else if (muted) {
      alloc.PauseReason = PauseMuted;
    } else if (pubMuted) {
      alloc.PauseReason = PausePubMuted;
    } else {
      const i32 limit = std::min(maxLayer.Spatial, maxSeenLayer.Spatial);
      i32 highest = InvalidLayerSpatial, request = InvalidLayerSpatial;
      for (i32 al : availableLayers) {
        if (al > request && al <= limit) request = al;
        if (al > highest) highest = al;
      }
      if (request == InvalidLayerSpatial && highest != InvalidLayerSpatial && allowOvershoot && IsOvershootOkay())
        request = highest;
      if (currentLayer.IsValid()) {
        if ((request == requestSpatial && currentLayer.Spatial == requestSpatial) || request == InvalidLayerSpatial)
          alloc.TargetLayer = VideoLayer{currentLayer.Spatial, getMaxTemporal()};
        else
          alloc.TargetLayer = VideoLayer{request, getMaxTemporal()};
        alloc.RequestLayerSpatial = alloc.TargetLayer.Spatial;
      } else {  // opportunistic
        i32 maxSpatial = maxLayer.Spatial;
        if (allowOvershoot && IsOvershootOkay() && maxSeenLayer.Spatial > maxSpatial) maxSpatial = maxSeenLayer.Spatial;
        alloc.TargetLayer = VideoLayer{std::min(maxSeenLayer.Spatial, maxSpatial), getMaxTemporal()};
        alloc.RequestLayerSpatial = request == InvalidLayerSpatial ? limit : request;
      }
    }
    if (!alloc.TargetLayer.IsValid()) {
      alloc.TargetLayer = InvalidLayer();
      alloc.RequestLayerSpatial = InvalidLayerSpatial;
    }
    if (alloc.TargetLayer.IsValid()) alloc.BandwidthRequested = optimal;
    alloc.BandwidthDelta =
        alloc.BandwidthRequested - getBandwidthNeeded(brs, vls.GetTarget(), lastAllocation.BandwidthRequested);
    alloc.DistanceToDesired = getDistanceToDesired(muted, pubMuted, vls.GetMaxSeen(), availableLayers, brs,
                                                   alloc.TargetLayer, vls.GetMax());
    return updateAllocation(alloc);
  }
  // updateAllocation forwarder.go:1353-1373 (+ setTargetLayer :1375-1382)
  VideoAllocation updateAllocation(VideoAllocation alloc) {
    if (alloc.TargetLayer.IsValid() && mime == MimeH264) alloc.TargetLayer.Temporal = 0;
    lastAllocation = alloc;
    lastAllocIsDeficient = alloc.IsDeficient;
    vls.SetTarget(alloc.TargetLayer);
    vls.SetRequestSpatial(alloc.TargetLayer.IsValid() ? alloc.RequestLayerSpatial : InvalidLayerSpatial);
    if (!vls.GetTarget().IsValid()) resyncLocked();
    return lastAllocation;
  }
  // f.lastAllocation as the reference returns it: the last allocation call's
  // result with IsDeficient as SetAllocation (LKF_CTL_SET_ALLOCATION) last set it
  VideoAllocation LastAllocation() const {
    VideoAllocation a = lastAllocation;
    a.IsDeficient = lastAllocIsDeficient;
    return a;
  }
  // AllocateNextHigher forwarder.go:1107-1217; returns (allocation, boosted)
  std::pair<VideoAllocation, bool> AllocateNextHigher(i64 availableChannelCapacity,
                                                      const std::vector<i32> &availableLayers, const Bitrates &brs,
                                                      bool allowOvershoot) {
    if (kind == KindAudio || !lastAllocIsDeficient) return {LastAllocation(), false};
    const VideoLayer targetLayer = vls.GetTarget();
    if (targetLayer.IsValid() && !(targetLayer == vls.GetCurrent())) return {LastAllocation(), false};
    const VideoLayer maxLayer = vls.GetMax(), maxSeenLayer = vls.GetMaxSeen();
    const i64 optimal = getOptimalBandwidthNeeded(muted, pubMuted, maxSeenLayer.Spatial, brs, maxLayer);
    const i64 already = targetLayer.IsValid() ? brs[targetLayer.Spatial][targetLayer.Temporal] : 0;
    const bool overshoot = allowOvershoot && IsOvershootOkay();
    // doAllocation: 0 = not done, 1 = done (no fit), 2 = done (boosted)
    VideoAllocation result;
    auto doAllocation = [&](i32 minS, i32 maxS, i32 minT, i32 maxT) -> int {
      for (i32 s = minS; s <= maxS; s++)
        for (i32 t = minT; t <= maxT; t++) {
          const i64 bwr = brs[s][t];
          if (bwr == 0) continue;
          if (!overshoot && bwr - already > availableChannelCapacity) {
            result = LastAllocation();
            return 1;
          }
          const VideoLayer nt{s, t};
          VideoAllocation a;
          a.IsDeficient = true;
          a.BandwidthRequested = bwr;
          a.BandwidthDelta = bwr - already;
          a.BandwidthNeeded = optimal;
          a.Brs = brs;
          a.TargetLayer = nt;
          a.RequestLayerSpatial = nt.Spatial;
          a.MaxLayer = maxLayer;
          a.DistanceToDesired = getDistanceToDesired(muted, pubMuted, maxSeenLayer, availableLayers, brs, nt, maxLayer);
          if (nt.GreaterThan(maxLayer) || bwr >= optimal) a.IsDeficient = false;
          result = updateAllocation(a);
          return 2;
        }
      return 0;
    };
    int done = 0;
    if (targetLayer.IsValid())
      done = doAllocation(targetLayer.Spatial, targetLayer.Spatial, targetLayer.Temporal + 1, maxLayer.Temporal);
    if (!done) done = doAllocation(targetLayer.Spatial + 1, maxLayer.Spatial, 0, maxLayer.Temporal);
    if (!done && overshoot && maxLayer.IsValid())
      done = doAllocation(maxLayer.Spatial + 1, DefaultMaxLayerSpatial, 0, DefaultMaxLayerTemporal);
    if (!done) return {LastAllocation(), false};
    return {result, done == 2};
  }
  // GetNextHigherTransition forwarder.go:1219-1306 (read-only)
  struct VideoTransition {
    VideoLayer From{0, 0}, To{0, 0};
    i64 BandwidthDelta = 0;
  };
  std::pair<VideoTransition, bool> GetNextHigherTransition(const Bitrates &brs, bool allowOvershoot) const {
    if (kind == KindAudio || !lastAllocIsDeficient) return {VideoTransition{}, false};
    const VideoLayer targetLayer = vls.GetTarget();
    if (targetLayer.IsValid() && !(targetLayer == vls.GetCurrent())) return {VideoTransition{}, false};
    const i64 already = targetLayer.IsValid() ? brs[targetLayer.Spatial][targetLayer.Temporal] : 0;
    VideoTransition tr;
    auto findNextHigher = [&](i32 minS, i32 maxS, i32 minT, i32 maxT) -> bool {
      for (i32 s = minS; s <= maxS; s++)
        for (i32 t = minT; t <= maxT; t++) {
          const i64 bwr = brs[s][t];
          if (bwr == 0 || bwr < already) continue;
          tr.From = targetLayer;
          tr.To = VideoLayer{s, t};
          tr.BandwidthDelta = bwr - already;
          return true;
        }
      return false;
    };
    const VideoLayer maxLayer = vls.GetMax();
    if (targetLayer.IsValid() && findNextHigher(targetLayer.Spatial, targetLayer.Spatial, targetLayer.Temporal + 1,
                                                maxLayer.Temporal))
      return {tr, true};
    if (findNextHigher(targetLayer.Spatial + 1, maxLayer.Spatial, 0, maxLayer.Temporal)) return {tr, true};
    if (allowOvershoot && IsOvershootOkay() && maxLayer.IsValid() &&
        findNextHigher(maxLayer.Spatial + 1, DefaultMaxLayerSpatial, 0, DefaultMaxLayerTemporal))
      return {tr, true};
    return {VideoTransition{}, false};
  }
  // Pause forwarder.go:1308-1351
  VideoAllocation Pause(const std::vector<i32> &availableLayers, const Bitrates &brs) {
    // the reference dereferences f.vls (nil for audio): the stream allocator
    // pauses only video; an audio request answers lastAllocation unchanged,
    // as AllocateOptimal does (:598-600)
    if (kind == KindAudio) return LastAllocation();
    const VideoLayer maxLayer = vls.GetMax(), maxSeenLayer = vls.GetMaxSeen();
    const i64 optimal = getOptimalBandwidthNeeded(muted, pubMuted, maxSeenLayer.Spatial, brs, maxLayer);
    VideoAllocation a;
    a.BandwidthRequested = 0;
    a.BandwidthDelta = 0 - getBandwidthNeeded(brs, vls.GetTarget(), lastAllocation.BandwidthRequested);
    a.Brs = brs;
    a.BandwidthNeeded = optimal;
    a.TargetLayer = InvalidLayer();
    a.RequestLayerSpatial = InvalidLayerSpatial;
    a.MaxLayer = maxLayer;
    a.DistanceToDesired =
        getDistanceToDesired(muted, pubMuted, maxSeenLayer, availableLayers, brs, InvalidLayer(), maxLayer);
    if (muted)
      a.PauseReason = PauseMuted;
    else if (pubMuted)
      a.PauseReason = PausePubMuted;
    else if (optimal == 0)
      a.PauseReason = PauseFeedDry;
    else {
      a.IsDeficient = true;
      a.PauseReason = PauseBandwidth;
    }
    return updateAllocation(a);
  }
  // ---- the stream allocator's cooperative pass (forwarder.go:727-1105) ----
  // VideoAllocationProvisional forwarder.go:96-106
  struct Provisional {
    VideoLayer allocatedLayer = InvalidLayer();
    bool muted = false, pubMuted = false;
    VideoLayer maxSeenLayer = InvalidLayer();
    Bitrates bitrates{};
    std::vector<i32> availableLayers;
    VideoLayer maxLayer = InvalidLayer(), currentLayer = InvalidLayer();
  } provisional;
  // ProvisionalAllocatePrepare :727-743
  void ProvisionalAllocatePrepare(const std::vector<i32> &availableLayers, const Bitrates &bitrates) {
    provisional = Provisional{};
    provisional.muted = muted;
    provisional.pubMuted = pubMuted;
    provisional.maxSeenLayer = vls.GetMaxSeen();
    provisional.bitrates = bitrates;
    provisional.maxLayer = vls.GetMax();
    provisional.currentLayer = vls.GetCurrent();
    provisional.availableLayers = availableLayers;
  }
  // ProvisionalAllocateReset :745-750
  void ProvisionalAllocateReset() { provisional.allocatedLayer = InvalidLayer(); }
  // ProvisionalAllocate :752-794 -> (isCandidate, usedBitrate)
  std::pair<bool, i64> ProvisionalAllocate(i64 availableChannelCapacity, VideoLayer layer, bool allowPause,
                                           bool allowOvershoot) {
    Provisional &p = provisional;
    if (p.muted || p.pubMuted || p.maxSeenLayer.Spatial == InvalidLayerSpatial || !p.maxLayer.IsValid() ||
        ((!allowOvershoot || !IsOvershootOkay()) && layer.GreaterThan(p.maxLayer)))
      return {false, 0};
    const i64 required = p.bitrates[layer.Spatial][layer.Temporal];
    if (required == 0) return {false, 0};
    i64 already = 0;
    if (p.allocatedLayer.IsValid()) already = p.bitrates[p.allocatedLayer.Spatial][p.allocatedLayer.Temporal];
    if (!layer.GreaterThan(p.maxLayer) && required <= availableChannelCapacity + already) {
      p.allocatedLayer = layer;
      return {true, required - already};
    }
    if (!allowPause && (!p.allocatedLayer.IsValid() || !layer.GreaterThan(p.allocatedLayer))) {
      p.allocatedLayer = layer;
      return {true, required - already};
    }
    return {false, 0};
  }
  // ProvisionalAllocateGetCooperativeTransition :796-929
  VideoTransition ProvisionalAllocateGetCooperativeTransition(bool allowOvershoot) {
    Provisional &p = provisional;
    const VideoLayer existing = vls.GetTarget();
    if (p.muted || p.pubMuted) {
      p.allocatedLayer = InvalidLayer();
      return VideoTransition{existing, p.allocatedLayer,
                             -getBandwidthNeeded(p.bitrates, existing, lastAllocation.BandwidthRequested)};
    }
    if (existing.IsValid()) {
      VideoLayer maximal = InvalidLayer();
      i64 maximalBw = 0;
      for (i32 s = p.maxLayer.Spatial; s >= 0; s--) {
        for (i32 t = p.maxLayer.Temporal; t >= 0; t--)
          if (p.bitrates[s][t] != 0) {
            maximal = VideoLayer{s, t};
            maximalBw = p.bitrates[s][t];
            break;
          }
        if (maximalBw != 0) break;
      }
      if (maximal.IsValid()) {
        if (!existing.GreaterThan(maximal) && p.bitrates[existing.Spatial][existing.Temporal] != 0) {
          p.allocatedLayer = existing;
          return VideoTransition{existing, existing, 0};
        }
        if (existing.GreaterThan(maximal)) {
          p.allocatedLayer = maximal;
          return VideoTransition{existing, maximal,
                                 maximalBw - getBandwidthNeeded(p.bitrates, existing, lastAllocation.BandwidthRequested)};
        }
      }
    }
    auto findNextLayer = [&](i32 minS, i32 maxS, i32 minT, i32 maxT, i64 &bw) {
      VideoLayer l = InvalidLayer();
      bw = 0;
      for (i32 s = minS; s <= maxS; s++) {
        for (i32 t = minT; t <= maxT; t++)
          if (p.bitrates[s][t] != 0) {
            l = VideoLayer{s, t};
            bw = p.bitrates[s][t];
            break;
          }
        if (bw != 0) break;
      }
      return l;
    };
    VideoLayer target = InvalidLayer();
    i64 required = 0;
    if (!existing.IsValid()) {
      target = findNextLayer(0, p.maxLayer.Spatial, 0, p.maxLayer.Temporal, required);
      if (required == 0 && p.maxLayer.IsValid() && allowOvershoot && IsOvershootOkay())
        target = findNextLayer(p.maxLayer.Spatial + 1, DefaultMaxLayerSpatial, 0, DefaultMaxLayerTemporal, required);
    }
    if (!target.IsValid()) {
      target = p.currentLayer;
      if (target.IsValid()) required = p.bitrates[target.Spatial][target.Temporal];
    }
    p.allocatedLayer = target;
    return VideoTransition{vls.GetTarget(), target,
                           required - getBandwidthNeeded(p.bitrates, existing, lastAllocation.BandwidthRequested)};
  }
  // ProvisionalAllocateGetBestWeightedTransition :931-1025
  VideoTransition ProvisionalAllocateGetBestWeightedTransition() {
    Provisional &p = provisional;
    const VideoLayer target = vls.GetTarget();
    if (p.muted || p.pubMuted) {
      p.allocatedLayer = InvalidLayer();
      return VideoTransition{target, p.allocatedLayer,
                             0 - getBandwidthNeeded(p.bitrates, target, lastAllocation.BandwidthRequested)};
    }
    i32 maxReachT = InvalidLayerTemporal;
    for (i32 t = p.maxLayer.Temporal; t >= 0; t--) {
      for (i32 s = p.maxLayer.Spatial; s >= 0; s--)
        if (p.bitrates[s][t] != 0) {
          maxReachT = t;
          break;
        }
      if (maxReachT != InvalidLayerTemporal) break;
    }
    if (maxReachT == InvalidLayerTemporal) {
      p.allocatedLayer = p.currentLayer;
      return VideoTransition{target, p.allocatedLayer,
                             0 - getBandwidthNeeded(p.bitrates, target, lastAllocation.BandwidthRequested)};
    }
    const i64 existingBw = getBandwidthNeeded(p.bitrates, target, lastAllocation.BandwidthRequested);
    VideoLayer best = InvalidLayer();
    i64 bestDelta = 0;
    float bestValue = 0;
    for (i32 s = 0; s <= target.Spatial; s++) {
      for (i32 t = 0; t <= target.Temporal; t++) {
        if (s == target.Spatial && t == target.Temporal) break;
        // int64(math.Max(float64(0), float64(existing - brs))) (exact below 2^53)
        const i64 delta = i64(std::max(0.0, double(existingBw - p.bitrates[s][t])));
        const i32 transitionCost = target.Spatial != s ? TransitionCostSpatial : 0;
        const i32 qualityCost = (maxReachT + 1) * (target.Spatial - s) + (target.Temporal - t);
        float value = 0;
        if (transitionCost + qualityCost != 0) value = float(delta) / float(transitionCost + qualityCost);
        if (value > bestValue || (value == bestValue && delta > bestDelta)) {
          bestValue = value;
          bestDelta = delta;
          best = VideoLayer{s, t};
        }
      }
    }
    p.allocatedLayer = best;
    return VideoTransition{target, best, -bestDelta};
  }
  // ProvisionalAllocateCommit :1027-1105
  VideoAllocation ProvisionalAllocateCommit() {
    Provisional &p = provisional;
    const i64 optimal = getOptimalBandwidthNeeded(p.muted, p.pubMuted, p.maxSeenLayer.Spatial, p.bitrates, p.maxLayer);
    VideoAllocation a;
    a.BandwidthRequested = 0;
    a.BandwidthDelta = 0 - getBandwidthNeeded(p.bitrates, vls.GetTarget(), lastAllocation.BandwidthRequested);
    a.Brs = p.bitrates;
    a.BandwidthNeeded = optimal;
    a.TargetLayer = p.allocatedLayer;
    a.RequestLayerSpatial = p.allocatedLayer.Spatial;
    a.MaxLayer = p.maxLayer;
    a.DistanceToDesired = getDistanceToDesired(p.muted, p.pubMuted, p.maxSeenLayer, p.availableLayers, p.bitrates,
                                               p.allocatedLayer, p.maxLayer);
    if (p.muted) {
      a.PauseReason = PauseMuted;
    } else if (p.pubMuted) {
      a.PauseReason = PausePubMuted;
    } else if (optimal == 0) {
      if (p.allocatedLayer.IsValid()) {  // overshoot
        a.BandwidthRequested = p.bitrates[p.allocatedLayer.Spatial][p.allocatedLayer.Temporal];
        a.BandwidthDelta =
            a.BandwidthRequested - getBandwidthNeeded(p.bitrates, vls.GetTarget(), lastAllocation.BandwidthRequested);
      } else {
        a.PauseReason = PauseFeedDry;
        if (p.currentLayer.IsValid() && p.currentLayer.Spatial <= p.maxLayer.Spatial) {
          p.allocatedLayer = p.currentLayer;
          a.TargetLayer = p.allocatedLayer;
          a.RequestLayerSpatial = a.TargetLayer.Spatial;
        }
      }
    } else {
      if (p.allocatedLayer.IsValid()) a.BandwidthRequested = p.bitrates[p.allocatedLayer.Spatial][p.allocatedLayer.Temporal];
      a.BandwidthDelta =
          a.BandwidthRequested - getBandwidthNeeded(p.bitrates, vls.GetTarget(), lastAllocation.BandwidthRequested);
      if (p.allocatedLayer.GreaterThan(p.maxLayer) || a.BandwidthRequested >= optimal) {
        a.IsDeficient = false;
      } else {
        a.IsDeficient = true;
        if (!p.allocatedLayer.IsValid()) a.PauseReason = PauseBandwidth;
      }
    }
    return updateAllocation(a);
  }

  // Resync / resyncLocked forwarder.go:1384-1397
  void Resync() { resyncLocked(); }
  void resyncLocked() {
    vls.SetCurrent(InvalidLayer());
    lastSSRC = 0;
    if (pubMuted) resumeBehindThreshold = ResumeBehindThresholdSeconds;
  }

  // GetTranslationParams forwarder.go:1436-1454; `now` is the virtual clock.
  Err GetTranslationParams(const ExtPacket &p, i32 layer, i64 now, TranslationParams &tp) {
    tp = TranslationParams{};
    if (muted || pubMuted) {
      tp.shouldDrop = true;
      tp.dropReason = 0;
      return OK;
    }
    if (kind == KindAudio) return getTranslationParamsCommon(p, layer, now, tp);
    if (kind == KindVideo) return getTranslationParamsVideo(p, layer, now, tp);
    return ErrUnknownKind;
  }

  // processSourceSwitch forwarder.go:1456-1647
  Err processSourceSwitch(const ExtPacket &p, i32 layer, i64 now) {
    if (!started) {
      started = true;
      referenceLayerSpatial = layer;
      rtpMunger.SetLastSnTs(p);
      if (hasVP8Munger) vp8.SetLast(p);
      return OK;
    } else if (referenceLayerSpatial == InvalidLayerSpatial) {
      referenceLayerSpatial = layer;
    }
    RTPMungerState st = rtpMunger.GetLast();
    u64 extLastTS = st.ExtLastTS;
    u64 extExpectedTS = extLastTS;
    u64 extRefTS = extExpectedTS;
    i64 switchingAt = now;
    if (getReferenceLayerRTPTimestamp) {
      u32 ts = 0;
      Err e = getReferenceLayerRTPTimestamp(p.Header.Timestamp, layer, referenceLayerSpatial, ts);
      if (e != OK) return e;
      extRefTS = (extRefTS & 0xFFFFFFFF00000000ull) + u64(ts);
      u32 expectedTS32 = u32(extExpectedTS);
      if (u32(ts - expectedTS32) < (1u << 31) && ts < expectedTS32) extRefTS += (1ull << 32);
      if (u32(expectedTS32 - ts) < (1u << 31) && expectedTS32 < ts && extRefTS >= (1ull << 32))
        extRefTS -= (1ull << 32);
    }
    if (getExpectedRTPTimestamp) {
      u64 tsExt = 0;
      if (getExpectedRTPTimestamp(switchingAt, tsExt) == OK) {
        extExpectedTS = tsExt;
      } else if (preStartTime != 0) {
        i64 timeSinceFirst = now - preStartTime;
        u64 rtpDiff = u64(timeSinceFirst * i64(clockRate) / 1000000000LL);
        extExpectedTS = extFirstTS + rtpDiff;
        if (refTSOffset == 0) refTSOffset = extExpectedTS - extRefTS;
      }
    }
    extRefTS += refTSOffset;

    u64 extNextTS = 0;
    if (lastSSRC == 0) {
      double diffSeconds = double(i64(extExpectedTS - extRefTS)) / double(clockRate);
      if (diffSeconds >= 0.0) {
        if (resumeBehindThreshold > 0 && diffSeconds > resumeBehindThreshold)
          extNextTS = extExpectedTS;
        else if (diffSeconds > ResumeBehindHighTresholdSeconds)
          extNextTS = extExpectedTS;
        else
          extNextTS = extRefTS;
      } else {
        extNextTS = extRefTS;
      }
      resumeBehindThreshold = 0.0;
    } else {
      double diffSeconds = double(i64(extRefTS - extLastTS)) / double(clockRate);
      if (diffSeconds < 0.0) {
        if (std::fabs(diffSeconds) > LayerSwitchBehindThresholdSeconds) return ErrSwitchTooFarBehind;
        extNextTS = extLastTS + 1;
      } else {
        extNextTS = extRefTS;
      }
    }
    if (i64(extNextTS - extLastTS) <= 0) extNextTS = extLastTS + 1;
    rtpMunger.UpdateSnTsOffsets(p, 1, extNextTS - extLastTS);
    if (hasVP8Munger) vp8.UpdateOffsets(p);
    return OK;
  }

  // getTranslationParamsCommon forwarder.go:1650-1671
  Err getTranslationParamsCommon(const ExtPacket &p, i32 layer, i64 now, TranslationParams &tp) {
    if (lastSSRC != p.Header.SSRC) {
      if (processSourceSwitch(p, layer, now) != OK) {
        tp.shouldDrop = true;
        tp.dropReason = 4;
        return OK;
      }
      lastSSRC = p.Header.SSRC;
    }
    TranslationParamsRTP r;
    Err e = rtpMunger.UpdateAndGetSnTs(p, tp.marker, r);
    if (e != OK) {
      tp.shouldDrop = true;
      tp.dropReason = e == ErrPaddingOnlyPacket ? 5 : e == ErrDuplicatePacket ? 6 : e == ErrOutOfOrderSequenceNumberCacheMiss ? 7 : 10;
      if (e == ErrPaddingOnlyPacket || e == ErrDuplicatePacket || e == ErrOutOfOrderSequenceNumberCacheMiss) return OK;
      return e;
    }
    tp.hasRTP = true;
    tp.rtp = r;
    return OK;
  }

  // getTranslationParamsVideo forwarder.go:1679-1765
  Err getTranslationParamsVideo(const ExtPacket &p, i32 layer, i64 now, TranslationParams &tp) {
    if (!vls.GetTarget().IsValid()) {
      tp.shouldDrop = true;
      tp.dropReason = 1;
      return OK;
    }
    VideoLayerSelectorResult res = vls.Select(p, layer);
    if (!res.IsSelected) {
      tp.shouldDrop = true;
      tp.dropReason = 2;
      if (started && res.IsRelevant) {
        TranslationParamsRTP r;
        if (rtpMunger.UpdateAndGetSnTs(p, res.RTPMarker, r) == OK && r.snOrdering == SequenceNumberOrderingContiguous)
          rtpMunger.PacketDropped(p);
      }
      return OK;
    }
    tp.isResuming = res.IsResuming;
    tp.isSwitching = res.IsSwitching;
    tp.ddBytes = res.DependencyDescriptorExtension;
    tp.marker = res.RTPMarker;
    if (FlagPauseOnDowngrade && lastAllocIsDeficient && vls.GetTarget().Spatial < vls.GetCurrent().Spatial) {
      tp.shouldDrop = true;
      tp.dropReason = 3;
      if (res.IsSwitching) vls.Rollback();
      return OK;
    }
    Err e = getTranslationParamsCommon(p, layer, now, tp);
    if (tp.shouldDrop || p.Payload.empty()) {
      if (res.IsSwitching) vls.Rollback();
      return e;
    }
    auto tsel = vls.SelectTemporal(p);
    i32 tl = tsel.first;
    bool isSwitching = tsel.second;
    std::vector<u8> cb;
    Err ce = OK;
    if (hasVP8Munger) {
      ce = vp8.UpdateAndGet(p, tp.rtp.snOrdering == SequenceNumberOrderingOutOfOrder,
                            tp.rtp.snOrdering == SequenceNumberOrderingGap, tl, cb);
    }
    // codecmunger.Null.UpdateAndGet returns (nil, nil) (null.go)
    if (ce != OK) {
      tp.hasRTP = false;
      tp.rtp = TranslationParamsRTP{};
      tp.shouldDrop = true;
      tp.dropReason = ce == ErrFilteredVP8TemporalLayer ? 8 : ce == ErrOutOfOrderVP8PictureIdCacheMiss ? 9 : 10;
      if (ce == ErrFilteredVP8TemporalLayer || ce == ErrOutOfOrderVP8PictureIdCacheMiss) {
        if (ce == ErrFilteredVP8TemporalLayer) rtpMunger.PacketDropped(p);
        if (res.IsSwitching || isSwitching) vls.Rollback();
        return OK;
      }
      if (res.IsSwitching || isSwitching) vls.Rollback();
      return ce;
    }
    tp.codecBytes = cb;
    return OK;
  }

  // GetSnTsForPadding forwarder.go:1798-1813 (maybeStart's math/rand start
  // values are injected by the caller: forwarder.go:1775-1776)
  void maybeStart(i64 now, u16 randSN, u32 randTS) {
    if (started) return;
    started = true;
    preStartTime = now;
    ExtPacket p;
    p.Header.SequenceNumber = randSN;
    p.Header.Timestamp = randTS;
    p.ExtSequenceNumber = randSN;
    p.ExtTimestamp = randTS;
    rtpMunger.SetLastSnTs(p);
    extFirstTS = randTS;
  }
  Err GetSnTsForPadding(int num, bool forceMarker, i64 now, u16 randSN, u32 randTS, std::vector<SnTs> &out) {
    maybeStart(now, randSN, randTS);
    if (!vls.GetTarget().IsValid()) forceMarker = true;
    return rtpMunger.UpdateAndGetPaddingSnTs(num, 0, 0, forceMarker, 0, out);
  }
  // GetSnTsForBlankFrames forwarder.go:1815-1839
  Err GetSnTsForBlankFrames(u32 frameRate, int numPackets, i64 now, u16 randSN, u32 randTS, std::vector<SnTs> &out,
                            bool &frameEndNeeded) {
    maybeStart(now, randSN, randTS);
    frameEndNeeded = !rtpMunger.IsOnFrameBoundary();
    if (frameEndNeeded) numPackets++;
    u64 extLastTS = rtpMunger.GetLast().ExtLastTS;
    u64 extExpectedTS = extLastTS;
    if (getExpectedRTPTimestamp) {
      u64 t = 0;
      if (getExpectedRTPTimestamp(now, t) == OK) extExpectedTS = t;
    }
    if (i64(extExpectedTS - extLastTS) <= 0) extExpectedTS = extLastTS + 1;
    return rtpMunger.UpdateAndGetPaddingSnTs(numPackets, clockRate, frameRate, frameEndNeeded, extExpectedTS, out);
  }
  // GetPadding forwarder.go:1841-1846
  Err GetPadding(bool frameEndNeeded, std::vector<u8> &out) {
    out.clear();
    if (!hasVP8Munger) return OK;  // Null codec munger returns nil
    return vp8.UpdateAndGetPadding(!frameEndNeeded, out);
  }
};

// -----------------------------------------------------------------------------
// sequencer — pkg/sfu/sequencer.go:26-370 (virtual ms clock)
// -----------------------------------------------------------------------------
constexpr u32 defaultRtt = 70;
constexpr u32 ignoreRetransmission = 100;
constexpr u8 maxAck = 3;

struct PacketMeta {  // sequencer.go:44-73
  u16 sourceSeqNo = 0;
  u16 targetSeqNo = 0;
  u32 timestamp = 0;
  bool marker = false;
  u32 lastNack = 0;
  u8 nacked = 0;
  i8 layer = 0;
  std::vector<u8> codecBytes;
  std::vector<u8> ddBytes;
};

struct ExtPacketMeta {
  PacketMeta meta;
  u64 extSequenceNumber = 0;
  u64 extTimestamp = 0;
  u64 slot = 0;  // the ring slot the record was read from (engine-defined: lkf_rtx.reserved - 1)
};

struct Sequencer {
  int size;
  i64 startTimeMs;
  bool initialized = false;
  u64 extStartSN = 0, extHighestSN = 0, snOffset = 0, extHighestTS = 0;
  std::vector<PacketMeta> meta;
  bool hasRangeMap;
  RangeMap<u64, u64> snRangeMap;
  u32 rtt = defaultRtt;

  // newSequencer sequencer.go:97-110; startTimeMs replaces time.Now().UnixMilli()
  Sequencer(int sz, bool maybeSparse, i64 startMs)
      : size(sz), startTimeMs(startMs), meta(sz), hasRangeMap(maybeSparse), snRangeMap((sz + 1) / 2) {}

  void setRTT(u32 r) { rtt = r == 0 ? defaultRtt : r; }
  u32 getRefTime(i64 atMs) const { return u32(atMs - startTimeMs); }

  // push sequencer.go:123-209 (packetTime in virtual ms)
  void push(i64 packetTimeMs, u64 extIncomingSN, u64 extModifiedSN, u64 extModifiedTS, bool marker, i8 layer,
            const std::vector<u8> &codecBytes, const std::vector<u8> &ddBytes) {
    if (!initialized) {
      initialized = true;
      extStartSN = extModifiedSN;
      extHighestSN = extModifiedSN;
      extHighestTS = extModifiedTS;
      updateSNOffset();
    }
    if (extModifiedSN < extStartSN) return;
    u64 extHighestSNAdjusted = extHighestSN - snOffset;
    u64 extModifiedSNAdjusted = extModifiedSN - snOffset;
    if (extModifiedSN < extHighestSN) {
      if (hasRangeMap) {
        u64 off = 0;
        if (snRangeMap.GetValue(extModifiedSN, off) != OK) return;
        extModifiedSNAdjusted = extModifiedSN - off;
      }
    }
    if (i64(extModifiedSNAdjusted - extHighestSNAdjusted) <= -i64(size)) return;
    if (extModifiedSNAdjusted > extHighestSNAdjusted) {
      int numInvalidated = 0;
      for (u64 esn = extHighestSNAdjusted + 1; esn != extModifiedSNAdjusted; esn++) {
        invalidateSlot(int(esn % u64(size)));
        numInvalidated++;
        if (numInvalidated >= size) break;
      }
    }
    u64 slot = extModifiedSNAdjusted % u64(size);
    PacketMeta &m = meta[slot];
    m.sourceSeqNo = u16(extIncomingSN);
    m.targetSeqNo = u16(extModifiedSN);
    m.timestamp = u32(extModifiedTS);
    m.marker = marker;
    m.layer = layer;
    m.codecBytes = codecBytes;
    m.ddBytes = ddBytes;
    m.lastNack = getRefTime(packetTimeMs);
    m.nacked = 0;
    if (extModifiedSN > extHighestSN) extHighestSN = extModifiedSN;
    if (extModifiedTS > extHighestTS) extHighestTS = extModifiedTS;
  }
  // pushPadding sequencer.go:211-261
  void pushPadding(u64 s, u64 e) {
    if (!hasRangeMap) return;
    if (s <= extHighestSN) {
      for (u64 sn = s; sn != e + 1; sn++) {
        i64 diff = i64(sn - extHighestSN);
        if (diff >= 0 || diff < -i64(size)) continue;
        u64 off = 0;
        if (snRangeMap.GetValue(sn, off) != OK) continue;
        invalidateSlot(int((sn - off) % u64(size)));
      }
      return;
    }
    if (snRangeMap.ExcludeRange(s, e + 1) != OK) return;
    extHighestSN = e;
    updateSNOffset();
  }
  // getExtPacketMetas sequencer.go:263-332 (nowMs = virtual clock)
  std::vector<ExtPacketMeta> getExtPacketMetas(const std::vector<u16> &seqNo, i64 nowMs) {
    std::vector<ExtPacketMeta> res;
    if (!initialized) return res;
    u64 off = 0;
    u32 refTime = getRefTime(nowMs);
    u16 highestSN = u16(extHighestSN);
    u32 highestTS = u32(extHighestTS);
    for (u16 sn : seqNo) {
      u16 diff = u16(highestSN - sn);
      if (diff > (1 << 15)) continue;
      u64 extSN = u64(sn) + (extHighestSN & 0xFFFFFFFFFFFF0000ull);
      if (sn > highestSN) extSN -= (1ull << 16);
      if (hasRangeMap) {
        if (snRangeMap.GetValue(extSN, off) != OK) continue;
      }
      u64 extSNAdjusted = extSN - off;
      u64 extHighestSNAdjusted = extHighestSN - snOffset;
      if (extHighestSNAdjusted - extSNAdjusted >= u64(size)) continue;
      u64 slot = extSNAdjusted % u64(size);
      PacketMeta &m = meta[slot];
      if (m.targetSeqNo != sn || isInvalidSlot(int(slot))) continue;
      u32 lim = u32(std::min(double(ignoreRetransmission), double(2 * rtt)));
      if (m.nacked < maxAck && u32(refTime - m.lastNack) > lim) {
        m.nacked++;
        m.lastNack = refTime;
        u64 extTS = u64(m.timestamp) + (extHighestTS & 0xFFFFFFFF00000000ull);
        if (m.timestamp > highestTS) extTS -= (1ull << 32);
        ExtPacketMeta epm;
        epm.meta = m;
        epm.extSequenceNumber = extSN;
        epm.extTimestamp = extTS;
        epm.slot = slot;
        res.push_back(epm);
      }
    }
    return res;
  }
  void updateSNOffset() {
    if (!hasRangeMap) return;
    u64 off = 0;
    if (snRangeMap.GetValue(extHighestSN + 1, off) != OK) return;
    snOffset = off;
  }
  void invalidateSlot(int slot) {
    if (slot >= (int)meta.size()) return;
    meta[slot] = PacketMeta{};
  }
  bool isInvalidSlot(int slot) const {
    if (slot >= (int)meta.size()) return true;
    const PacketMeta &m = meta[slot];
    return m.sourceSeqNo == 0 && m.targetSeqNo == 0 && m.lastNack == 0;
  }
};

// -----------------------------------------------------------------------------
// audio.AudioLevel — pkg/sfu/audio/audiolevel.go:15-134 (virtual ms clock)
// Go math.Log10 / math.Pow vs libm: float bits PARITY UNPINNED (the reference
// test checks thresholds only); speaker outputs are compared after the
// float32 quantisation of room.go:274-276.
// -----------------------------------------------------------------------------
struct AudioLevelParams {
  u8 ActiveLevel = 35;
  u8 MinPercentile = 40;
  u32 ObserveDuration = 400;
  u32 SmoothIntervals = 2;
};

inline double ConvertAudioLevel(double level) { return std::pow(10.0, level * (-1.0 / 20)); }

struct AudioLevel {
  AudioLevelParams params;
  u32 minActiveDuration;
  double smoothFactor = 1;
  double activeThreshold;
  double smoothedLevel = 0;
  u8 loudestObservedLevel = 127;
  u32 activeDuration = 0;
  u32 observedDuration = 0;
  i64 lastObservedAtNs = 0;  // virtual ns; 0 = time.Time{} (always stale)

  explicit AudioLevel(AudioLevelParams p) : params(p) {
    minActiveDuration = u32(p.MinPercentile) * p.ObserveDuration / 100;
    activeThreshold = ConvertAudioLevel(double(p.ActiveLevel));
    if (p.SmoothIntervals > 0) smoothFactor = double(2) / double(p.SmoothIntervals + 1);
  }
  // Observe audiolevel.go:70-102
  void Observe(u8 level, u32 durationMs, i64 arrivalNs) {
    lastObservedAtNs = arrivalNs;
    observedDuration += durationMs;
    if (level <= params.ActiveLevel) {
      activeDuration += durationMs;
      if (loudestObservedLevel > level) loudestObservedLevel = level;
    }
    if (observedDuration >= params.ObserveDuration) {
      double s = 0.0;
      if (activeDuration >= minActiveDuration) {
        double activityWeight = 20 * std::log10(double(activeDuration) / double(params.ObserveDuration));
        double adjusted = double(loudestObservedLevel) - activityWeight;
        double linear = ConvertAudioLevel(adjusted);
        s = smoothedLevel + (linear - smoothedLevel) * smoothFactor;
      }
      resetLocked(s);
    }
  }
  // GetLevel audiolevel.go:105-112
  std::pair<double, bool> GetLevel(i64 nowNs) {
    resetIfStaleLocked(nowNs);
    return {smoothedLevel, smoothedLevel >= activeThreshold};
  }
  // arrivalTime.Sub(lastObservedAt).Milliseconds() truncates toward zero
  void resetIfStaleLocked(i64 nowNs) {
    if ((nowNs - lastObservedAtNs) / 1000000 < i64(2 * params.ObserveDuration)) return;
    resetLocked(0.0);
  }
  void resetLocked(double s) {
    smoothedLevel = s;
    loudestObservedLevel = 127;
    activeDuration = 0;
    observedDuration = 0;
  }
};

// Speaker ranking: Room.GetActiveSpeakers room.go:254-279 (+ constants
// room.go:51-52).  sort.Slice is UNSTABLE in Go; the engine and this oracle
// both break ties by ascending participant index (documented divergence:
// the reference's tie order is unspecified).
struct SpeakerInfo {
  u32 participant;
  float level;
};
inline std::vector<SpeakerInfo> RankSpeakers(const std::vector<std::pair<double, bool>> &levels) {
  std::vector<SpeakerInfo> sp;
  for (u32 i = 0; i < levels.size(); i++) {
    if (!levels[i].second) continue;
    sp.push_back(SpeakerInfo{i, float(levels[i].first)});
  }
  std::stable_sort(sp.begin(), sp.end(), [](const SpeakerInfo &a, const SpeakerInfo &b) { return a.level > b.level; });
  for (auto &s : sp) s.level = float(std::ceil(double(s.level * 8.0f)) * (1.0 / 8));
  return sp;
}

// -----------------------------------------------------------------------------
// RTPStatsReceiver.Update flow classification — pkg/sfu/buffer/
// rtpstats_receiver.go:76-241 (counters used by tests kept; jitter and
// snapshot bookkeeping out of scope).  history = livekit/protocol
// utils.Bitmap (4096 bits; not vendored) restated with empty-range ClearRange
// a no-op (pinned by rtpstats_receiver_test.go:246-267).
// -----------------------------------------------------------------------------
struct RTPFlowState {
  bool IsNotHandled = false;
  bool HasLoss = false;
  u64 LossStartInclusive = 0;
  u64 LossEndExclusive = 0;
  bool IsDuplicate = false;
  bool IsOutOfOrder = false;
  u64 ExtSequenceNumber = 0;
  u64 ExtTimestamp = 0;
};

constexpr u64 cHistorySize = 4096;
constexpr i64 cNumSequenceNumbers = 65536;

struct HistoryBitmap {
  u64 bits[cHistorySize / 64] = {};
  void Set(u64 v) { bits[(v >> 6) & (cHistorySize / 64 - 1)] |= (1ull << (v & 63)); }
  bool IsSet(u64 v) const { return (bits[(v >> 6) & (cHistorySize / 64 - 1)] >> (v & 63)) & 1; }
  void ClearRange(u64 lo, u64 hi) {  // inclusive; lo > hi -> no-op
    if (lo > hi) return;
    if (hi - lo + 1 >= cHistorySize) {
      std::memset(bits, 0, sizeof(bits));
      return;
    }
    for (u64 v = lo; v != hi + 1; v++) bits[(v >> 6) & (cHistorySize / 64 - 1)] &= ~(1ull << (v & 63));
  }
};

struct RTPStatsReceiver {
  bool initialized = false;
  bool ended = false;
  WrapAround<u16, u64> sequenceNumber{false};
  WrapAround<u32, u64> timestamp{false};
  HistoryBitmap history;
  u64 packetsOutOfOrder = 0, packetsDuplicate = 0, packetsLost = 0, packetsPadding = 0, frames = 0;
  u64 bytes = 0, headerBytes = 0, bytesDuplicate = 0, headerBytesDuplicate = 0, bytesPadding = 0,
      headerBytesPadding = 0;
  // rtpStatsBase timing and jitter (rtpstats_base.go:133-190): packet times on
  // the caller's clock (the datagram arrival), clock rate of the stream
  i64 firstTime = 0, highestTime = 0;
  u64 lastTransit = 0, lastJitterExtTimestamp = 0;
  double jitter = 0, maxJitter = 0;
  u32 clockRate = 0;
  u32 gapHistogram[101] = {};  // cGapHistogramNumBins rtpstats_base.go:31

  bool isInRange(u64 esn, u64 ehsn) const {  // rtpstats_receiver.go:427-430
    i64 diff = i64(ehsn - esn);
    return diff >= 0 && diff < i64(cHistorySize);
  }
  // rtpStatsBase.updateGapHistogram rtpstats_base.go:871-882
  void updateGapHistogram(i64 gap) {
    if (gap < 2) return;
    const i64 missing = gap - 1;
    if (missing > i64(101))
      gapHistogram[100]++;
    else
      gapHistogram[missing - 1]++;
  }
  // rtpStatsBase.updateJitter rtpstats_base.go:775-810 (Go's int64 products wrap:
  // formed in u64; no snapshots)
  void updateJitter(u64 ets, i64 packetTime) {
    if (lastJitterExtTimestamp == ets) return;
    const i64 since = i64(u64(packetTime) - u64(firstTime));
    const u64 packetTimeRTP = u64(i64(u64(since) * u64(i64(clockRate))) / 1000000000LL);
    const u64 transit = packetTimeRTP - ets;
    if (lastTransit != 0) {
      i64 d = i64(transit - lastTransit);
      if (d < 0) d = i64(0 - u64(d));
      jitter += (double(d) - jitter) / 16;
      if (jitter > maxJitter) maxJitter = jitter;
    }
    lastTransit = transit;
    lastJitterExtTimestamp = ets;
  }
  RTPFlowState Update(u16 sn, u32 ts, bool marker, int payloadSize) { return Update(0, sn, ts, marker, 12, payloadSize, 0); }
  RTPFlowState Update(u16 sn, u32 ts, bool marker, int hdrSize, int payloadSize, int paddingSize) {
    return Update(0, sn, ts, marker, hdrSize, payloadSize, paddingSize);
  }
  // Update rtpstats_receiver.go:76-241 (snapshots / report timing out of scope)
  RTPFlowState Update(i64 packetTime, u16 sn, u32 ts, bool marker, int hdrSize, int payloadSize, int paddingSize) {
    RTPFlowState fs;
    const u64 pktSize = u64(hdrSize + payloadSize + paddingSize);
    if (ended) {
      fs.IsNotHandled = true;
      return fs;
    }
    WrapAroundResult<u16, u64> rsn;
    WrapAroundResult<u32, u64> rts;
    if (!initialized) {
      if (payloadSize == 0) {
        fs.IsNotHandled = true;
        return fs;
      }
      initialized = true;
      firstTime = packetTime;
      highestTime = packetTime;
      rsn = sequenceNumber.Update(sn);
      rts = timestamp.Update(ts);
    } else {
      rsn = sequenceNumber.Update(sn);
      if (rsn.IsUnhandled) {
        fs.IsNotHandled = true;
        return fs;
      }
      rts = timestamp.Update(ts);
    }
    i64 gapSN = i64(rsn.ExtendedVal - rsn.PreExtendedHighest);
    if (gapSN <= 0) {
      if (gapSN != 0) packetsOutOfOrder++;
      if (isInRange(rsn.ExtendedVal, rsn.PreExtendedHighest)) {
        if (history.IsSet(rsn.ExtendedVal)) {
          bytesDuplicate += pktSize;
          headerBytesDuplicate += u64(hdrSize);
          packetsDuplicate++;
          fs.IsDuplicate = true;
        } else {
          packetsLost--;
          history.Set(rsn.ExtendedVal);
        }
      }
      fs.IsOutOfOrder = true;
      fs.ExtSequenceNumber = rsn.ExtendedVal;
      fs.ExtTimestamp = rts.ExtendedVal;
    } else {
      updateGapHistogram(gapSN);
      history.ClearRange(rsn.PreExtendedHighest + 1, rsn.ExtendedVal - 1);
      packetsLost += u64(gapSN - 1);
      history.Set(rsn.ExtendedVal);
      // the first packet of a timestamp (rtpstats_receiver.go:209-213)
      if (ts != u32(rts.PreExtendedHighest)) highestTime = packetTime;
      if (gapSN > 1) {
        fs.HasLoss = true;
        fs.LossStartInclusive = rsn.PreExtendedHighest + 1;
        fs.LossEndExclusive = rsn.ExtendedVal;
      }
      fs.ExtSequenceNumber = rsn.ExtendedVal;
      fs.ExtTimestamp = rts.ExtendedVal;
    }
    if (!fs.IsDuplicate) {
      if (payloadSize == 0) {
        packetsPadding++;
        bytesPadding += pktSize;
        headerBytesPadding += u64(hdrSize);
      } else {
        bytes += pktSize;
        headerBytes += u64(hdrSize);
        if (marker) frames++;
        updateJitter(rts.ExtendedVal, packetTime);
      }
    }
    return fs;
  }
};

// -----------------------------------------------------------------------------
// rtp.Packet.Unmarshal (pion/rtp v1.8.3 packet.go / header.go), restated:
// fixed header, CSRCs, one-byte (0xBEDE) / two-byte (0x1000) / RFC 3550
// extension blocks, padding.  PARITY UNPINNED (no reference test).
// -----------------------------------------------------------------------------
struct RtpParsed {
  u8 b0 = 0, b1 = 0;
  bool padding = false, extension = false, marker = false;
  int cc = 0;
  u8 pt = 0;
  u16 sn = 0;
  u32 ts = 0, ssrc = 0;
  int hdrSize = 0;  // n: payload offset
  int payloadLen = 0;
  int paddingSize = 0;
  u16 extProfile = 0;
  int nExt = 0;
  u8 extId[16];
  int extOff[16], extLen[16];
  // Header.GetExtension(id): first extension with that id (header.go)
  bool GetExtension(u8 id, int &off, int &len) const {
    if (!extension) return false;
    for (int i = 0; i < nExt; i++)
      if (extId[i] == id) {
        off = extOff[i];
        len = extLen[i];
        return true;
      }
    return false;
  }
};
inline bool rtp_unmarshal(const u8 *buf, int len, RtpParsed &h) {
  h = RtpParsed{};
  if (len < 12) return false;
  h.b0 = buf[0];
  h.b1 = buf[1];
  h.padding = (buf[0] >> 5) & 1;
  h.extension = (buf[0] >> 4) & 1;
  h.cc = buf[0] & 0xf;
  int n = 12 + 4 * h.cc;
  if (len < n) return false;
  h.marker = buf[1] >> 7;
  h.pt = buf[1] & 0x7f;
  h.sn = u16((buf[2] << 8) | buf[3]);
  h.ts = (u32(buf[4]) << 24) | (u32(buf[5]) << 16) | (u32(buf[6]) << 8) | buf[7];
  h.ssrc = (u32(buf[8]) << 24) | (u32(buf[9]) << 16) | (u32(buf[10]) << 8) | buf[11];
  if (h.extension) {
    if (len < n + 4) return false;
    h.extProfile = u16((buf[n] << 8) | buf[n + 1]);
    n += 2;
    const int extLen = ((buf[n] << 8) | buf[n + 1]) * 4;
    n += 2;
    const int extEnd = n + extLen;
    if (len < extEnd) return false;
    if (h.extProfile == 0xBEDE || h.extProfile == 0x1000) {
      while (n < extEnd) {
        if (buf[n] == 0x00) {  // padding
          n++;
          continue;
        }
        u8 id;
        int pl;
        if (h.extProfile == 0xBEDE) {
          id = buf[n] >> 4;
          pl = (buf[n] & 0x0f) + 1;
          n++;
          if (id == 15) break;  // extensionIDReserved
        } else {
          id = buf[n];
          n++;
          if (len <= n) return false;
          pl = buf[n];
          n++;
        }
        if (len <= n + pl) return false;
        if (h.nExt < 16) {
          h.extId[h.nExt] = id;
          h.extOff[h.nExt] = n;
          h.extLen[h.nExt] = pl;
          h.nExt++;
        }
        n += pl;
      }
    } else {  // RFC 3550 extension: one element, id 0
      h.extId[0] = 0;
      h.extOff[0] = n;
      h.extLen[0] = extEnd - n;
      h.nExt = 1;
      n = extEnd;
    }
  }
  int end = len;
  if (h.padding) {
    if (end <= n) return false;
    h.paddingSize = buf[end - 1];
    end -= h.paddingSize;
  }
  if (end < n) return false;
  h.hdrSize = n;
  h.payloadLen = end - n;
  return true;
}

// -----------------------------------------------------------------------------
// buffer.IsH264KeyFrame helpers.go:248-309 / IsAV1KeyFrame :343-420
// (restated as written, including the AV1 W-field OBU walk)
// -----------------------------------------------------------------------------
inline bool IsH264KeyFrame(const u8 *p, int n) {
  if (n < 1) return false;
  const int nalu = p[0] & 0x1F;
  if (nalu == 0) return false;
  if (nalu <= 23) return nalu == 7;
  if (nalu == 24 || nalu == 25 || nalu == 26 || nalu == 27) {
    int i = 1;
    if (nalu == 25 || nalu == 26 || nalu == 27) i += 2;
    while (i < n) {
      if (i + 2 > n) return false;
      const int length = (int(p[i]) << 8) | int(p[i + 1]);
      i += 2;
      if (i + length > n) return false;
      int offset = 0;
      if (nalu == 26)
        offset = 3;
      else if (nalu == 27)
        offset = 4;
      if (offset >= length) return false;
      const int nn = p[i + offset] & 0x1F;
      if (nn == 7) return true;
      i += length;
    }
    return false;
  }
  if (nalu == 28 || nalu == 29) {
    if (n < 2) return false;
    if ((p[1] & 0x80) == 0) return false;
    return (p[1] & 0x1F) == 7;
  }
  return false;
}

inline bool IsAV1KeyFrame(const u8 *payload, int n) {
  if (n < 2) return false;
  if ((payload[0] & 0x88) != 0x08) return false;  // Z=0, N=1
  const int w = (payload[0] & 0x30) >> 4;
  // getObu(data, last) -> (obu ptr/len, consumed length, truncated)
  auto getObu = [](const u8 *data, int dn, bool last, const u8 *&obu, int &olen, int &length, bool &trunc) {
    trunc = false;
    if (last) {
      obu = data;
      olen = dn;
      length = dn;
      return;
    }
    int offset = 0, len = 0;
    for (;;) {
      if (dn <= offset) {
        obu = nullptr;
        olen = 0;
        length = offset;
        trunc = offset > 0;
        return;
      }
      const u8 l = data[offset];
      len |= int(l & 0x7f) << (offset * 7);
      offset++;
      if ((l & 0x80) == 0) break;
    }
    if (dn < offset + len) {
      obu = data + offset;
      olen = dn - offset;
      length = dn;
      trunc = true;
      return;
    }
    obu = data + offset;
    olen = len;
    length = offset + len;
  };
  int offset = 1, i = 0;
  for (;;) {
    const u8 *obu;
    int olen, length;
    bool truncated;
    getObu(payload + offset, n - offset, w == i + 1, obu, olen, length, truncated);
    if (olen < 1) return false;
    const int tpe = (obu[0] & 0x38) >> 3;
    if (i == 0) {
      if (tpe != 1) return false;  // OBU_SEQUENCE_HEADER
    } else if (tpe == 3 || tpe == 6) {  // OBU_FRAME_HEADER / OBU_FRAME
      if (olen < 2) return false;
      if ((obu[1] & 0x80) != 0) return false;  // show_existing_frame
      return (obu[1] & 0x60) == 0;             // KEY_FRAME
    }
    if (truncated || i >= w) return false;
    offset += length;
    i++;
  }
}

}  // namespace orc
