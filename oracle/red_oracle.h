// =============================================================================
//  red_oracle.h — TEST INFRASTRUCTURE ONLY (checker of the GPU RED kernels).
//
//  CPU restatement of livekit-server v1.5.2's RED (RFC 2198) paths for Opus
//  (SURVEY.md §8(f) 3):
//    RedReceiver        pkg/sfu/redreceiver.go:40-207   primary Opus -> RED
//    RedPrimaryReceiver pkg/sfu/redprimaryreceiver.go:37-311  RED -> primary
//                       (+ recovery of lost packets from the redundant blocks)
//  Pinned by the reference's redreceiver_test.go (oracle/kat_red.inc).
// =============================================================================
#pragma once
#include <cstdint>
#include <vector>

namespace orc_red {
using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;

constexpr int maxRedCount = 2;     // redreceiver.go:31
constexpr int mtuSize = 1500;      // :32
constexpr u8 opusPT = 111;         // :37

struct Pkt {  // the rtp.Packet fields these paths read
  u16 sn = 0;
  u32 ts = 0;
  u8 pt = 0;
  std::vector<u8> payload;
};

enum Err { OK = 0, ErrIncompleteRedHeader, ErrIncompleteRedBlock, ErrRedSpace };

// encodeRedForPrimary redreceiver.go:163-207; returns the RED payload length
inline Err encodeRedForPrimary(std::vector<const Pkt *> redPkts, const Pkt &primary, std::vector<u8> &out) {
  size_t payloadSize = primary.payload.size() + 1;
  for (auto *p : redPkts) payloadSize += p->payload.size() + 4;
  if (payloadSize > size_t(mtuSize)) redPkts.clear();
  out.clear();
  for (auto *p : redPkts) {
    u32 h = u32(0x80 | opusPT);
    h <<= 14;
    h |= (primary.ts - p->ts) & 0x3FFF;
    h <<= 10;
    h |= u32(p->payload.size()) & 0x3FF;
    out.push_back(u8(h >> 24));
    out.push_back(u8(h >> 16));
    out.push_back(u8(h >> 8));
    out.push_back(u8(h));
  }
  out.push_back(opusPT);
  redPkts.push_back(&primary);
  for (auto *p : redPkts) {
    if (out.size() + p->payload.size() > size_t(mtuSize)) return ErrRedSpace;  // copy() short of space
    out.insert(out.end(), p->payload.begin(), p->payload.end());
  }
  return OK;
}

// RedReceiver: pktBuff history + encodeRedForPrimary (redreceiver.go:124-161)
struct RedEncoder {
  bool has[maxRedCount] = {false, false};
  Pkt buf[maxRedCount];
  Err Encode(const Pkt &pkt, std::vector<u8> &out) {
    int lastNil = -1;
    for (int i = maxRedCount - 1; i >= 0; i--)
      if (!has[i]) {
        lastNil = i;
        break;
      }
    std::vector<const Pkt *> red;
    for (int i = lastNil + 1; i < maxRedCount; i++) {
      const Pkt &prev = buf[i];
      if (pkt.sn == prev.sn || u16(pkt.sn - prev.sn) > u16(maxRedCount) || u32(pkt.ts - prev.ts) >= (1u << 14)) continue;
      red.push_back(&prev);
    }
    std::vector<Pkt> keep;  // red points into buf, which the insert below may rotate
    for (auto *p : red) keep.push_back(*p);
    for (int i = maxRedCount - 1; i >= 0; i--) {
      if (!has[i] || u16(pkt.sn - buf[i].sn) < (1u << 15)) {
        for (int j = 0; j < i; j++) {
          buf[j] = buf[j + 1];
          has[j] = has[j + 1];
        }
        buf[i] = pkt;
        has[i] = true;
        break;
      }
    }
    std::vector<const Pkt *> kp;
    for (auto &p : keep) kp.push_back(&p);
    return encodeRedForPrimary(kp, pkt, out);
  }
};

// extractPktsFromRed redprimaryreceiver.go:200-269.  The primary keeps the
// RED packet's header as written there (its payload type is not replaced).
inline Err extractPktsFromRed(const Pkt &red, u8 recoverBits, std::vector<Pkt> &pkts) {
  struct Block {
    u32 tsOffset = 0;
    size_t length = 0;
    u8 pt = 0;
    bool primary = false;
  };
  pkts.clear();
  const u8 *p = red.payload.data();
  size_t n = red.payload.size();
  std::vector<Block> blocks;
  size_t blockLength = 0;
  for (;;) {
    if (n < 1) return ErrIncompleteRedHeader;
    if ((p[0] & 0x80) == 0) {
      Block b;
      b.pt = p[0] & 0x7F;
      b.primary = true;
      blocks.push_back(b);
      p++;
      n--;
      break;
    }
    if (n < 4) return ErrIncompleteRedHeader;
    u32 h = (u32(p[0]) << 24) | (u32(p[1]) << 16) | (u32(p[2]) << 8) | u32(p[3]);
    Block b;
    b.length = h & 0x03FF;
    h >>= 10;
    b.tsOffset = h & 0x3FFF;
    h >>= 14;
    b.pt = u8(h & 0x7F);
    blocks.push_back(b);
    blockLength += b.length;
    p += 4;
    n -= 4;
  }
  if (n < blockLength) return ErrIncompleteRedBlock;
  for (size_t i = 0; i < blocks.size(); i++) {
    const Block &b = blocks[i];
    if (b.primary) {
      Pkt q;
      q.sn = red.sn;
      q.ts = red.ts;
      q.pt = red.pt;
      q.payload.assign(p, p + n);
      pkts.push_back(q);
      break;
    }
    const size_t recoverIndex = blocks.size() - i - 1;
    if (recoverIndex < 1 || (recoverBits & (1u << (recoverIndex - 1))) == 0) {
      p += b.length;
      n -= b.length;
      continue;
    }
    Pkt q;
    q.sn = u16(red.sn - u16(recoverIndex));
    q.ts = red.ts - b.tsOffset;
    q.pt = b.pt;
    q.payload.assign(p, p + b.length);
    pkts.push_back(q);
    p += b.length;
    n -= b.length;
  }
  return OK;
}

// RedPrimaryReceiver.getSendPktsFromRed redprimaryreceiver.go:145-198
struct RedDecoder {
  bool first = false;
  u16 lastSeq = 0;
  u8 pktHistory = 0;
  Err Decode(const Pkt &red, std::vector<Pkt> &pkts) {
    bool needRecover = false;
    if (!first) {
      lastSeq = red.sn;
      pktHistory = 0;
      first = true;
    } else {
      const u16 diff = u16(red.sn - lastSeq);
      if (diff == 0) {
      } else if (diff > 0x8000) {
        if (u16(65535 - diff) < 8) {
          pktHistory |= u8(1u << (65535 - diff));
          needRecover = true;
        }
      } else if (diff > 8) {
        lastSeq = red.sn;
        pktHistory = 0;
        needRecover = true;
      } else {
        lastSeq = red.sn;
        pktHistory = u8((u32(pktHistory) << diff) | (1u << (diff - 1)));
        needRecover = true;
      }
    }
    u8 recoverBits = 0;
    if (needRecover) {
      u16 bitIndex = u16(lastSeq - red.sn);
      for (int i = 0; i < maxRedCount; i++) {
        if (bitIndex > 7) break;
        if ((pktHistory & u8(1u << bitIndex)) == 0) recoverBits |= u8(1u << i);
        bitIndex++;
      }
    }
    return extractPktsFromRed(red, recoverBits, pkts);
  }
};

// extractPrimaryEncodingForRED redprimaryreceiver.go:271-311
inline Err extractPrimaryEncodingForRED(const std::vector<u8> &payload, std::vector<u8> &out) {
  const u8 *p = payload.data();
  size_t n = payload.size(), blockLength = 0;
  for (;;) {
    if (n < 1) return ErrIncompleteRedHeader;
    if ((p[0] & 0x80) == 0) {
      p++;
      n--;
      break;
    }
    if (n < 4) return ErrIncompleteRedHeader;
    blockLength += ((u32(p[2]) << 8) | p[3]) & 0x03FF;
    p += 4;
    n -= 4;
  }
  if (n < blockLength) return ErrIncompleteRedBlock;
  out.assign(p + blockLength, p + n);
  return OK;
}

}  // namespace orc_red
