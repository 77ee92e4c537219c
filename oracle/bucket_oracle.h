// Test infrastructure (CPU oracle): the receiver's packet bucket, the ring
// every Buffer keeps its packets in for NACK -> RTX reads.
//
// The algorithm lives in a third-party dependency absent from /root/reference:
// github.com/livekit/mediatransportutil v0.0.0-20231213075826-cccbf2b93d3f
// (go.mod:20), pkg/bucket.  Restated from its published algorithm; the
// reference's call sites anchor it:
//   - Buffer.calc adds every packet that survives the padding / SN-adjustment
//     steps with AddPacketWithSequenceNumber(pkt, adjusted SN) and produces no
//     ExtPacket when the add fails (ErrPacketTooOld, ErrRTXPacket)
//     (pkg/sfu/buffer/buffer.go:464-481);
//   - WebRTCReceiver.ReadRTP(buf, layer, sn) -> Buffer.GetPacket -> Bucket
//     .GetPacket (pkg/sfu/receiver.go:559-566, buffer.go:772-784; a closed
//     Buffer returns io.EOF), called by DownTrack.retransmitPackets with the
//     sequencer record's layer and sourceSeqNo (downtrack.go:1630);
//   - sizes: video buckets PacketBufferSize (500, config.go:326) slots, audio
//     200 slots, of MaxPktSize = 1500 bytes (buffer/factory.go:31-44).
// No reference test covers the bucket: parity unpinned (engine = this
// restatement on the same inputs; the RTX bytes read back are checked against
// the datagrams the trace generator wrote).
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace orc_bucket {

constexpr int kMaxPktSize = 1500;
constexpr uint16_t kInvalid = 65535;  // invalidPktSize

enum Err : int { OK = 0, TOO_OLD, RTX_PACKET, TOO_NEW, SIZE_INVALID, MISMATCH, TOO_LARGE };

struct Bucket {
  std::vector<uint8_t> buf;  // maxSteps slots: 2-byte size (big-endian), then the packet
  int maxSteps;
  bool init = false;
  int step = 0;  // the slot after the head's
  uint16_t headSN = 0;

  explicit Bucket(int slots) : buf(size_t(slots) * kMaxPktSize), maxSteps(slots) { invalidate(0, maxSteps); }

  int wrap(int s) const {
    while (s >= maxSteps) s -= maxSteps;
    while (s < 0) s += maxSteps;
    return s;
  }
  size_t offset(int s) const { return size_t(wrap(s)) * kMaxPktSize; }
  uint16_t be16(size_t o) const { return uint16_t((buf[o] << 8) | buf[o + 1]); }
  void put16(size_t o, uint16_t v) {
    buf[o] = uint8_t(v >> 8);
    buf[o + 1] = uint8_t(v);
  }
  void invalidate(int start, int n) {
    if (n > maxSteps) n = maxSteps;
    for (int i = 0; i < n; i++) put16(offset(start + i), kInvalid);
  }
  // the packet with its sequence number field set to sn (the adjusted SN the
  // Buffer stores it under, so GetPacket's stored-SN check matches it)
  void store(size_t off, const uint8_t *pkt, int len, uint16_t sn) {
    put16(off, uint16_t(len));
    std::memcpy(&buf[off + 2], pkt, size_t(len));
    put16(off + 2 + 2, sn);
  }

  // AddPacketWithSequenceNumber
  Err Add(const uint8_t *pkt, int len, uint16_t sn) {
    if (len > kMaxPktSize - 2) return TOO_LARGE;  // (the Go copy would run into the next slot)
    if (!init) {
      headSN = uint16_t(sn - 1);
      init = true;
    }
    const uint16_t diff = uint16_t(sn - headSN);
    if (diff == 0 || diff > (1u << 15)) {  // the head again, or older: set
      const int back = int(uint16_t(headSN - sn));
      if (back >= maxSteps) return TOO_OLD;
      const size_t off = offset(step - back - 1);
      if (be16(off) != kInvalid && be16(off + 2 + 2) == sn) return RTX_PACKET;  // do not overwrite a duplicate
      store(off, pkt, len, sn);
      return OK;
    }
    // push: invalidate the skipped slots, store at the head
    const int gap = int(diff) - 1;
    headSN = sn;
    invalidate(step, gap);
    store(offset(step + gap), pkt, len, sn);
    step = wrap(step + gap + 1);
    return OK;
  }

  // GetPacket: the stored bytes of sn
  Err Get(uint16_t sn, const uint8_t *&p, int &len) const {
    const int diff = int(int16_t(uint16_t(headSN - sn)));
    if (diff < 0) return TOO_NEW;
    if (diff >= maxSteps) return TOO_OLD;
    const size_t off = offset(step - diff - 1);
    const uint16_t sz = be16(off);
    if (sz == kInvalid) return SIZE_INVALID;
    if (be16(off + 2 + 2) != sn) return MISMATCH;
    p = &buf[off + 2];
    len = sz;
    return OK;
  }
};

}  // namespace orc_bucket
