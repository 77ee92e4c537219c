// nack_oracle.h — TEST INFRASTRUCTURE (CPU oracle), never linked into the
// product library.
//
// The receive-side NACK queue of buffer.Buffer: mediatransportutil's
// nack.NackQueue (github.com/livekit/mediatransportutil
// v0.0.0-20231213075826-cccbf2b93d3f, go.mod:20, pkg/nack/nack.go — not
// vendored in /root/reference), restated from its published source, as
// Buffer uses it:
//   Bind: nacker = nack.NewNACKQueue(nack.NackQueueParamsDefault) for a codec
//         with NACK feedback, not for audio/red   (buffer.go:248-256)
//   SetRTT(rtt) when rtt != 0                      (buffer.go:400-414)
//   updateStreamState: Remove(hdr SN), then Push(uint16(lost)) for lost in
//         [LossStartInclusive, LossEndExclusive)   (buffer.go:545-567)
//   calc's deferred doNACKs: Pairs() -> RTCP TransportLayerNack{SenderSSRC =
//         MediaSSRC = mediaSSRC, Nacks}, rtpStats.UpdateNack(numSeqNumsNacked)
//                                                  (buffer.go:417-421, :673-710)
// On the virtual clock every time.Now() of one calc is the datagram's
// arrival time (Buffer.Write calls calc(pkt, time.Now()), buffer.go:268-288).
// Pinned by buffer_test.go:50-161 (TestNack: five tries per lost SN with an
// RTT-scaled backoff, across the 16-bit wrap), transcribed in kat_nack.inc.
#pragma once
#include <cstdint>
#include <vector>

namespace orc {

// NackQueueParamsDefault
struct NackQueueParams {
  uint8_t MaxTries = 5;
  int CacheSize = 100;
  int64_t MinIntervalNs = 20000000;   // 20 ms
  int64_t MaxIntervalNs = 400000000;  // 400 ms
  // BackoffFactor 1.25: rtt * 1.25^k is exact in float64 for k <= 3 (the only
  // exponents getNack uses: tries - 1 with tries < MaxTries), so
  // time.Duration(float64(rtt) * math.Pow(1.25, k)) == (rtt * 5^k) / 4^k
};
constexpr uint32_t kNackDefaultRtt = 70;  // nack.go defaultRtt (ms)

struct NackPair {  // rtcp.NackPair
  uint16_t PacketID;
  uint16_t LostPackets;
};

class NackQueue {
 public:
  struct Nack {
    uint16_t seqNum;
    uint8_t tries;
    int64_t lastNackedAt;  // ns, virtual clock
  };
  NackQueueParams params;
  std::vector<Nack> nacks;
  uint32_t rtt = kNackDefaultRtt;

  void SetRTT(uint32_t r) { rtt = r; }

  void Remove(uint16_t sn) {
    for (size_t i = 0; i < nacks.size(); i++) {
      if (nacks[i].seqNum != sn) continue;
      nacks.erase(nacks.begin() + long(i));
      break;
    }
  }

  void Push(uint16_t sn, int64_t now) {
    if (int(nacks.size()) >= params.CacheSize) nacks.erase(nacks.begin());
    nacks.push_back(Nack{sn, 0, now});
  }

  // nack.getNack: (shouldSend, shouldRemove)
  void getNack(Nack &n, int64_t now, bool &send, bool &remove) const {
    send = remove = false;
    if (n.tries >= params.MaxTries) {
      remove = true;
      return;
    }
    int64_t required = 0;
    if (n.tries > 0) {
      required = params.MaxIntervalNs;
      uint64_t num = rtt, den = 1;
      for (int k = 0; k < int(n.tries) - 1; k++) {
        num *= 5;
        den *= 4;
      }
      const int64_t backoff = int64_t(num / den) * 1000000;
      if (backoff < required) required = backoff;
    }
    if (required < params.MinIntervalNs) required = params.MinIntervalNs;
    if (now - n.lastNackedAt < required) return;
    n.tries++;
    n.lastNackedAt = now;
    send = true;
  }

  // NackQueue.Pairs: the pairs to send now and numSeqNumsNacked
  std::vector<NackPair> Pairs(int64_t now, int &numNacked) {
    numNacked = 0;
    std::vector<NackPair> nps;
    if (nacks.empty()) return nps;
    uint16_t baseSN = uint16_t(nacks[0].seqNum - 17);  // far back: the first send opens a pair
    std::vector<uint16_t> purge;
    bool active = false;
    NackPair np{0, 0};
    for (auto &n : nacks) {
      bool send, remove;
      getNack(n, now, send, remove);
      if (remove) {
        purge.push_back(n.seqNum);
        continue;
      }
      if (!send) continue;
      numNacked++;
      const uint16_t sn = n.seqNum;
      if (uint16_t(sn - baseSN) > 16) {
        if (active) nps.push_back(np);
        baseSN = sn;
        np.PacketID = sn;
        np.LostPackets = 0;
        active = true;
      } else {
        // 1 << (sn - baseSN - 1) on uint16: a shift of 16 or more (sn == baseSN,
        // the uint16 difference minus one wraps) yields 0
        const uint16_t sh = uint16_t(uint16_t(sn - baseSN) - 1);
        if (sh < 16) np.LostPackets = uint16_t(np.LostPackets | (1u << sh));
      }
    }
    if (active) nps.push_back(np);
    for (uint16_t sn : purge) Remove(sn);
    return nps;
  }
};

}  // namespace orc
