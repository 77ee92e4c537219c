// fwd_state.h — HBM layout of the MI355X forwarding engine's per-DownTrack
// state (shared by the host engine and the HIP kernels).
//
// Hot state (DTHot, 256 B AoS, one per DownTrack) holds every field the
// per-packet recurrence touches on the common path: RTPMunger
// (rtpmunger.go:73-92) incl. the open range of its RangeMap, the Forwarder
// scalars (forwarder.go:187-215), the VideoLayerSelector layers
// (videolayerselector/base.go), the VP8 munger scalars (codecmunger/vp8.go:52-70),
// the sequencer head (sequencer.go:82-95) and the RTPStatsSender start point
// (rtpstats_sender.go:245-262).  A decide lane loads it once per batch into
// registers and stores it back once (2 x 256 B per active DownTrack).
//
// Cold state (rare paths only): the RTPMunger RangeMap's closed ranges
// (ring of 100), the VP8 munger's missing/dropped/exempted picture-id maps
// (rings), and the sequencer packetMeta ring (seq_size x 32 B).
#pragma once
#include <stdint.h>

namespace lkf {

constexpr int kRangeCap = 100;      // NewRangeMap(100) rtpmunger.go:97 (closed ranges)
constexpr int kMissCap = 100;       // 50 kept + 50 staging (exact orderedmap trim semantics)
constexpr int kMissKeep = 50;       // missingPictureIdsThreshold vp8.go:28
constexpr int kDropKeep = 20;       // droppedPictureIdsThreshold vp8.go:29
constexpr int kExemptKeep = 20;     // exemptedPictureIdsThreshold vp8.go:30
constexpr int kSetCap = 24;         // 20 kept (+ transient), 16-B multiple for wide copies

// DTHot.flags
enum : uint32_t {
  F_MUTED = 1u << 0,
  F_PUBMUTED = 1u << 1,
  F_STARTED = 1u << 2,
  F_RESUME_BEHIND = 1u << 3,  // resumeBehindThreshold == 0.2 (else 0.0)
  F_DEFICIENT = 1u << 4,      // lastAllocation.IsDeficient
  F_LAST_MARKER = 1u << 5,
  F_SECOND_LAST_MARKER = 1u << 6,
  F_RTX_GATE = 1u << 7,
  F_WR_MAX_MBIT = 1u << 8,
  F_PICID_USED = 1u << 9,
  F_TL0_USED = 1u << 10,
  F_TID_USED = 1u << 11,
  F_KEYIDX_USED = 1u << 12,
  F_SEQ_INIT = 1u << 13,
  F_STATS_INIT = 1u << 14,
  F_PLAYOUT_ACKED = 1u << 15,
  F_VIDEO = 1u << 16,
  F_VP8 = 1u << 17,        // codecmunger.VP8 attached
  F_SIMULCAST = 1u << 18,  // videolayerselector.Simulcast
  F_TLS_VP8 = 1u << 19,    // temporallayerselector.VP8
  F_HAS_EXPECTED = 1u << 20,
  F_ACTIVE = 1u << 21,
  F_VP9 = 1u << 22,  // videolayerselector.VP9 (SVC without dependency descriptor)
  F_DD = 1u << 23,   // videolayerselector.DependencyDescriptor (VP9 / AV1 with the DD extension)
  F_SEQ_RM = 1u << 24,  // the sequencer's RangeMap holds padding exclusions (SeqRM, sequencer.go:211-261)
};

// The video sequencer's RangeMap((size + 1) / 2) (sequencer.go:97-110).  Only
// pushPadding (WritePaddingRTP, downtrack.go:814-816) changes it; until then
// it maps every sequence number to 0 and no kernel reads it (F_SEQ_RM clear).
// One region per DownTrack: this header, then `cap` closed ranges (a ring,
// oldest at head), region stride = seqrm_stride(cap).
struct alignas(16) SeqRM {
  uint64_t openStart, openValue;  // the open range
  uint64_t snOffset;              // sequencer.snOffset (updateSNOffset sequencer.go:334-345)
  uint32_t head, count;
};
static_assert(sizeof(SeqRM) == 32, "SeqRM header is 32 B");

struct alignas(16) DTHot {
  // ---- 64-bit ------------------------------------------------------------
  uint64_t extHighestIncomingSN;  // rtpmunger.go:76
  uint64_t extLastSN, extSecondLastSN, snOffset;
  uint64_t extLastTS, extSecondLastTS, tsOffset;
  uint64_t extRtxGateSn;
  uint64_t rmOpenStart, rmOpenValue;  // RangeMap open range (value of ranges[len-1])
  uint64_t extFirstTS, refTSOffset;   // forwarder.go:201,204
  int64_t preStartTime;               // ns, 0 == zero time
  uint64_t seqExtStartSN, seqExtHighestSN, seqExtHighestTS;
  int64_t seqStartMs;
  int64_t statsFirstTime;
  uint64_t statsExtStartTS;
  // ---- 32-bit ------------------------------------------------------------
  uint32_t flags;
  uint32_t lastSSRC;
  int32_t referenceLayerSpatial;
  int32_t maxS, maxT, seenS, seenT, tgtS, tgtT, ptgtS, ptgtT, curS, curT, prevS, prevT, reqS;
  int32_t wrMaxPictureId, wrTotalWrap, wrLastWrap;  // VP8PictureIdWrapHandler vp8.go:381
  int32_t extLastPictureId, pictureIdOffset;
  // ---- small -----------------------------------------------------------
  uint16_t rmHead, rmCount;
  uint8_t missHead, missCount, dropHead, dropCount, exHead, exCount;
  uint8_t lastTl0, tl0Off, lastKeyIdx, keyIdxOff;
  uint16_t seqHighSlot;  // seqExtHighestSN % seq_size (valid once F_SEQ_INIT)
  uint8_t pad[4];
};
static_assert(sizeof(DTHot) == 256, "DTHot must be 256 B");

// per-batch counters (lkf_stats as u64 words) and the partial copies the
// decide waves add into (stats buffer = (1 + kStatCopies) * kStatWords)
constexpr int kStatWords = 4 + LKF_DROP_NREASONS;
constexpr int kStatCopies = 64;

// Static per-DownTrack parameters (Bind-time: downtrack.go:362-432), 32 B.
struct alignas(16) DevDT {
  uint32_t track;
  uint32_t ssrc;
  uint8_t pt, extPlayout, extAbs, extDD;
  uint8_t playout[3];
  uint8_t active;
  uint8_t extTcc;   // transport-cc extension id (pion TWCC HeaderExtensionInterceptor), 0: none
  uint8_t pad[3];
  uint32_t twccGroup;  // transport-wide sequence counter (its transport's, or the DownTrack's own)
  uint32_t pad2[2];
};
static_assert(sizeof(DevDT) == 32, "DevDT must be 32 B");

struct RangeEntry {  // closed range of utils.RangeMap (rangemap.go:43-47)
  uint64_t start, end, value;
};
inline uint32_t seqrm_cap(uint32_t seqSize) { return (seqSize + 1) / 2 > 1 ? (seqSize + 1) / 2 : 1; }  // minRanges 1
inline uint64_t seqrm_stride(uint32_t cap) { return (sizeof(SeqRM) + uint64_t(cap) * sizeof(RangeEntry) + 15) & ~15ull; }

struct VP8Cold {  // ordered maps of codecmunger.VP8 (vp8.go:67-69) as rings
  int32_t missKey[kMissCap];
  int32_t missVal[kMissCap];
  int32_t dropKey[kSetCap];
  int32_t exKey[kSetCap];
};
static_assert(sizeof(VP8Cold) % 16 == 0, "VP8Cold must be 16-B granular");

struct alignas(16) SeqMeta {  // packetMeta sequencer.go:44-73 (32 B)
  uint16_t sourceSeqNo, targetSeqNo;
  uint32_t timestamp;
  uint32_t lastNack;
  uint8_t marker, nacked;
  int8_t layer;
  uint8_t codecLen;
  uint8_t codec[8];
  uint8_t pad[8];
};
static_assert(sizeof(SeqMeta) == 32, "SeqMeta must be 32 B");

// Decide -> emit hand-off record, one per forwarded tuple (24 B), written at
// slot_base[dt] + j (j = the DownTrack's forwarded ordinal in the batch).
// Only what emit cannot rebuild travels:
//   - the munged SN / TS as their low 32 bits: emit widens them against the
//     DownTrack's FwdBase (its first forwarded record of the batch); a record
//     beyond 2^31 of it is flagged T_WIDE and its full values kept aside;
//   - the munged VP8 descriptor as its three munged fields (picture id,
//     TL0PICIDX, KEYIDX): emit re-marshals it from them and the packet's own
//     descriptor bits (VP8.MarshalTo helpers.go:170-227), as decide did;
//   - the layer, the header length and the incoming header size are the
//     packet's (lkf_pkt) or recomputed by emit.
// RTPStatsSender.Update needs none of it: decide folds it in (ss_fold).
struct alignas(8) FwdRec {
  uint32_t sn, ts;    // low 32 bits of the munged extended SN / TS
  uint32_t pkt;
  uint32_t rel16;     // byte offset in the DownTrack's output region / 16 (packets are 16-B aligned)
  uint16_t outLen;
  uint8_t flags;      // lkf_out flags | T_DD | T_PLAYOUT | T_CODEC
  uint8_t ddLen;      // dependency-descriptor extension bytes (T_DD)
  uint32_t aux;       // T_CODEC: munged picture id | TL0PICIDX << 16 | KEYIDX << 24; T_DD: DD arena offset
};
static_assert(sizeof(FwdRec) == 24, "FwdRec must be 24 B");
struct alignas(16) FwdBase {  // per DownTrack and batch: its first forwarded record's munged SN / TS
  uint64_t sn, ts;
};
// a record's 64-bit value from its low 32 bits and the DownTrack's base
__host__ __device__ inline uint64_t widen32(uint64_t base, uint32_t lo) {
  return base + uint64_t(int64_t(int32_t(lo - uint32_t(base))));
}
// T_WIDE: the record's munged SN or TS lies 2^31 or more from its DownTrack's
// FwdBase (a source switch can move the munged timestamp that far, e.g. after
// a reference-layer offset change): its full values are in the batch's wide
// side array at the record's slot (written and read only for such records)
enum : uint8_t { T_WIDE = 0x10, T_DD = 0x20, T_PLAYOUT = 0x40, T_CODEC = 0x80 };

// ---- dependency descriptor (AV1 / VP9 SVC, §8(a) a9 + a16) -----------------
// Sizes at the reference's maxima (dependencydescriptorextension.go:65-68,
// dependencydescriptorreader.go:217-303): 32 decode targets and so up to 32
// chains, 64 templates; frame diffs are unbounded there except by the
// extension's length (a two-byte element carries at most 255 bytes), so:
//   - a structure's template frame diffs share one pool (5 bits each: at most
//     408 fit in 255 bytes);
//   - a frame keeps up to kDDFdInline frame diffs in its DDPkt; a longer list
//     (custom frame diffs, 6+ bits each: at most 340) goes to the batch's
//     spill array (k_dd_decode), a template's longer list stays in the pool.
// FrameChain.expectFrames (round 6: no longer capped at 16): every frame a
// chain can wait on lies in the decision cache's window around cLast, so the
// set is a 512-bit ring over [cLast - 256, cLast + 256) (dd_device.h) plus one
// frame beyond it for the packet whose frame number jumped ahead of cLast.
// Engine limits that remain: the structure ring kDDSlots structures per track,
// the spill array its capacity; beyond them a packet is flagged (error bit 16
// -> LKF_EINVAL / LKF_ENOSPC at lkf_sync), never decided silently.
constexpr int kDDChains = 32;      // MaxDecodeTargets (NumChains <= NumDecodeTargets)
constexpr int kDDFdPool = 416;     // template frame diffs of one structure (408 fit in 255 bytes)
constexpr int kDDFdInline = 8;     // frame diffs kept in a DDPkt
constexpr int kDDExpWords = 8;     // FrameChain.expectFrames: a 512-bit ring over [cLast - 256, cLast + 256)
constexpr int kDDExpRow = 10;      // u64 per chain row: the ring, the frame beyond it, padding (80 B)
constexpr int kDDSlots = 8;        // structure ring per track
constexpr int kDDMaxBytes = 255;   // marshalled DD (pion two-byte extension element)
constexpr int kSeqDDBytes = 256;   // a sequencer slot's ddBytes entry: length byte + kDDMaxBytes

struct DDTmpl {  // dependencydescriptor.FrameDependencyTemplate of a structure (32 B)
  uint8_t sid, tid;
  uint16_t nfd;        // frame diffs (1..16 each), at fdPool[fdOff ..) of the structure
  uint16_t fdOff;
  // marshalling a packet of this template without custom fields: the template
  // findBestTemplate picks (best) and the fields it must write custom (bestC:
  // 1 DTIs, 2 frame diffs, 4 chain diffs); set when the structure is read
  uint8_t best, bestC;
  uint64_t dtis;       // 2-bit DecodeTargetIndication per decode target
  uint32_t chains[4];  // 4-bit frame_chain_fdiff per chain (chain c: word c / 8, nibble c % 8)
};
static_assert(sizeof(DDTmpl) == 32, "DDTmpl must be 32 B");

constexpr int kDDSerBytes = 256;  // a serialized structure (an attaching descriptor is at most 255 B)
struct alignas(16) DDStruct {  // FrameDependencyStructure + ProcessFrameDependencyStructure
  uint8_t structureId, numDT, numChains, numTmpl;
  uint8_t numRes, pad;
  uint16_t nfdPool;            // template frame diffs in fdPool
  uint8_t protectedBy[32];     // DecodeTargetProtectedByChain
  uint16_t resW[4], resH[4];   // Resolutions (width, height)
  uint8_t dtTarget[32], dtS[32], dtT[32];  // decode targets sorted high -> low layer
  uint8_t pad2[8];
  DDTmpl t[64];
  uint8_t fdPool[kDDFdPool];
  // the structure as a descriptor that attaches it writes it (structureId
  // through the resolutions), serialized once when the forwarding side reads
  // it (k_dd_decode); serBits 0xffff: not writable (the marshal fails).
  // After the pool: decide never stages it (read from the ring in HBM)
  uint16_t serBits;
  uint8_t pad3[14];
  uint8_t ser[kDDSerBytes];
};
static_assert(sizeof(DDStruct) % 16 == 0, "DDStruct must be 16-B granular");
static_assert(__builtin_offsetof(DDStruct, t) % 16 == 0 && __builtin_offsetof(DDStruct, fdPool) % 16 == 0,
              "DDStruct staging granules");
__host__ __device__ inline uint32_t dd_tmpl_chain(const DDTmpl &t, int c) { return (t.chains[c >> 3] >> (4 * (c & 7))) & 0xfu; }
struct DDPkt;
__host__ __device__ inline uint32_t dd_chain_diff(const DDPkt &p, int c);

enum : uint8_t { DP_FIRST = 1, DP_LAST = 2, DP_ATTACHED = 4, DP_ACTIVE = 8, DP_VALID = 16 };
// where a frame's frame diffs are (DDPkt.fdKind): in fd[], in the parse-time
// structure's pool (fdRef = offset), in the batch's spill array (fdRef =
// offset), or not kept (the ingress parser, which needs only their count)
enum : uint8_t { FD_INLINE = 0, FD_POOL = 1, FD_SPILL = 2, FD_NONE = 3 };
struct alignas(16) DDPkt {  // one packet's parsed descriptor (k_dd_decode -> k_decide_dt), 96 B
  uint64_t extFN, extKFN;
  uint64_t dtis;         // FrameDependencies.DecodeTargetIndications (2 bits each)
  uint32_t activeMask;   // ActiveDecodeTargetsBitmask (valid with DP_ACTIVE)
  uint16_t frameNumber;
  uint16_t nfd;          // FrameDependencies.FrameDiffs: count (where: fdKind)
  uint8_t sid, tid, ndti, nchain, flags;  // flags: DP_*
  uint8_t extFlags;      // LKF_DD_*
  uint8_t slot;          // structure ring slot the descriptor was read with (attached: written to)
  uint8_t fdKind;        // FD_*
  uint8_t tmplIdx;       // the template the descriptor names (structure slot's index)
  uint8_t custom;        // custom fields present: 1 DTIs, 2 frame diffs, 4 chain diffs
  uint8_t pad[2];
  uint32_t fdRef;
  uint16_t fd[kDDFdInline];
  uint64_t chainDiffs[kDDChains / 8];  // FrameDependencies.ChainDiffs (8 bits each: chain c in word c / 8)
};
constexpr uint32_t kDDPktScalar = 48;  // the bytes of DDPkt before fd[] (the selector's fast path copies these)
static_assert(__builtin_offsetof(DDPkt, fd) == kDDPktScalar, "the scalar part ends where fd[] starts");
static_assert(sizeof(DDPkt) == 96, "DDPkt must be 96 B");
__host__ __device__ inline uint32_t dd_chain_diff(const DDPkt &p, int c) {
  return uint32_t(p.chainDiffs[c >> 3] >> (8 * (c & 7))) & 0xffu;
}

struct DDTrack {  // per-track structure-ring cursor (forwarding side)
  uint32_t cur;    // slot of the current structure
  uint32_t valid;  // a structure has been seen
  uint32_t pad[2];
};

// Per-DownTrack DependencyDescriptor selector state
// (videolayerselector/dependencydescriptor.go:27-43, selectordecisioncache.go:49-58,
// framechain.go:22-31, decodetarget.go:24-28, framenumberwrapper.go)
enum : uint32_t { DS_KF_VALID = 1, DS_HAS_MASK = 2, DS_HAS_PREV_MASK = 4, DS_FN_INIT = 8, DS_CACHE_INIT = 16 };
struct alignas(16) DDState {
  uint64_t cBase, cLast;        // SelectorDecisionCache(256, 80)
  uint64_t masks[8];            // 2 bits per entity
  uint64_t extKeyFrameNum;
  uint64_t fnLast, fnOffset;    // FrameNumberWrapper
  uint32_t flags;               // DS_*
  uint32_t mask, prevMask;      // activeDecodeTargetsBitmask / previous
  uint32_t dtActive;            // DecodeTarget.active, by position in the sorted list
  uint32_t chBroken, chActive, chUpdating;  // per chain
  uint8_t slot;                 // structure ring slot of d.structure
  uint8_t numChains, numTargets;  // len(d.chains), len(d.decodeTargets)
  uint8_t pad;
  uint8_t expFar[kDDChains];    // exp[c][8] holds a waited-on frame beyond the ring
  uint64_t pad2;                // (exp rows 16-B aligned)
  uint64_t exp[kDDChains][kDDExpRow];  // FrameChain.expectFrames (a set: see dd_device.h); rows < numChains staged
};
constexpr uint32_t kDDStateHead = 176;  // the bytes of DDState before exp[][] (always staged)
static_assert(sizeof(DDState) % 16 == 0, "DDState must be 16-B granular");
static_assert(__builtin_offsetof(DDState, exp) == kDDStateHead, "DDState head");

struct DevTrack {  // track table (24 x 4 B)
  uint32_t kind, codec, hasRefTS, clockRate;
  uint32_t layerOffsets[9];  // [ref*3 + layer]
  uint32_t ddIdx;            // index into the DD structure tables (0xffffffff: no DD selector)
  uint32_t pad[2];
};

// ---- ingress: one received stream = one buffer.Buffer (buffer.go:66-130) ----
// per-DownTrack totals since it was added (lkf_downtrack_summaries): written
// by the DownTrack's decide wave (no atomics: one wave per DownTrack)
struct DTCum {
  uint64_t packets, bytes;
  uint32_t flags;  // DTHot flags after the last batch (F_DEFICIENT)
  uint32_t pad;
  uint64_t pad2;
};
static_assert(sizeof(DTCum) == 32, "DTCum is 32 B");

// DownTrack.rtpStats: buffer.RTPStatsSender (rtpstats_sender.go:135-171 and
// the rtpStatsBase counters rtpstats_base.go:133-190 it updates per sent
// packet).  One per DownTrack, plus its gap histogram and its 4096-entry
// snInfo ring (u32 per slot: pktSize | hdrSize << 16 | flags << 24).
constexpr int kSnInfoSize = 4096;  // cSnInfoSize rtpstats_sender.go:30
constexpr int kGapBins = 101;      // cGapHistogramNumBins rtpstats_base.go:31
constexpr int kGapWords = 104;     // per-DownTrack histogram stride (16-B multiple)
struct alignas(16) SenderStats {
  uint64_t extStartSN, extHighestSN, extStartTS, extHighestTS;
  int64_t firstTime, highestTime;  // ns, virtual clock (packet arrival / call time)
  uint64_t lastTransit, lastJitterExtTimestamp;
  uint64_t bytes, headerBytes, bytesDuplicate, headerBytesDuplicate, bytesPadding, headerBytesPadding;
  uint64_t packetsDuplicate, packetsPadding, packetsOutOfOrder, packetsLost;
  double jitter, maxJitter;
  uint32_t frames, keyFrames, initialized, clockRate;
  uint32_t pad[4];
};
static_assert(sizeof(SenderStats) == 192, "SenderStats is 192 B");

// Forwarder.provisional: VideoAllocationProvisional (forwarder.go:96-106),
// one per DownTrack, written by lkf_provisional_prepare / lkf_allocate_all
struct alignas(16) ProvState {
  int64_t brs[3][4];                       // bitrates
  int32_t allocS, allocT;                  // allocatedLayer
  int32_t seenS, seenT, maxS, maxT, curS, curT;  // maxSeenLayer, maxLayer, currentLayer
  uint32_t avail;                          // availableLayers (bit set)
  uint32_t muted;                          // 1 muted, 2 pubMuted
  uint32_t pad[2];
};
static_assert(sizeof(ProvState) == 144, "ProvState is 144 B");

// StreamTrackerDependencyDescriptor (streamtracker_dd.go:27-289), one per DD
// track that has one (lkf_add_stream_tracker_dd)
enum : uint32_t { DT_PAUSED = 1, DT_STOPPED = 2, DT_WORKER = 4 };
struct alignas(16) DDTrkState {
  int64_t bytes[3][4], bitrate[3][4];
  int32_t maxS, maxT;
  uint32_t flags;         // DT_*
  uint32_t changedMask;   // onBitrateAvailable per spatial layer by the last report
  uint32_t notif[3];      // onStatusChanged calls per spatial layer
  int32_t lastNotified[3];
  uint32_t track, pad;
};
static_assert(sizeof(DDTrkState) % 16 == 0, "DDTrkState is 16-B granular");

constexpr int kHistWords = 64;  // cHistorySize 4096 bits (rtpstats_receiver.go:30)

struct DevStream {  // static stream parameters (64 B)
  uint32_t track;
  int32_t layer;
  uint32_t ssrc;
  uint32_t clockRate;
  uint8_t codec, levelExt, activeLevel, minPercentile;
  uint32_t observeDuration;  // ms
  uint32_t minActiveDuration;
  uint32_t ddIdx;          // index of the stream's DependencyDescriptorParser (0xffffffff: none)
  double smoothFactor;
  double activeThreshold;  // ConvertAudioLevel(ActiveLevel)
  uint8_t ddExt;           // dependency-descriptor extension id
  uint8_t nack;            // the Buffer has a NackQueue (NACK feedback negotiated)
  uint8_t closed;          // Buffer.Close (lkf_remove_track): datagrams are not processed
  uint8_t twccExt;         // transport-cc extension id (0: no TWCC responder)
  uint8_t pad1[12];
};
static_assert(sizeof(DevStream) == 64, "DevStream must be 64 B");

enum : uint32_t {
  S_INIT = 1u << 0,       // RTPStatsReceiver.initialized
  S_SN_INIT = 1u << 1,    // WrapAround sequenceNumber initialized
  S_TS_INIT = 1u << 2,    // WrapAround timestamp initialized
  S_LVL_TS_INIT = 1u << 3 // latestTSForAudioLevelInitialized
};

struct alignas(16) StreamHot {  // per-stream ingress state (256 B)
  // WrapAround<uint16, uint64> / WrapAround<uint32, uint64> (wraparound.go:33-186)
  uint64_t snCycles, snExtHighest, tsCycles, tsExtHighest;
  // padding-exclusion RangeMap(100) open range (buffer.go:134)
  uint64_t rmOpenStart, rmOpenValue;
  // RTPStatsReceiver counters
  uint64_t packetsLost, packetsOutOfOrder, packetsDuplicate, packetsPadding;
  uint64_t bytes, headerBytes, bytesDuplicate, headerBytesDuplicate, bytesPadding, headerBytesPadding, frames;
  uint64_t nacks;  // rtpStats.nacks: sequence numbers NACKed (UpdateNack, rtpstats_base.go:315-324)
  // AudioLevel (audiolevel.go:36-50)
  double smoothedLevel;
  int64_t lastObservedNs;
  uint32_t activeDuration, observedDuration;
  uint32_t tsStart, tsHighest;
  uint32_t latestTSForAudioLevel;
  uint32_t flags;
  uint16_t snStart, snHighest;
  uint16_t rmHead, rmCount;
  // rtpStatsBase timing and receive jitter (rtpstats_receiver.go:106-107,
  // :209-213, :237; rtpstats_base.go:775-810): virtual clock = arrival
  int64_t firstTime, highestTime;
  uint64_t lastTransit, lastJitterExtTs;
  double jitter, maxJitter;
  uint8_t loudest;
  uint8_t pad[15];
};
static_assert(sizeof(StreamHot) == 256, "StreamHot must be 256 B");

// One stream's NACK queue: mediatransportutil nack.NackQueue with
// NackQueueParamsDefault (MaxTries 5, CacheSize 100, MinInterval 20 ms,
// MaxInterval 400 ms, BackoffFactor 1.25) as buffer.Buffer drives it
// (buffer.go:545-567, :673-710).  Entries in queue order (oldest first),
// structure of arrays so a wave holds two entries per lane.
constexpr int kNackCap = 100;  // NackQueueParamsDefault.CacheSize
constexpr int kNackSlots = 128;
constexpr uint32_t kNackMaxTries = 5;
constexpr uint32_t kNackDefaultRtt = 70;  // nack.go defaultRtt (ms)
struct alignas(16) NackState {
  int64_t last[kNackSlots];   // lastNackedAt, ns (virtual clock)
  uint16_t sn[kNackSlots];    // seqNum
  uint8_t tries[kNackSlots];
  uint32_t count;             // entries
  uint32_t rtt;               // ms (SetRTT)
  uint64_t nacks;             // rtpStats.nacks (UpdateNack): kept here, not in StreamHot, because the
                              // queues run beside the next ingest's stream kernel, which rewrites StreamHot
};
static_assert(sizeof(NackState) % 16 == 0, "NackState must be 16-B granular");

struct alignas(16) IngParsed {  // k_ing_parse -> k_ing_stream / k_ing_out (48 B)
  uint32_t ts, ssrc;
  uint16_t sn, hdrSize, payloadLen;
  uint8_t paddingSize, flags;  // IP_*
  uint8_t level, b0, b1;
  uint8_t vfirst, vbits, vhs, tl0, tid, keyidx;
  uint16_t pid;
  uint32_t track;
  uint8_t vp9bits, sid;  // codecs.VP9Packet flags (LKF_VP9_*) and SID
  uint16_t ddOff;        // the DD extension payload (Header.GetExtension), ddLen 0: absent
  uint8_t ddLen;
  uint8_t pad[11];
};
static_assert(sizeof(IngParsed) == 48, "IngParsed must be 48 B");
// IP_VP8_BAD: the codec payload (VP8 or VP9) failed to unmarshal
enum : uint8_t { IP_OK = 1, IP_MARKER = 2, IP_LEVEL = 4, IP_VP8 = 8, IP_KF = 16, IP_VP8_BAD = 32, IP_VP9 = 64 };
// IP_VP8_BAD: the codec payload (VP8, or VP9 without a DD) failed to unmarshal

// One received stream's buffer.DependencyDescriptorParser
// (dependencydescriptorparser.go:35-61) with its FrameIntegrityChecker(180,
// 1024) (frameintegrity.go:150-211).  Its structures: two slots (current and
// the one an attached structure is read into).
constexpr int kFICFrames = 180, kFICPktWords = 16;
enum : uint32_t { DI_SEQ_INIT = 1, DI_FN_INIT = 2, DI_HAS_STRUCT = 4, DI_CUR = 8, DI_FC_INIT = 16, DI_PH_INIT = 32 };
struct alignas(16) DDIngState {
  uint64_t seqCycles, seqExtHighest, fnCycles, fnExtHighest;  // WrapAround<uint16,uint64> x2
  uint16_t seqStart, seqHighest, fnStart, fnHighest;
  uint32_t flags;  // DI_*
  uint32_t activeMask;
  uint64_t structureExtFN, activeExtSeq;
  uint64_t fcBase, fcLast, phBase, phLast;
  uint64_t phBits[kFICPktWords];
  uint64_t feStart[kFICFrames], feEnd[kFICFrames];
  uint8_t feFlags[kFICFrames];  // 1 hasStart, 2 hasEnd, 4 integrity
  uint8_t pad[12];
};
static_assert(sizeof(DDIngState) % 16 == 0, "DDIngState must be 16-B granular");
struct IngDD {  // k_ing_stream -> k_ing_out: one datagram's ExtDependencyDescriptor (32 B)
  uint64_t extFN, extKFN;
  uint16_t ddOff;
  uint8_t ddLen, flags;  // LKF_DD_*
  uint8_t present, sid, tid, pad;
  uint64_t pad2;
};

// Per-run batch descriptor: what changes from one lkf_run to the next for
// the prep-stage kernels (batch pointers, length, control-op count).  The host
// writes it at the head of the run's page-locked staging buffer; the run's
// first kernel (k_h2d) pulls it into device memory with the control ops, and
// the kernels after it read it there — so the prep stage is the same kernel
// sequence every run and is replayed as one HIP graph.
struct alignas(16) RunDesc {
  uint64_t pkts;   // const lkf_pkt *
  uint64_t arena;  // const uint8_t *
  uint64_t dd;     // const lkf_pkt_dd * (0: none)
  uint64_t nDev;   // const uint64_t *: the batch length on the device (an ingest), or 0
  uint32_t n;      // packets (with nDev: the launch bound)
  uint32_t nev;    // control ops staged behind the descriptor
  uint32_t evCap;  // staging capacity (ops): the lane list starts at 64 + 48 * evCap
  uint32_t pad[5];
};
static_assert(sizeof(RunDesc) == 64, "RunDesc is 64 B");

// internal control op (not an lkf_ctl op): a track's reference-layer offsets
// table from this packet on (lkf_sender_report / lkf_set_layer_offsets*):
// offsets[0..7] packed two per a[] word, offsets[8] in pad
constexpr int32_t kOpLayerOffsets = 100;
constexpr uint32_t kDTOffsWords = 12;  // per DownTrack offsets row (9 used)

struct DevEvent {  // one queued lkf_ctl op (48 B)
  uint32_t at;
  int32_t op;
  int64_t a[4];
  int64_t pad;
};

}  // namespace lkf
