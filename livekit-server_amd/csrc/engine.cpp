// engine.cpp — host side of liblkfwd.so (the C-ABI of include/lkfwd.h).
//
// Owns the HBM-resident per-DownTrack state and the per-batch scratch, turns
// queued control ops into a per-lane event list, and enqueues the batch
// pipeline (forward_kernels.hip).  There is no CPU forwarding path: every
// per-packet decision runs in the gfx950 kernels.
//
// Two-stage pipeline across batches.  Batch n's "decide" stage (batch init,
// track ranges, slot scan, k_decide, output scan) runs on the engine's
// high-priority decide stream after the caller's stream (which orders the
// batch's inputs); its "emit" stage (k_emit, counters) runs on a low-priority
// emit stream after an event.  The decide of batch n+1 depends only on decide
// n (DownTrack state), so it overlaps emit n.  Per-batch scratch and outputs are double-buffered by run
// parity: batch n's outputs stay valid until run n+2 is enqueued, and a
// device batch's input buffers must stay valid until its emit stage is done
// (lkf_sync, or the enqueue of run n+2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/lkfwd.h"
#include "fwd_state.h"
#include "kernels.h"

using namespace lkf;

namespace {

// Every device buffer the engine allocates, base -> bytes (all engines of the
// process).  Each device -> host copy of an engine buffer is checked against
// it (check_dev_range): a source range that does not lie inside one live
// allocation — a freed or reallocated buffer, or a length past the end — is
// reported as an error instead of reaching the copy engine.
struct DevRegistry {
  std::mutex m;
  std::map<uintptr_t, size_t> a;
};
DevRegistry &dreg() {
  static DevRegistry r;
  return r;
}

template <typename T>
hipError_t dalloc(T **p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  const hipError_t r = hipMalloc(reinterpret_cast<void **>(p), n * sizeof(T));
  if (r == hipSuccess) {
    std::lock_guard<std::mutex> g(dreg().m);
    dreg().a[reinterpret_cast<uintptr_t>(*p)] = n * sizeof(T);
  }
  return r;
}

hipError_t dfree(void *p) {
  if (p) {
    std::lock_guard<std::mutex> g(dreg().m);
    dreg().a.erase(reinterpret_cast<uintptr_t>(p));
  }
  return hipFree(p);
}

// [src, src + n) inside one live allocation of this registry
bool dev_range_ok(const void *src, size_t n) {
  const uintptr_t s = reinterpret_cast<uintptr_t>(src);
  std::lock_guard<std::mutex> g(dreg().m);
  auto it = dreg().a.upper_bound(s);
  if (it == dreg().a.begin()) return false;
  --it;
  return s >= it->first && n <= it->second && s - it->first <= it->second - n;
}

template <typename T>
static hipError_t grow(T **p, uint64_t &cap, uint64_t need) {
  if (need <= cap) return hipSuccess;
  if (*p) (void)dfree(*p);
  cap = std::max<uint64_t>(need, 1024);
  return dalloc(p, cap);
}

constexpr int kStatsWords = 4 + LKF_DROP_NREASONS;
constexpr uint32_t kIdle = 0xffffffffu;

// Per-batch device scratch, outputs and events (two of them, by run parity).
struct BatchCtx {
  uint32_t *dTBegin = nullptr, *dTEnd = nullptr, *dTRuns = nullptr, *dErr = nullptr;
  uint64_t *dSlotBase = nullptr, *dPartA = nullptr, *dPartB = nullptr, *dTot = nullptr;
  FwdRec *dRecs = nullptr;    // decide -> emit: forwarded records at slotBase[dt] + j
  FwdBase *dFBase = nullptr;  // per DownTrack: the base of its records' 32-bit SN / TS
  FwdBase *dWide = nullptr;   // per tuple slot: a T_WIDE record's full SN / TS
  uint32_t *dFwdCnt = nullptr;
  uint64_t *dFwdBytes = nullptr, *dRecBase = nullptr, *dByteBase = nullptr;
  uint32_t *dGFirst = nullptr;  // emit group g -> output position owning record 64g
  uint32_t *dTwccBase = nullptr;  // per DownTrack: the batch's first transport-wide sequence number
  uint32_t *dLayerList = nullptr, *dLayerBefore = nullptr, *dLayerCnt = nullptr;  // k_layer_index
  lkf_out *dOut = nullptr;
  uint8_t *dOutArena = nullptr;
  uint64_t *dStats = nullptr;
  lkf_pkt *dPktsOwn = nullptr;  // lkf_submit copies land here
  uint8_t *dArenaOwn = nullptr;
  lkf_raw_pkt *dRawPkts = nullptr;  // lkf_ingest copies land here
  uint64_t *dBktStore = nullptr;    // per datagram: what the bucket store copies (kernels.h BucketLaunch)
  // dependency descriptor (allocated with the first DD track): lkf_submit_dd
  // copies, decoded descriptors, marshalled DD bytes + their bump cursor
  lkf_pkt_dd *dDDIn = nullptr;
  DDPkt *dDDPkt = nullptr;
  uint8_t *dDDArena = nullptr;
  uint64_t *dDDUsed = nullptr;  // [0] the arena's bump cursor, [1] the spill's (u32)
  uint16_t *dDDSpill = nullptr;  // custom frame-diff lists longer than kDDFdInline (k_dd_decode)
  DevEvent *dEvents = nullptr;   // this batch's control ops (per-wave CSR)
  uint32_t *dEvOff = nullptr;
  uint32_t *dEvLane = nullptr;   // lane of each op (sorted), for k_ev_offsets
  uint64_t evCap = 0, evOffCap = 0, evLaneCap = 0;
  hipEvent_t prepped = nullptr;  // prep stage done (prep stream)
  hipEvent_t pulled = nullptr;   // the control-op pull from the staging buffer done (own stream)
  hipEvent_t decided = nullptr;  // decide stage done (decide stream)
  hipEvent_t sent = nullptr;     // sender statistics done (sender stream)
  hipEvent_t emitted = nullptr;  // emit stage done (emit stream)
  hipEvent_t ingested = nullptr;  // this context's ingest done (ingest stream)
  bool fromIngest = false;        // the pending batch of this context is an ingest's output
  // that ingest also prepared the batch (k_ing_out: track ranges, zeroed
  // counters) for this topology (tracks, DownTracks); lkf_run then skips
  // k_batch_init and k_track_ranges
  bool prepByIngest = false;
  uint32_t prepNT = 0, prepND = 0;
  uint64_t *dITotal = nullptr;    // that ingest's ExtPacket count (device; k_track_ranges reads it)
  bool used = false;
  // SRTP-protected copy of the output (lkf_protect; allocated on first use)
  uint8_t *dProt = nullptr;
  bool protectedRun = false;
  // the run's descriptor (device; k_h2d pulls it from the staging buffer)
  RunDesc *dDesc = nullptr;
  // page-locked, CPU-cached staging of the run's RunDesc + control-op CSR
  // (malloc + hipHostRegister; k_h2d reads it through the device mapping)
  uint8_t *stage = nullptr, *stageDev = nullptr;
  uint32_t stageCap = 0;  // ops
  // the prep stage (k_h2d ... layer index) and the decide stage's tail
  // (counters, output scan) as HIP graphs, captured for the engine's topology
  // epoch; replayed every run (one launch each instead of ~11)
  // (two prep graphs: [1] with the ingest's prep fused in — k_batch_init /
  // k_track_ranges left out — [0] without; a context alternating between an
  // ingest-prepared batch and another replays both instead of re-capturing)
  hipGraphExec_t gPrep[2] = {nullptr, nullptr}, gScan = nullptr, gCtl = nullptr;
  uint64_t gPrepEpoch[2] = {0, 0}, gScanEpoch = 0, gCtlEpoch = 0;
};

}  // namespace

struct lkf_engine {
  int dev = 0;
  // LKF_HOST_PROF=1: wall time of lkf_run's host sections (printed by lkf_destroy)
  bool hostProf = false;
  double hp[9] = {};  // pre, stage wait, csr build, launches, total, runs, staging copies; ingest total, ingests
  std::vector<uint32_t> fill;  // event CSR fill cursors
  std::vector<std::pair<uint32_t, uint32_t>> sortA, sortB;  // control-op radix sort (lane, index)
  hipStream_t own = nullptr;    // copies, lookups
  hipStream_t d2hS = nullptr;   // lkf_drain_run_async's device -> host copies (created on first use)
  hipStream_t prepS = nullptr;  // ingest + batch preparation (high priority)
  // the ingests' stream (Buffer.calc): the prep stream.  A stream of its own
  // (ingest n+1 beside batch n's preparation; a run's preparation waits for its
  // ingest's event, which stays) measured 9 % slower on every step shape, even
  // those without an ingest: one more high-priority stream than the runtime's
  // hardware queues, so two of the engine's streams shared one (r5 A/B)
  hipStream_t ingS = nullptr;
  hipStream_t decS = nullptr;   // decide stage (high priority)
  hipStream_t emitS = nullptr;  // emit stage (low priority)
  hipStream_t sendS = nullptr;  // sender statistics of a decided batch (low priority, beside its emit)
  // transport-wide sequence numbers (pion TWCC header-extension interceptor,
  // send-side BWE): a counter per transport (DownTracks bound to it count
  // together, in record order) or per unbound DownTrack
  std::vector<int32_t> dtTransport;
  uint32_t *dTwccCtrD = nullptr, *dTwccCtrT = nullptr, *dTwccTOff = nullptr, *dTwccTList = nullptr;
  uint32_t twccTCap = 0, twccListCap = 0, nTwccT = 0;
  bool anyTwcc = false, twccDirty = false;
  hipStream_t sideS = nullptr;  // an ingest's NACK queues, beside the rest of the ingest and the run
  hipEvent_t sideFork = nullptr, sideDone[2] = {nullptr, nullptr};
  bool sidePending[2] = {false, false};  // an ingest waits for the NACK queues of the one two back
  hipEvent_t bktDone[2] = {nullptr, nullptr};
  bool bktPending[2] = {false, false};   // ... and for its bucket copies
  hipStream_t cur = nullptr;    // caller's stream of the last lkf_run
  hipEvent_t inEv = nullptr;    // caller-stream work before a run
  hipEvent_t bktEv = nullptr;   // an ingest's bucket decisions (the sender stream copies after it)
  bool bktStorePending = false; // the next run's context waits for those copies
  lkf_cfg cfg{};
  std::string err;

  // topology (host mirror)
  std::vector<lkf_track_params> tracks;
  std::vector<uint32_t> trackDD;  // per track: DD table index or 0xffffffff
  std::vector<uint8_t> trackActive;  // 0 after lkf_remove_track
  std::vector<lkf_downtrack_params> dtp;
  std::vector<uint8_t> active;
  // the DownTrack's sequencer may hold padding exclusions (lkf_padding sent
  // packets): it is decided by k_decide_dt<true>, which carries that path
  std::vector<uint8_t> seqRM;
  bool schedDirty = true;
  std::vector<uint32_t> sched;   // lane -> dt (kIdle = padding)
  std::vector<int32_t> dtLane;   // dt -> lane (-1 inactive)
  std::vector<uint32_t> waveTrack;
  // topology added since the last flush (uploaded in one copy each)
  std::vector<DevTrack> pendTracks;
  std::vector<DTHot> pendHot;
  std::vector<DevDT> pendDTs;
  // ingress streams (host mirror + uploads pending)
  std::vector<lkf_stream_params> streams;
  std::vector<DevStream> pendStreams;
  bool spkDirty = true;

  // queued control ops
  struct Pend {
    uint32_t dt;
    DevEvent ev;
  };
  std::vector<Pend> pending;
  // topology epoch: bumped by every change the captured stage graphs depend
  // on (tables, schedule, DD / tracker allocations); a context re-captures
  // its graphs when its epoch is older
  uint64_t epoch = 1;
  uint64_t topoGen = 0;  // bumped by every topology change (tracks, DownTracks, streams, removals, rooms)
  bool useGraph = true;  // LKF_GRAPH=0: the stages as direct launches (A/B)
  bool debugDD = false;  // LKF_DEBUG_DD=1: report the DD cursors (diagnostic)

  // device: persistent state
  DevTrack *dTracks = nullptr;
  DTHot *dHot = nullptr;
  DTCum *dDTCum = nullptr;  // per DownTrack sendingPacket totals (lkf_downtrack_summaries)
  // per DownTrack RTPStatsSender (sender_kernels.hip): statistics, gap
  // histogram, snInfo ring; host-listed updates (padding / blank / RTX)
  SenderStats *dSS = nullptr;
  uint32_t *dSSGap = nullptr;
  uint32_t *dSSRing = nullptr;
  SenderUpd *dSSList = nullptr;
  uint32_t *dSSGroups = nullptr;
  uint32_t ssListCap = 0;
  int64_t rtxNow = 0;  // now_ns of the last lkf_rtx_lookup (the RTX packets' sendingPacket time)
  // sequencer ddBytes (sequencer.go:198-199) of the DownTracks that can forward
  // a dependency descriptor: [ring index][slot] kSeqDDBytes, grown on demand
  uint8_t *dSeqDD = nullptr;
  uint32_t *dSeqDDIdx = nullptr;   // per DownTrack: ring index or 0xffffffff
  uint32_t *dSeqDDList = nullptr;  // ring index -> DownTrack
  uint32_t nSeqDD = 0, seqDDCap = 0;
  std::vector<uint32_t> seqDDList;
  uint8_t *dRtxDD = nullptr;  // lkf_rtx_emit: per record kSeqDDBytes
  // the cooperative allocation pass: per DownTrack provisional state + call buffers
  ProvState *dProv = nullptr;
  lkf_prov_req *dProvReq = nullptr;
  lkf_alloc_group *dProvGroups = nullptr;
  uint8_t *dProvOut = nullptr;
  uint32_t provCap = 0, provGroupCap = 0;
  // dependency-descriptor stream trackers (lkf_add_stream_tracker_dd)
  DDTrkState *dDDTrk = nullptr;
  uint32_t *dTrackDDTrk = nullptr;  // track -> DD tracker (0xffffffff none), max_tracks
  std::vector<int32_t> trackDDTrk;
  uint32_t nDDTrk = 0, ddTrkCap = 0;
  int32_t *dDDTrkIds = nullptr;
  lkf_dd_tracker_status *dDDTrkOut = nullptr;
  uint64_t ddTrkIdsCap = 0, ddTrkOutCap = 0;
  uint32_t rtxDDCap = 0;
  DevDT *dDTs = nullptr;
  RangeEntry *dRm = nullptr;
  VP8Cold *dVc = nullptr;
  SeqMeta *dSeq = nullptr;
  uint32_t *dSched = nullptr;
  uint32_t *dWaveTrack = nullptr;
  uint32_t *dEvOff = nullptr;
  uint32_t *dPerm = nullptr;  // output position -> DownTrack (track-major)
  size_t schedCap = 0;
  DevEvent *dEvents = nullptr;
  uint64_t evCap = 0;
  uint64_t *dCum = nullptr;
  // sticky error word: every batch's decide/emit error bits (bits 0-7) and
  // every ingest's error bits (<< 8) are OR-ed in on the GPU; lkf_sync reports
  // and clears it (per-context error words are reused every kCtx runs)
  uint32_t *dSticky = nullptr;

  // dependency-descriptor selector tables (allocated with the first DD track)
  uint32_t nDDTracks = 0;
  bool ddAlloc = false;
  uint64_t ddArenaCap = 0;
  uint32_t ddSpillCap = 0;
  DDStruct *dDDStruct = nullptr;  // [ddIdx * kDDSlots + slot]
  DDTrack *dDDTrack = nullptr;
  DDState *dDDState = nullptr;    // per DownTrack
  size_t ddStateInit = 0;         // DownTracks whose DDState is zeroed
  uint32_t ddTrackInit = 0;
  std::vector<uint8_t> dtIsDD;    // per DownTrack: SVC (DD selector or VP9), scheduled in k_decide_dt<true>
  uint32_t ddLanes = 0;
  // ingress DependencyDescriptorParser per DD stream (allocated with the first)
  uint32_t nDDStreams = 0, ddStreamInit = 0;
  DDIngState *dDDIng = nullptr;      // [stream.ddIdx]
  DDStruct *dDDIngStruct = nullptr;  // [stream.ddIdx * 2 + DI_CUR slot]
  IngDD *dIngDD = nullptr;           // per datagram of an ingest

  // batch input for the next run
  const lkf_pkt_dd *curDD = nullptr;
  const lkf_pkt *curPkts = nullptr;
  const uint8_t *curArena = nullptr;
  uint32_t curN = 0;
  uint64_t curArenaLen = 0;
  bool haveBatch = false;
  const uint64_t *curNDev = nullptr;  // device-side batch length (ingest-produced batch)
  bool ingestStarted = false;         // this run's start event precedes its ingest

  // three batch contexts: batch n+1 is ingested/prepared while batch n decides
  // and batch n-1 emits (its buffers are not reused until n+2)
#ifndef LKF_CTX  // batch contexts in flight (A/B)
#define LKF_CTX 3
#endif
  static constexpr int kCtx = LKF_CTX;
  BatchCtx ctx[kCtx];
  uint64_t nRuns = 0;
  int lastCtx = -1;
  // pinned bounce buffer of the host drains (D2H into caller memory that may
  // be pageable goes through it, on the engine's own stream)
  uint8_t *bounce = nullptr, *bounceDev = nullptr;
  size_t bounceCap = 0;

  // NACK -> RTX scratch (grown on demand)
  lkf_nack *dNacks = nullptr;
  uint32_t *dNackG = nullptr, *dNackValid = nullptr;
  lkf_rtx *dRtx = nullptr;
  uint32_t rtxCap = 0;
  lkf_raw_pkt *dRtxSrc = nullptr;
  uint32_t *dRtxLen = nullptr;
  uint64_t *dRtxOff = nullptr;
  uint8_t *dRtxIn = nullptr, *dRtxOut = nullptr;
  uint64_t rtxInCap = 0, rtxOutCap = 0;

  // stream trackers (lkf_add_stream_tracker): device state, tick scratch
  TrackerState *dTrk = nullptr;
  uint32_t nTrk = 0, trkCap = 0;
  int32_t *dTrkIds = nullptr;
  lkf_tracker_status *dTrkOut = nullptr;
  uint64_t trkIdsCap = 0, trkOutCap = 0;
  // RED per-track state (lkf_red_encode / lkf_red_decode), allocated at first use
  RedEncState *dRedEnc = nullptr;
  RedDecState *dRedDec = nullptr;
  struct RedScratch {
    lkf_pkt *in = nullptr, *out = nullptr;
    uint8_t *inArena = nullptr, *outArena = nullptr;
    uint32_t *g = nullptr, *cnt = nullptr;
    int32_t *map = nullptr;
    uint64_t *off = nullptr;
    uint64_t inCap = 0, outCap = 0, inArenaCap = 0, outArenaCap = 0, gCap = 0, cntCap = 0, mapCap = 0, offCap = 0;
  } red;
  // lastAllocation.BandwidthRequested per DownTrack (lkf_allocate_optimal)
  lkf_allocation *dLastAlloc = nullptr;  // lastAllocation per DownTrack
  lkf_alloc_req *dAllocReq = nullptr;
  int64_t *dAllocCapacity = nullptr;
  lkf_allocation *dAllocOut = nullptr;
  uint32_t allocCap = 0;
  // the sequencers' padding RangeMaps (SeqRM regions) and padding scratch
  uint8_t *dSrm = nullptr;
  uint64_t srmStride = 0;
  uint32_t srmCap = 0;
  lkf_pad_req *dPadReq = nullptr;
  uint64_t *dPadOff = nullptr;  // [2 * cap]: record bases, then arena bases
  uint32_t *dPadCnt = nullptr;  // [2 * cap]: packets, then bytes
  uint32_t padCap = 0;
  lkf_out *dPadOut = nullptr;
  uint64_t padOutCap = 0;
  uint8_t *dPadArena = nullptr;
  uint64_t padArenaCap = 0;

  // seq lookup scratch
  uint16_t *dSns = nullptr;
  lkf_seq_meta *dSeqOut = nullptr;
  uint32_t *dSeqN = nullptr;
  uint32_t seqScratchCap = 0;

  // timing ring: [0] decide-stage start, [1] decide kernel start, [2] decide
  // kernel end (decide stream), [3] emit kernel start, [4] emit kernel end
  // (emit stream)
  static constexpr int kRing = 256;
  hipEvent_t ring[kRing][5] = {};
  uint32_t emitGrid = 2048;       // persistent grid-stride launch (LKF_EMIT_PERSISTENT=1)
  bool emitPersistent = false;
  uint32_t emitLdsPad = 5900;  // bytes of LDS reserved per emit workgroup of an ingest-fed batch (12 per CU)
  uint32_t emitCapFanout = 16;  // ... when the batch has fewer DownTracks per track than this
  uint32_t decideK = 0;  // DownTracks per decide wave (0: from the batch's packets per track)
  // SRTP protect (tables allocated with the first transport or lkf_protect)
  std::vector<lkf_transport_params> transports;
  lkf_transport_params *dTransports = nullptr;
  SrtpKeys *dSrtpKeys = nullptr;
  uint32_t transportCap = 0;
  uint32_t *dAesTab = nullptr;
  SrtpDT *dSrtpDT = nullptr;
  hipEvent_t protRing[256][2] = {};  // k_srtp_roc start / k_srtp_protect end per run (timing)
  std::vector<uint8_t> protRun;      // per ring slot: that run was protected
  // ingress (one buffer.Buffer per stream) + speakers
  uint32_t maxStreams = 0;
  DevStream *dStreams = nullptr;
  StreamHot *dStreamHot = nullptr;
  uint64_t *dHist = nullptr;
  uint32_t *dRxGap = nullptr;  // per stream RTPStatsReceiver gap histogram (kGapWords u32)
  RangeEntry *dStreamRings = nullptr;
  IngParsed *dParsed = nullptr;
  lkf_flow *dFlows = nullptr;
  uint32_t *dTwcc = nullptr;  // per datagram TWCC push word of the last ingest
  // the receivers' RTX buckets (kernels.h BucketState): per stream state, slot
  // tags / batch owners / bytes, per datagram slot
  BucketState *dBkt = nullptr;
  uint32_t *dBktTag = nullptr;
  uint64_t *dBktOwner = nullptr;
  uint32_t bktEpoch = 0;
  uint8_t *dBktRing = nullptr;
  uint64_t bktSlots = 0, bktCap = 0;
  int32_t *dBktStream = nullptr;
  uint16_t *dBktSn = nullptr;
  uint32_t bktReadCap = 0;
  uint32_t *dFwdFlag = nullptr;
  uint64_t *dPos = nullptr, *dIPartA = nullptr, *dIPartB = nullptr, *dITotal = nullptr;
  uint32_t *dITBegin = nullptr, *dITEnd = nullptr, *dITRuns = nullptr, *dIErr = nullptr;
  uint32_t *dIList = nullptr, *dIListCnt = nullptr;  // per-stream datagram lists (k_ing_lists)
  // The ingest scratch the NACK queues (side stream) and the bucket copies
  // (sender stream) read after the ingest chain has moved on: two sets,
  // alternating per ingest, so an ingest waits only for the side work of the
  // ingest two back.  The d* pointers above and below name the last ingest's set.
  struct IngSet {
    IngParsed *parsed = nullptr;
    lkf_flow *flows = nullptr;
    uint32_t *fwd = nullptr, *tBegin = nullptr, *tEnd = nullptr, *list = nullptr, *listCnt = nullptr;
    uint32_t *nackInfo = nullptr, *nackPairOff = nullptr, *nackPairCnt = nullptr;
    lkf_nack_pair *nackPairs = nullptr;
    NackIn *nackIn = nullptr;  // the NACK kernel's per-datagram input, in list order
  } ing[2];
  int ingPar = 0;
  // NACK queues (allocated with the first stream that has one) and the last
  // ingest's RTCP NACKs (per datagram result + bump-allocated pairs)
  NackState *dNack = nullptr;
  uint32_t *dNackInfo = nullptr, *dNackPairOff = nullptr, *dNackPairCnt = nullptr;
  lkf_nack_pair *dNackPairs = nullptr;
  uint32_t nackPairCap = 0;
  uint64_t *dNackRecPos = nullptr, *dNackPairPos = nullptr, *dNackTot = nullptr;
  uint64_t *dNackPartA = nullptr, *dNackPartB = nullptr;  // the compaction's scan partials (side stream)
  lkf_rtcp_nack *dNackOut = nullptr;
  lkf_nack_pair *dNackPairsOut = nullptr;
  uint32_t lastIngestN = 0;
  const lkf_raw_pkt *ingRaws = nullptr;  // the last ingest's datagram descriptors (device)
  // speaker ranking tables (rebuilt when topology changes)
  uint32_t nRooms = 0;
  uint32_t *dRoomPartOff = nullptr, *dPartId = nullptr, *dPartMicOff = nullptr, *dMics = nullptr, *dRoomId = nullptr;
  lkf_speaker *dSpkSlots = nullptr;
  uint32_t *dSpkCounts = nullptr;
  size_t spkCap = 0;
  std::vector<uint32_t> spkRoomIds;  // host copy of dRoomId
  // lkf_room_summaries_enqueue: the records' layout for (rows, k, s) and the
  // topology it was built for; two events order the caller's stream after the
  // packs (ingest and decide streams)
  std::vector<uint32_t> rsRooms;
  uint32_t rsK = 0, rsS = 0;
  uint64_t rsGen = ~0ull;
  int32_t *dRsRowEng = nullptr;
  uint32_t *dRsSlotOff = nullptr, *dRsSlotDts = nullptr;
  int64_t *dRsSlotSub = nullptr;
  hipEvent_t rsSpk = nullptr, rsDec = nullptr;
  // device -> host copies refused by the range check (CHKRANGE) since the last
  // lkf_debug_check of this engine (lkf_debug_check folds them in)
  std::atomic<uint64_t> rangeViolations{0};
  // Sender-report-driven reference-layer offsets (StreamTrackerManager,
  // streamtrackermanager.go:561-627): per track the newest sender report of
  // each layer and the offsets table as of the last queued change.  Queued
  // changes (track, at_pkt, table) expand into per-DownTrack ops of the next
  // lkf_run (kOpLayerOffsets); tracks[t].layer_offsets is the table as of the
  // last run (a DownTrack added now starts from it).
  struct TrackSR {
    uint64_t ntp[3] = {0, 0, 0};
    uint32_t rtp[3] = {0, 0, 0};
    uint8_t have[3] = {0, 0, 0};
    uint32_t offs[9] = {};
  };
  std::vector<TrackSR> trkSR;
  struct TrackOp {
    uint32_t track, at;
    uint32_t offs[9];
  };
  std::vector<TrackOp> trkOps;
  uint32_t *dDTOffs = nullptr;  // per DownTrack kDTOffsWords: the offsets its Forwarder reads
  // the current batch's descriptors / DD side array are engine allocations
  // (lkf_submit / lkf_ingest*) rather than the caller's (lkf_submit_device)
  bool curOwned = false, curDDOwned = false;
};

static int fail(lkf_engine *e, const char *what, hipError_t r) {
  char buf[256];
  snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(r));
  e->err = buf;
  return LKF_EHIP;
}
#define HIPCHK(call, what)                          \
  do {                                              \
    hipError_t _r = (call);                         \
    if (_r != hipSuccess) return fail(e, what, _r); \
  } while (0)

// NewForwarder + DetermineCodec + NewRTPMunger + videolayerselector.NewBase +
// newSequencer (forwarder.go:217-338, rtpmunger.go:94, base.go NewBase,
// sequencer.go:97) as the initial HBM state of one DownTrack.
static void init_hot(DTHot &h, const lkf_track_params &tp, const lkf_downtrack_params &p) {
  std::memset(&h, 0, sizeof(h));
  h.referenceLayerSpatial = -1;
  h.maxS = h.maxT = h.seenS = h.seenT = -1;
  h.tgtS = h.tgtT = h.ptgtS = h.ptgtT = -1;
  h.curS = h.curT = h.prevS = h.prevT = -1;
  h.reqS = -1;
  h.rmOpenStart = 0;  // NewRangeMap: initRanges(0, 0)
  h.rmOpenValue = 0;
  uint32_t f = F_ACTIVE;
  if (tp.kind == LKF_KIND_VIDEO) {
    f |= F_VIDEO;
    h.maxT = 3;  // vls.SetMaxTemporal(DefaultMaxLayerTemporal) forwarder.go:235-237
    const bool svc = tp.codec == LKF_CODEC_VP9 || tp.codec == LKF_CODEC_AV1;
    if (tp.codec == LKF_CODEC_VP8) f |= F_VP8 | F_SIMULCAST | F_TLS_VP8;
    if (tp.codec == LKF_CODEC_H264) f |= F_SIMULCAST;
    if (svc && tp.has_dd) f |= F_DD;                             // DependencyDescriptor :301-334
    if (tp.codec == LKF_CODEC_VP9 && !tp.has_dd) f |= F_VP9;      // VP9 selector
    if (tp.codec == LKF_CODEC_AV1 && !tp.has_dd) f |= F_SIMULCAST;  // AV1 without DD: Simulcast
  }
  if (p.has_expected_ts) f |= F_HAS_EXPECTED;
  h.flags = f;
  h.seqStartMs = p.bind_time_ns / 1000000;
}

static bool track_has_dd(const lkf_track_params &p) {
  return p.kind == LKF_KIND_VIDEO && p.has_dd && (p.codec == LKF_CODEC_VP9 || p.codec == LKF_CODEC_AV1);
}

static DevTrack to_dev_track(const lkf_track_params &p, uint32_t ddIdx) {
  DevTrack t;
  std::memset(&t, 0, sizeof(t));
  t.ddIdx = ddIdx;
  t.kind = p.kind;
  t.codec = p.codec;
  t.hasRefTS = p.has_ref_ts;
  t.clockRate = p.clock_rate;
  for (int r = 0; r < 3; r++)
    for (int l = 0; l < 3; l++) t.layerOffsets[r * 3 + l] = p.layer_offsets[r][l];
  return t;
}

// Waits for every queued stage (run, own and emit streams).
template <typename T>
static hipError_t stage_alloc(T **host, T **dev, size_t n) {
  const size_t bytes = (n * sizeof(T) + 4095) & ~size_t(4095);
  void *p = std::aligned_alloc(4096, bytes);
  if (!p) return hipErrorOutOfMemory;
  hipError_t r = hipHostRegister(p, bytes, hipHostRegisterMapped);
  if (r != hipSuccess) {
    std::free(p);
    return r;
  }
  void *d = nullptr;
  r = hipHostGetDevicePointer(&d, p, 0);
  if (r != hipSuccess) {
    (void)hipHostUnregister(p);
    std::free(p);
    return r;
  }
  *host = static_cast<T *>(p);
  *dev = static_cast<T *>(d);
  return hipSuccess;
}
template <typename T>
static void stage_free(T **host, T **dev) {
  if (*host) {
    (void)hipHostUnregister(*host);
    std::free(*host);
  }
  *host = *dev = nullptr;
}

static int drain_streams(lkf_engine *e) {
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  if (e->cur && e->cur != e->own) HIPCHK(hipStreamSynchronize(e->cur), "sync run stream");
  HIPCHK(hipStreamSynchronize(e->own), "sync own stream");
  HIPCHK(hipStreamSynchronize(e->ingS), "sync ingest stream");
  HIPCHK(hipStreamSynchronize(e->prepS), "sync prep stream");
  HIPCHK(hipStreamSynchronize(e->decS), "sync decide stream");
  HIPCHK(hipStreamSynchronize(e->emitS), "sync emit stream");
  if (e->sendS) HIPCHK(hipStreamSynchronize(e->sendS), "sync sender stream");
  if (e->sideS) HIPCHK(hipStreamSynchronize(e->sideS), "sync side stream");
  return LKF_OK;
}

// A device -> host copy whose source range is not inside one live engine
// allocation (a length past a buffer's end, a freed or reallocated buffer):
// refused with LKF_EHIP and counted (lkf_debug_check folds the count into its
// violation total).  A pageable D2H copy of such a range is what surfaces as
// "an illegal memory access" from the copy call itself (the runtime's staging
// copy reads the bad range) — round 2's recorded fault was exactly that
// (a drain of tot[3] bytes past the output arena).
// every engine's refusals, for lkf_debug_check(NULL) (the whole device)
static std::atomic<uint64_t> gRangeViolationsAll{0};
static int range_fail(lkf_engine *e, const void *src, size_t n, const char *what) {
  char buf[256];
  snprintf(buf, sizeof(buf), "internal: %s: device range [%p, +%zu) outside every live engine allocation", what, src,
           n);
  e->err = buf;
  e->rangeViolations.fetch_add(1, std::memory_order_relaxed);
  gRangeViolationsAll.fetch_add(1, std::memory_order_relaxed);
  return LKF_EHIP;
}
#define CHKRANGE(src, n, what)                                                     \
  do {                                                                             \
    if ((n) && !dev_range_ok(src, n)) return range_fail(e, src, n, what);          \
  } while (0)
static int copy_to_host(lkf_engine *e, void *dst, const void *src, size_t n, const char *what);
#define D2H(dst, src, n, what)                                   \
  do {                                                           \
    const int _rc = copy_to_host(e, dst, src, n, what);          \
    if (_rc) return _rc;                                         \
  } while (0)

// Device -> caller host memory, range-checked (CHKRANGE).  A page-locked
// destination is copied directly; a pageable one (numpy arrays, std::vector,
// the stack) through the engine's pinned bounce buffer on its own stream.
static int copy_to_host(lkf_engine *e, void *dst, const void *src, size_t n, const char *what) {
  constexpr size_t kChunk = size_t(16) << 20;
  CHKRANGE(src, n, what);
  hipPointerAttribute_t pa;
  if (hipPointerGetAttributes(&pa, dst) == hipSuccess && pa.type == hipMemoryTypeHost) {  // page-locked: direct
    HIPCHK(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost), what);
    return LKF_OK;
  }
  (void)hipGetLastError();  // (an unregistered pointer is not an error here)
  if (!e->bounce) {
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&e->bounce), kChunk, hipHostMallocDefault), "alloc bounce");
    e->bounceCap = kChunk;
  }
  for (size_t off = 0; off < n; off += kChunk) {
    const size_t k = std::min(kChunk, n - off);
    HIPCHK(hipMemcpyAsync(e->bounce, static_cast<const uint8_t *>(src) + off, k, hipMemcpyDeviceToHost, e->own), what);
    HIPCHK(hipStreamSynchronize(e->own), what);
    std::memcpy(static_cast<uint8_t *>(dst) + off, e->bounce, k);
  }
  return LKF_OK;
}

// hipMemcpy from pageable host memory may return before its DMA lands, and
// the engine's streams are non-blocking (they do not order against the null
// stream): every host-side upload ends with a device sync before any engine
// stream can read what it wrote.
static int upload_done(lkf_engine *e) {
  HIPCHK(hipDeviceSynchronize(), "upload sync");
  return LKF_OK;
}
static int sender_list(lkf_engine *e, std::vector<SenderUpd> &list);

// Orders the sender stream after everything queued so far on the decide, emit
// and own streams.  The per-run sender statistics run on the sender stream
// (long batches) or on the emit stream right after emit (short batches,
// k_sender_stats_thread); a control call that updates RTPStatsSender from the
// sender stream (padding, blank frames, RTX) must come after both, or a
// queued tick's Update and the call's load/store of the same SenderStats race.
static int sender_after_queued(lkf_engine *e) {
  for (hipStream_t s : {e->decS, e->emitS, e->own}) {
    HIPCHK(hipEventRecord(e->inEv, s), "event");
    HIPCHK(hipStreamWaitEvent(e->sendS, e->inEv, 0), "wait queued stage");
  }
  return LKF_OK;
}

// The DD selector tables and per-batch DD buffers, allocated when the first
// track with the dependency-descriptor selector appears (streams drained).
static int ensure_dd(lkf_engine *e) {
  const lkf_cfg &c = e->cfg;
  if ((e->nDDTracks || e->nDDStreams) && !e->ctx[0].dDDIn)  // ingest output / lkf_submit_dd input
    for (auto &x : e->ctx) HIPCHK(dalloc(&x.dDDIn, c.max_batch_pkts), "alloc dd in");
  if (e->nDDStreams && !e->dDDIng) {
    HIPCHK(dalloc(&e->dDDIng, e->maxStreams), "alloc dd parsers");
    HIPCHK(dalloc(&e->dDDIngStruct, size_t(e->maxStreams) * 2), "alloc dd parser structures");
    HIPCHK(hipMemset(e->dDDIngStruct, 0, size_t(e->maxStreams) * 2 * sizeof(DDStruct)), "dd parser structures reset");
    HIPCHK(dalloc(&e->dIngDD, c.max_batch_pkts), "alloc ingest dd");
  }
  if (e->nDDStreams > e->ddStreamInit) {  // a fresh parser per new DD stream
    HIPCHK(hipMemset(e->dDDIng + e->ddStreamInit, 0, size_t(e->nDDStreams - e->ddStreamInit) * sizeof(DDIngState)),
           "dd parser reset");
    e->ddStreamInit = e->nDDStreams;
  }
  if (e->ddAlloc || e->nDDTracks == 0) return LKF_OK;
  HIPCHK(dalloc(&e->dDDStruct, size_t(c.max_tracks) * kDDSlots), "alloc dd structures");
  HIPCHK(dalloc(&e->dDDTrack, c.max_tracks), "alloc dd tracks");
  HIPCHK(dalloc(&e->dDDState, c.max_downtracks), "alloc dd state");
  HIPCHK(hipMemset(e->dDDTrack, 0, size_t(c.max_tracks) * sizeof(DDTrack)), "dd tracks reset");
  HIPCHK(hipMemset(e->dDDStruct, 0, size_t(c.max_tracks) * kDDSlots * sizeof(DDStruct)), "dd structures reset");
  e->ddArenaCap = c.max_out_bytes / 4 + (1u << 20);
  e->ddSpillCap = uint32_t(std::min<uint64_t>(uint64_t(c.max_batch_pkts) * kDDFdInline + 4096, 0x7fffffffu));
  for (auto &x : e->ctx) {
    HIPCHK(dalloc(&x.dDDPkt, c.max_batch_pkts), "alloc dd pkts");
    HIPCHK(dalloc(&x.dDDArena, e->ddArenaCap), "alloc dd arena");
    HIPCHK(dalloc(&x.dDDUsed, 2), "alloc dd cursor");
    // (zeroed here too: k_layer_index zeroes it per batch, but recycled memory
    // must never be read as a cursor; DESIGN.md §6 round-5 cursor report)
    HIPCHK(hipMemset(x.dDDUsed, 0, 2 * sizeof(uint64_t)), "dd cursor reset");
    HIPCHK(dalloc(&x.dDDSpill, e->ddSpillCap), "alloc dd spill");
  }
  e->ddAlloc = true;
  return LKF_OK;
}

// Uploads tracks / DownTracks added since the last flush (contiguous tails).
static int flush_topology(lkf_engine *e) {
  if (e->pendTracks.empty() && e->pendDTs.empty() && e->pendStreams.empty()) return LKF_OK;
  e->epoch++;  // the stage graphs read the topology's sizes
  e->topoGen++;
  int rc = drain_streams(e);
  if (rc) return rc;
  rc = ensure_dd(e);
  if (rc) return rc;
  if (e->ddAlloc && e->ddStateInit < e->dtp.size()) {  // NewDependencyDescriptor: zero selector state
    HIPCHK(hipMemset(e->dDDState + e->ddStateInit, 0, (e->dtp.size() - e->ddStateInit) * sizeof(DDState)),
           "dd state reset");
    e->ddStateInit = e->dtp.size();
  }
  if (!e->pendTracks.empty()) {
    size_t first = e->tracks.size() - e->pendTracks.size();
    HIPCHK(hipMemcpy(e->dTracks + first, e->pendTracks.data(), e->pendTracks.size() * sizeof(DevTrack),
                     hipMemcpyHostToDevice),
           "tracks upload");
    e->pendTracks.clear();
  }
  if (!e->pendDTs.empty()) {
    size_t first = e->dtp.size() - e->pendDTs.size();
    HIPCHK(hipMemcpy(e->dHot + first, e->pendHot.data(), e->pendHot.size() * sizeof(DTHot), hipMemcpyHostToDevice),
           "hot upload");
    HIPCHK(hipMemcpy(e->dDTs + first, e->pendDTs.data(), e->pendDTs.size() * sizeof(DevDT), hipMemcpyHostToDevice),
           "dt upload");
    HIPCHK(hipMemset(e->dDTCum + first, 0, e->pendDTs.size() * sizeof(DTCum)), "dt totals reset");
    {  // the track's reference-layer offsets as of the last run (later changes arrive as ops)
      std::vector<uint32_t> ro(e->pendDTs.size() * kDTOffsWords, 0u);
      for (size_t i = 0; i < e->pendDTs.size(); i++)
        std::memcpy(&ro[i * kDTOffsWords], e->tracks[e->pendDTs[i].track].layer_offsets, 9 * sizeof(uint32_t));
      HIPCHK(hipMemcpy(e->dDTOffs + first * kDTOffsWords, ro.data(), ro.size() * sizeof(uint32_t),
                       hipMemcpyHostToDevice),
             "dt offsets upload");
    }
    {  // NewRTPStatsSender (downtrack.go:315): zero statistics at the track's clock rate
      std::vector<SenderStats> ss(e->pendDTs.size());
      std::memset(ss.data(), 0, ss.size() * sizeof(SenderStats));
      for (size_t i = 0; i < ss.size(); i++) ss[i].clockRate = e->tracks[e->pendDTs[i].track].clock_rate;
      HIPCHK(hipMemcpy(e->dSS + first, ss.data(), ss.size() * sizeof(SenderStats), hipMemcpyHostToDevice),
             "sender stats init");
      HIPCHK(hipMemset(e->dSSGap + first * kGapWords, 0, e->pendDTs.size() * kGapWords * sizeof(uint32_t)),
             "sender gap reset");
      HIPCHK(hipMemset(e->dSSRing + first * kSnInfoSize, 0, e->pendDTs.size() * kSnInfoSize * sizeof(uint32_t)),
             "sender ring reset");
    }
    {  // DownTracks that can forward a DD (its selector and a negotiated extension id): a ddBytes ring
      std::vector<uint32_t> idx;
      const uint32_t n0 = e->nSeqDD;
      for (size_t i = 0; i < e->pendDTs.size(); i++) {
        const uint32_t d = uint32_t(first + i);
        const bool dd = track_has_dd(e->tracks[e->dtp[d].track]) && e->dtp[d].ext_dd != 0;
        idx.push_back(dd ? e->nSeqDD++ : 0xffffffffu);
        if (dd) e->seqDDList.push_back(d);
      }
      if (e->nSeqDD > e->seqDDCap) {  // grow (the streams are drained): copy the rings already filled
        const uint32_t cap = std::max<uint32_t>(e->nSeqDD, 2 * e->seqDDCap);
        const size_t per = size_t(e->cfg.seq_size) * kSeqDDBytes;
        uint8_t *nr = nullptr;
        HIPCHK(dalloc(&nr, size_t(cap) * per), "alloc sequencer dd");
        HIPCHK(hipMemset(nr, 0, size_t(cap) * per), "sequencer dd reset");
        if (e->dSeqDD) {
          HIPCHK(hipMemcpy(nr, e->dSeqDD, size_t(n0) * per, hipMemcpyDeviceToDevice), "sequencer dd move");
          HIPCHK(dfree(e->dSeqDD), "free sequencer dd");
        }
        if (e->dSeqDDList) HIPCHK(dfree(e->dSeqDDList), "free sequencer dd list");
        HIPCHK(dalloc(&e->dSeqDDList, cap), "alloc sequencer dd list");
        e->dSeqDD = nr;
        e->seqDDCap = cap;
      }
      HIPCHK(hipMemcpy(e->dSeqDDIdx + first, idx.data(), idx.size() * sizeof(uint32_t), hipMemcpyHostToDevice),
             "sequencer dd index");
      if (e->nSeqDD > n0)
        HIPCHK(hipMemcpy(e->dSeqDDList, e->seqDDList.data(), e->nSeqDD * sizeof(uint32_t), hipMemcpyHostToDevice),
               "sequencer dd list");
    }
    e->pendHot.clear();
    e->pendDTs.clear();
  }
  if (!e->pendStreams.empty()) {
    const size_t first = e->streams.size() - e->pendStreams.size();
    const size_t k = e->pendStreams.size();
    {  // RTX buckets (buffer/factory.go:31-44): audio 200 slots, video PacketBufferSize
      std::vector<BucketState> bs(k);
      uint64_t need = 0;
      for (size_t i = 0; i < k; i++) {
        const bool audio = e->tracks[e->streams[first + i].track].kind == LKF_KIND_AUDIO;
        std::memset(&bs[i], 0, sizeof(BucketState));
        bs[i].base = uint32_t(e->bktSlots + need);
        bs[i].maxSteps = audio ? 200u : e->cfg.seq_size;
        need += bs[i].maxSteps;
      }
      const uint64_t total = e->bktSlots + need;
      if (!e->dBkt) HIPCHK(dalloc(&e->dBkt, e->maxStreams), "alloc buckets");
      if (total > e->bktCap) {
        const uint64_t cap = std::max<uint64_t>(total, 2 * e->bktCap);
        uint32_t *tag = nullptr;
        uint64_t *own = nullptr;
        uint8_t *ring = nullptr;
        HIPCHK(dalloc(&tag, cap), "alloc bucket tags");
        HIPCHK(dalloc(&own, cap), "alloc bucket owners");
        HIPCHK(hipMemset(own, 0, cap * sizeof(uint64_t)), "bucket owners init");  // (epochs start at 1)
        HIPCHK(dalloc(&ring, cap * kBktSlot), "alloc bucket ring");
        if (e->bktSlots) {
          HIPCHK(hipMemcpy(tag, e->dBktTag, e->bktSlots * 4, hipMemcpyDeviceToDevice), "bucket tags copy");
          HIPCHK(hipMemcpy(ring, e->dBktRing, e->bktSlots * kBktSlot, hipMemcpyDeviceToDevice), "bucket ring copy");
        }
        for (void *p : {static_cast<void *>(e->dBktTag), static_cast<void *>(e->dBktOwner),
                        static_cast<void *>(e->dBktRing)})
          if (p) HIPCHK(dfree(p), "free bucket");
        e->dBktTag = tag;
        e->dBktOwner = own;
        e->dBktRing = ring;
        e->bktCap = cap;
      }
      HIPCHK(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(e->dBktTag + e->bktSlots), 0xFFFF0000u, need),
             "bucket tags init");  // every slot invalid (NewBucket)
      HIPCHK(hipMemcpy(e->dBkt + first, bs.data(), k * sizeof(BucketState), hipMemcpyHostToDevice), "buckets upload");
      e->bktSlots = total;
    }
    bool anyNack = false;
    for (const auto &d : e->pendStreams) anyNack = anyNack || d.nack;
    if (anyNack && !e->dNack) {  // nack.NewNACKQueue for the first Buffer with NACK feedback
      const lkf_cfg &c = e->cfg;
      HIPCHK(dalloc(&e->dNack, e->maxStreams), "alloc nack queues");
      HIPCHK(hipMemset(e->dNack, 0, size_t(e->maxStreams) * sizeof(NackState)), "nack queues reset");
      e->nackPairCap = uint32_t(std::min<uint64_t>(uint64_t(c.max_batch_pkts) * 8 + 4096, 1u << 30));
      // + every stream's block for the lane-parallel form (kernels.h kNackFastPairs)
      const uint64_t pairsAll = uint64_t(e->nackPairCap) + uint64_t(e->maxStreams) * kNackFastPairs;
      if (pairsAll >= (1ull << 32)) {
        e->err = "too many streams for the NACK pair buffer";
        return LKF_ENOSPC;
      }
      for (auto &g : e->ing) {
        HIPCHK(dalloc(&g.nackInfo, c.max_batch_pkts), "alloc nack info");
        HIPCHK(dalloc(&g.nackPairOff, c.max_batch_pkts), "alloc nack pair offsets");
        HIPCHK(dalloc(&g.nackPairCnt, 1), "alloc nack pair count");
        HIPCHK(dalloc(&g.nackPairs, pairsAll), "alloc nack pairs");
        HIPCHK(dalloc(&g.nackIn, 3 * size_t(c.max_batch_pkts) + 64), "alloc nack inputs");
        HIPCHK(hipMemset(g.nackInfo, 0, size_t(c.max_batch_pkts) * sizeof(uint32_t)), "nack info reset");
        HIPCHK(hipMemset(g.nackPairCnt, 0, sizeof(uint32_t)), "nack count reset");
      }
      e->dNackInfo = e->ing[e->ingPar].nackInfo;
      e->dNackPairOff = e->ing[e->ingPar].nackPairOff;
      e->dNackPairCnt = e->ing[e->ingPar].nackPairCnt;
      e->dNackPairs = e->ing[e->ingPar].nackPairs;
      HIPCHK(dalloc(&e->dNackRecPos, c.max_batch_pkts), "alloc nack positions");
      HIPCHK(dalloc(&e->dNackPairPos, c.max_batch_pkts), "alloc nack pair positions");
      HIPCHK(dalloc(&e->dNackTot, 2), "alloc nack totals");
      const size_t npart = scan_state_words(c.max_batch_pkts);  // (the compaction's scan state)
      HIPCHK(dalloc(&e->dNackPartA, npart), "alloc nack scan state");
      HIPCHK(hipMemset(e->dNackPartA, 0, npart * sizeof(uint64_t)), "nack scan state reset");
      HIPCHK(dalloc(&e->dNackOut, c.max_batch_pkts), "alloc nack records");
      HIPCHK(dalloc(&e->dNackPairsOut, pairsAll), "alloc nack pairs out");
    }
    if (e->dNack) {  // each new queue: empty, the stream's initial RTT (0: defaultRtt)
      for (size_t i = 0; i < k; i++) {
        const uint32_t rtt = e->streams[first + i].rtt_ms ? e->streams[first + i].rtt_ms : kNackDefaultRtt;
        HIPCHK(hipMemcpy(&e->dNack[first + i].rtt, &rtt, sizeof(rtt), hipMemcpyHostToDevice), "nack rtt");
      }
    }
    std::vector<StreamHot> hot(k);
    for (auto &h : hot) {
      std::memset(&h, 0, sizeof(h));
      h.loudest = 127;  // silentAudioLevel (audiolevel.go:24)
    }
    HIPCHK(hipMemcpy(e->dStreams + first, e->pendStreams.data(), k * sizeof(DevStream), hipMemcpyHostToDevice),
           "streams upload");
    HIPCHK(hipMemcpy(e->dStreamHot + first, hot.data(), k * sizeof(StreamHot), hipMemcpyHostToDevice),
           "stream state upload");
    HIPCHK(hipMemset(e->dHist + first * kHistWords, 0, k * kHistWords * sizeof(uint64_t)), "history reset");
    HIPCHK(hipMemset(e->dRxGap + first * kGapWords, 0, k * kGapWords * sizeof(uint32_t)), "gap histogram reset");
    e->pendStreams.clear();
  }
  return upload_done(e);
}

extern "C" {

const char *lkf_version(void) { return "lkfwd 0.2 (gfx950)"; }

const char *lkf_last_error(const lkf_engine *e) { return e ? e->err.c_str() : "null engine"; }

lkf_engine *lkf_create(int hip_device, const lkf_cfg *cfg) {
  if (!cfg) return nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || hip_device < 0 || hip_device >= ndev) return nullptr;
  if (cfg->seq_size > 65535) return nullptr;
  auto *e = new lkf_engine();
  e->dev = hip_device;
  e->cfg = *cfg;
  if (e->cfg.seq_size == 0) e->cfg.seq_size = 500;
  if (hipSetDevice(hip_device) != hipSuccess) {
    delete e;
    return nullptr;
  }
  const lkf_cfg &c = e->cfg;
  bool ok = true;
  auto A = [&](hipError_t r) { ok = ok && (r == hipSuccess); };
  // decide is the batch-to-batch critical path: its waves should win CU slots
  // over the emit stage of the previous batch when both are resident.
  int leastPrio = 0, greatestPrio = 0;
  A(hipDeviceGetStreamPriorityRange(&leastPrio, &greatestPrio));
  A(hipStreamCreateWithFlags(&e->own, hipStreamNonBlocking));
  // LKF_CU_SPLIT=D (A/B): of every 32 CUs, D run the prep/decide streams and the
  // rest the emit stream (hipExtStreamCreateWithCUMask), so the latency-bound
  // decide and the HBM-bound emit of consecutive batches stop competing for
  // the same CUs; 0 (default): all CUs, decide at high priority
  int cuSplit = 0;
  if (const char *v = getenv("LKF_CU_SPLIT")) cuSplit = atoi(v);
  if (cuSplit > 0 && cuSplit < 32) {
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, hip_device);
    const uint32_t words = uint32_t((ncu + 31) / 32);
    std::vector<uint32_t> mA(words, 0), mB(words, 0);
    for (int i = 0; i < ncu; i++) ((i % 32) < cuSplit ? mA : mB)[size_t(i / 32)] |= 1u << (i % 32);
    A(hipExtStreamCreateWithCUMask(&e->decS, words, mA.data()));
    A(hipExtStreamCreateWithCUMask(&e->prepS, words, mA.data()));
    e->ingS = e->prepS;
    A(hipExtStreamCreateWithCUMask(&e->emitS, words, mB.data()));
    A(hipExtStreamCreateWithCUMask(&e->sendS, words, mB.data()));
  } else {
    // LKF_PRIO=<decide><prep><emit><sender> (A/B): h(igh) or l(ow) each;
    // default "hhll" (the decide and prep chain ahead of emit for free CU slots)
    const char *pr = getenv("LKF_PRIO");
    auto prio = [&](int i, bool hi) { return (pr && int(strlen(pr)) > i) ? (pr[i] == 'h' ? greatestPrio : leastPrio)
                                                                         : (hi ? greatestPrio : leastPrio); };
    A(hipStreamCreateWithPriority(&e->decS, hipStreamNonBlocking, prio(0, true)));
    A(hipStreamCreateWithPriority(&e->prepS, hipStreamNonBlocking, prio(1, true)));
    e->ingS = e->prepS;
    A(hipStreamCreateWithPriority(&e->emitS, hipStreamNonBlocking, prio(2, false)));
    A(hipStreamCreateWithPriority(&e->sendS, hipStreamNonBlocking, prio(3, false)));
  }
  // LKF_SIDE_CUS=N (A/B): the NACK queues' side stream on N of every 32 CUs
  // (the last N of each XCD's), so its long latency-bound waves leave the
  // other CUs to emit; 0 (default): every CU
  int sideCus = 0;
  if (const char *v = getenv("LKF_SIDE_CUS")) sideCus = atoi(v);
  if (sideCus > 0 && sideCus < 32) {
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, hip_device);
    const uint32_t words = uint32_t((ncu + 31) / 32);
    std::vector<uint32_t> m(words, 0);
    for (int i = 0; i < ncu; i++)
      if ((i % 32) >= 32 - sideCus) m[size_t(i / 32)] |= 1u << (i % 32);
    A(hipExtStreamCreateWithCUMask(&e->sideS, words, m.data()));
  } else {
    A(hipStreamCreateWithFlags(&e->sideS, hipStreamNonBlocking));
  }
  A(hipEventCreateWithFlags(&e->inEv, hipEventDisableTiming));
  A(hipEventCreateWithFlags(&e->bktEv, hipEventDisableTiming));
  A(hipEventCreateWithFlags(&e->sideFork, hipEventDisableTiming));
  for (int i = 0; i < 2; i++) {
    A(hipEventCreateWithFlags(&e->sideDone[i], hipEventDisableTiming));
    A(hipEventCreateWithFlags(&e->bktDone[i], hipEventDisableTiming));
  }
  e->cur = e->own;
  A(dalloc(&e->dTracks, c.max_tracks));
  A(dalloc(&e->dHot, c.max_downtracks));
  A(dalloc(&e->dDTCum, c.max_downtracks));
  A(dalloc(&e->dTwccCtrD, c.max_downtracks));
  if (ok) A(hipMemset(e->dTwccCtrD, 0, size_t(c.max_downtracks) * sizeof(uint32_t)));
  A(dalloc(&e->dSS, c.max_downtracks));
  A(dalloc(&e->dSeqDDIdx, c.max_downtracks));
  A(dalloc(&e->dSSGap, size_t(c.max_downtracks) * kGapWords));
  A(dalloc(&e->dSSRing, size_t(c.max_downtracks) * kSnInfoSize));
  A(dalloc(&e->dDTs, c.max_downtracks));
  A(dalloc(&e->dRm, size_t(c.max_downtracks) * kRangeCap));
  A(dalloc(&e->dVc, c.max_downtracks));
  A(dalloc(&e->dSeq, size_t(c.max_downtracks) * c.seq_size));
  e->srmCap = seqrm_cap(c.seq_size);
  e->srmStride = seqrm_stride(e->srmCap);
  A(dalloc(&e->dSrm, size_t(c.max_downtracks) * e->srmStride));
  A(dalloc(&e->dLastAlloc, c.max_downtracks));
  A(dalloc(&e->dCum, kStatsWords));
  A(dalloc(&e->dSticky, 4));
  A(dalloc(&e->dPerm, c.max_downtracks));
  A(dalloc(&e->dDTOffs, size_t(c.max_downtracks) * kDTOffsWords));
  const size_t nparts = scan_state_words(c.max_downtracks);  // the slot and output scans' state
  for (auto &x : e->ctx) {
    A(dalloc(&x.dTBegin, c.max_tracks));
    A(dalloc(&x.dTEnd, c.max_tracks));
    A(dalloc(&x.dTRuns, c.max_tracks));
    A(dalloc(&x.dErr, 4));
    A(dalloc(&x.dSlotBase, c.max_downtracks));
    A(dalloc(&x.dPartA, nparts));
    A(hipMemset(x.dPartA, 0, nparts * sizeof(uint64_t)));
    A(dalloc(&x.dTot, 4));
    A(dalloc(&x.dRecs, c.max_batch_tuples));
    A(dalloc(&x.dFBase, c.max_downtracks));
    A(dalloc(&x.dWide, c.max_batch_tuples));
    A(dalloc(&x.dFwdCnt, c.max_downtracks));
    A(dalloc(&x.dFwdBytes, c.max_downtracks));
    A(dalloc(&x.dRecBase, c.max_downtracks));
    A(dalloc(&x.dByteBase, c.max_downtracks));
    A(dalloc(&x.dGFirst, c.max_out_pkts / 64 + 2));
    A(dalloc(&x.dTwccBase, c.max_downtracks));
    A(dalloc(&x.dLayerList, 3 * size_t(c.max_batch_pkts) + 64));
    A(dalloc(&x.dLayerBefore, 3 * size_t(c.max_batch_pkts) + 64));
    A(dalloc(&x.dLayerCnt, 3 * size_t(c.max_tracks)));
    A(dalloc(&x.dOut, c.max_out_pkts));
    A(dalloc(&x.dOutArena, c.max_out_bytes + 64));
    A(dalloc(&x.dStats, size_t(kStatsWords) * (1 + kStatCopies)));
    A(dalloc(&x.dPktsOwn, c.max_batch_pkts));
    A(dalloc(&x.dArenaOwn, c.max_batch_arena + 64));
    A(dalloc(&x.dRawPkts, c.max_batch_pkts));
    A(dalloc(&x.dBktStore, c.max_batch_pkts));
    A(dalloc(&x.dDesc, 1));
    A(dalloc(&x.dEvents, 4096));
    A(dalloc(&x.dEvLane, 4096));
    x.evCap = x.evLaneCap = 4096;
    A(hipEventCreateWithFlags(&x.decided, hipEventDisableTiming));
    A(hipEventCreateWithFlags(&x.prepped, hipEventDisableTiming));
    A(hipEventCreateWithFlags(&x.pulled, hipEventDisableTiming));
    A(hipEventCreateWithFlags(&x.emitted, hipEventDisableTiming));
    A(hipEventCreateWithFlags(&x.ingested, hipEventDisableTiming));
    A(dalloc(&x.dITotal, 2));
    A(hipEventCreateWithFlags(&x.sent, hipEventDisableTiming));
  }
  for (auto &r : e->ring)
    for (auto &ev : r) A(hipEventCreate(&ev));
  e->maxStreams = c.max_streams ? c.max_streams : 3 * c.max_tracks;
  A(dalloc(&e->dStreams, e->maxStreams));
  A(dalloc(&e->dStreamHot, e->maxStreams));
  A(dalloc(&e->dHist, size_t(e->maxStreams) * kHistWords));
  A(dalloc(&e->dRxGap, size_t(e->maxStreams) * kGapWords));
  A(dalloc(&e->dStreamRings, size_t(e->maxStreams) * kRangeCap));
  for (auto &g : e->ing) {
    A(dalloc(&g.parsed, c.max_batch_pkts));
    A(dalloc(&g.flows, c.max_batch_pkts));
    A(dalloc(&g.fwd, c.max_batch_pkts));
    A(dalloc(&g.tBegin, c.max_tracks));
    A(dalloc(&g.tEnd, c.max_tracks));
    A(dalloc(&g.list, 3 * size_t(c.max_batch_pkts) + 64));
    A(dalloc(&g.listCnt, 3 * size_t(c.max_tracks)));
  }
  e->dParsed = e->ing[0].parsed;
  e->dFlows = e->ing[0].flows;
  A(dalloc(&e->dTwcc, c.max_batch_pkts));
  e->dFwdFlag = e->ing[0].fwd;
  A(dalloc(&e->dPos, c.max_batch_pkts));
  const size_t ipart = scan_state_words(c.max_batch_pkts);  // the ingest scan's state
  A(dalloc(&e->dIPartA, ipart));
  A(hipMemset(e->dIPartA, 0, ipart * sizeof(uint64_t)));
  A(dalloc(&e->dITotal, 2));
  e->dITBegin = e->ing[0].tBegin;
  e->dITEnd = e->ing[0].tEnd;
  A(dalloc(&e->dITRuns, c.max_tracks));
  A(dalloc(&e->dIErr, 4));
  e->dIList = e->ing[0].list;
  e->dIListCnt = e->ing[0].listCnt;
  if (ok) {
    A(hipMemset(e->dSeq, 0, size_t(c.max_downtracks) * c.seq_size * sizeof(SeqMeta)));
    // Every persistent table starts zeroed: hipMalloc hands back memory an
    // earlier engine of the process wrote, and no kernel may ever see those
    // bytes (the rings are read only below their counts, but a zero start
    // makes every batch's inputs the same from one process to the next).
    A(hipMemset(e->dRm, 0, size_t(c.max_downtracks) * kRangeCap * sizeof(RangeEntry)));
    A(hipMemset(e->dVc, 0, size_t(c.max_downtracks) * sizeof(VP8Cold)));
    A(hipMemset(e->dSrm, 0, size_t(c.max_downtracks) * e->srmStride));
    A(hipMemset(e->dHot, 0, size_t(c.max_downtracks) * sizeof(DTHot)));
    A(hipMemset(e->dDTs, 0, size_t(c.max_downtracks) * sizeof(DevDT)));
    A(hipMemset(e->dDTCum, 0, size_t(c.max_downtracks) * sizeof(DTCum)));
    A(hipMemset(e->dSeqDDIdx, 0xff, size_t(c.max_downtracks) * sizeof(uint32_t)));
    A(hipMemset(e->dTracks, 0, size_t(c.max_tracks) * sizeof(DevTrack)));
    A(hipMemset(e->dStreamHot, 0, size_t(e->maxStreams) * sizeof(StreamHot)));
    A(hipMemset(e->dStreamRings, 0, size_t(e->maxStreams) * kRangeCap * sizeof(RangeEntry)));
    A(hipMemset(e->dHist, 0, size_t(e->maxStreams) * kHistWords * sizeof(uint64_t)));
    {  // VideoAllocationDefault (forwarder.go:111-116)
      lkf_allocation d = {};
      d.pause_reason = 3;
      d.target_spatial = d.target_temporal = d.request_spatial = d.max_spatial = d.max_temporal = -1;
      std::vector<lkf_allocation> v(c.max_downtracks, d);
      A(hipMemcpy(e->dLastAlloc, v.data(), v.size() * sizeof(lkf_allocation), hipMemcpyHostToDevice));
    }
    A(hipMemset(e->dCum, 0, kStatsWords * sizeof(uint64_t)));
    A(hipMemset(e->dSticky, 0, 4 * sizeof(uint32_t)));
    for (auto &x : e->ctx) {
      A(hipMemset(x.dArenaOwn, 0, c.max_batch_arena + 64));
      A(hipMemset(x.dTot, 0, 4 * sizeof(uint64_t)));
      A(hipMemset(x.dStats, 0, size_t(kStatsWords) * (1 + kStatCopies) * sizeof(uint64_t)));
      A(hipMemset(x.dErr, 0, 4 * sizeof(uint32_t)));
    }
    // hipMemset runs on the null stream, which the engine's non-blocking
    // streams do not wait for: finish the initialisation before any batch
    // (a late zero-fill raced the first batch's arena copy and sequencer writes)
    A(hipDeviceSynchronize());
  }
  if (!ok) {
    lkf_destroy(e);
    return nullptr;
  }
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, hip_device);
  // emit is grid-stride with one-wave workgroups: 24 waves per CU saturate
  // HBM and leave wave slots for the next batch's decide stage.
  int perCU = 24;
  if (const char *v = getenv("LKF_EMIT_WG_PER_CU")) perCU = std::max(1, atoi(v));
  if (const char *v = getenv("LKF_EMIT_PERSISTENT")) e->emitPersistent = atoi(v) != 0;
  if (const char *v = getenv("LKF_EMIT_LDS")) e->emitLdsPad = uint32_t(std::max(0, atoi(v)));  // (A/B)
  if (const char *v = getenv("LKF_EMIT_CAP_FANOUT")) e->emitCapFanout = uint32_t(std::max(0, atoi(v)));
  if (const char *v = getenv("LKF_DECIDE_K")) e->decideK = uint32_t(std::min(8, std::max(0, atoi(v))));
  e->emitGrid = uint32_t(cus) * uint32_t(perCU);
  if (const char *v = getenv("LKF_HOST_PROF")) e->hostProf = atoi(v) != 0;
  if (const char *v = getenv("LKF_GRAPH")) e->useGraph = atoi(v) != 0;
  if (const char *v = getenv("LKF_DEBUG_DD")) e->debugDD = atoi(v) != 0;
  return e;
}

void lkf_destroy(lkf_engine *e) {
  if (!e) return;
  if (e->hostProf && e->hp[5] > 0)
    fprintf(stderr,
            "lkf host ms/run: pre %.4f stage-wait %.4f csr %.4f copies %.4f launches %.4f total %.4f (%d runs)\n",
            e->hp[0] / e->hp[5], e->hp[1] / e->hp[5], e->hp[2] / e->hp[5], e->hp[6] / e->hp[5],
            e->hp[3] / e->hp[5], e->hp[4] / e->hp[5], int(e->hp[5]));
  if (e->hostProf && e->hp[8] > 0)
    fprintf(stderr, "lkf host ms/ingest: %.4f (%d ingests: the launches of the Buffer.calc chain, no host wait)\n",
            e->hp[7] / e->hp[8], int(e->hp[8]));
  (void)hipSetDevice(e->dev);
  if (e->cur && e->cur != e->own) (void)hipStreamSynchronize(e->cur);
  if (e->own) (void)hipStreamSynchronize(e->own);
  if (e->ingS) (void)hipStreamSynchronize(e->ingS);
  if (e->prepS) (void)hipStreamSynchronize(e->prepS);
  if (e->decS) (void)hipStreamSynchronize(e->decS);
  if (e->emitS) (void)hipStreamSynchronize(e->emitS);
  if (e->sendS) (void)hipStreamSynchronize(e->sendS);  // (bucket copies, sender updates)
  if (e->sideS) (void)hipStreamSynchronize(e->sideS);  // (NACK queues)
  if (e->d2hS) (void)hipStreamSynchronize(e->d2hS);    // (asynchronous drains)
  (void)hipDeviceSynchronize();                        // (anything else queued before the buffers go)
  for (void *p : {static_cast<void *>(e->dNacks), static_cast<void *>(e->dNackG), static_cast<void *>(e->dNackValid),
                  static_cast<void *>(e->dRtx), static_cast<void *>(e->dRtxSrc), static_cast<void *>(e->dRtxLen),
                  static_cast<void *>(e->dRtxOff), static_cast<void *>(e->dRtxIn), static_cast<void *>(e->dRtxOut),
                  static_cast<void *>(e->dSrm), static_cast<void *>(e->dPadReq), static_cast<void *>(e->dPadOff),
                  static_cast<void *>(e->dPadCnt), static_cast<void *>(e->dPadOut), static_cast<void *>(e->dPadArena),
                  static_cast<void *>(e->dLastAlloc), static_cast<void *>(e->dAllocReq), static_cast<void *>(e->dAllocCapacity),
                  static_cast<void *>(e->dRedEnc), static_cast<void *>(e->dRedDec), static_cast<void *>(e->dTrk),
                  static_cast<void *>(e->dTrkIds), static_cast<void *>(e->dTrkOut),
                  static_cast<void *>(e->red.in), static_cast<void *>(e->red.out), static_cast<void *>(e->red.inArena),
                  static_cast<void *>(e->red.outArena), static_cast<void *>(e->red.g), static_cast<void *>(e->red.cnt),
                  static_cast<void *>(e->red.map), static_cast<void *>(e->red.off),
                  static_cast<void *>(e->dAllocOut)})
    if (p) (void)dfree(p);
  void *ptrs[] = {e->dTracks,  e->dHot,  e->dDTCum, e->dDTs,    e->dRm,  e->dVc,  e->dSeq,    e->dSched,
                  e->dWaveTrack, e->dCum, e->dSticky, e->dSns, e->dSeqOut, e->dSeqN, e->dPerm, e->dDTOffs,
                  e->dStreams, e->dStreamHot, e->dHist, e->dRxGap, e->dStreamRings,
                  e->dTwcc, e->dBkt, e->dBktTag, e->dBktOwner, e->dBktRing, e->dBktStream, e->dBktSn,
                  e->dPos, e->dIPartA, e->dIPartB, e->dITotal, e->dITRuns, e->dIErr,
                  e->dRoomPartOff, e->dPartId, e->dPartMicOff, e->dMics, e->dRoomId, e->dSpkSlots,
                  e->dSpkCounts, e->dNack, e->dRsRowEng, e->dRsSlotOff, e->dRsSlotDts, e->dRsSlotSub,
                  e->dNackRecPos, e->dNackPairPos, e->dNackTot, e->dNackOut, e->dNackPairsOut, e->dNackPartA,
                  e->dNackPartB,
                  e->dSS, e->dSSGap, e->dSSRing, e->dSSList, e->dSSGroups, e->dSeqDD, e->dSeqDDIdx,
                  e->dSeqDDList, e->dRtxDD, e->dProv, e->dProvReq, e->dProvGroups, e->dProvOut,
                  e->dDDTrk, e->dTrackDDTrk, e->dDDTrkIds, e->dDDTrkOut, e->dTwccCtrD,
                  e->dTwccCtrT, e->dTwccTOff, e->dTwccTList};
  for (void *p : ptrs)
    if (p) (void)dfree(p);
  for (void *p : {static_cast<void *>(e->dDDStruct), static_cast<void *>(e->dDDTrack),
                  static_cast<void *>(e->dDDState), static_cast<void *>(e->dDDIng),
                  static_cast<void *>(e->dDDIngStruct), static_cast<void *>(e->dIngDD)})
    if (p) (void)dfree(p);
  for (auto &r : e->protRing)
    for (auto &ev : r)
      if (ev) (void)hipEventDestroy(ev);
  for (void *p : {static_cast<void *>(e->dTransports), static_cast<void *>(e->dSrtpKeys),
                  static_cast<void *>(e->dAesTab), static_cast<void *>(e->dSrtpDT)})
    if (p) (void)dfree(p);
  for (auto &x : e->ctx) {
    if (x.dProt) (void)dfree(x.dProt);
    for (void *p : {static_cast<void *>(x.dDDIn), static_cast<void *>(x.dDDPkt), static_cast<void *>(x.dDDArena),
                    static_cast<void *>(x.dDDUsed), static_cast<void *>(x.dDDSpill)})
      if (p) (void)dfree(p);
    void *q[] = {x.dTBegin, x.dTEnd,     x.dTRuns,   x.dErr,      x.dSlotBase, x.dPartA,
                 x.dPartB,  x.dTot,      x.dRecs,  x.dFBase,  x.dWide,  x.dFwdCnt,   x.dFwdBytes, x.dRecBase,
                 x.dByteBase, x.dOut,    x.dOutArena, x.dStats,   x.dPktsOwn,  x.dArenaOwn,
                 x.dRawPkts, x.dBktStore, x.dGFirst, x.dLayerList, x.dLayerBefore, x.dLayerCnt, x.dEvents, x.dEvOff, x.dEvLane, x.dTwccBase};
    for (void *p : q)
      if (p) (void)dfree(p);
    if (x.decided) (void)hipEventDestroy(x.decided);
    if (x.prepped) (void)hipEventDestroy(x.prepped);
    if (x.pulled) (void)hipEventDestroy(x.pulled);
    if (x.emitted) (void)hipEventDestroy(x.emitted);
    if (x.ingested) (void)hipEventDestroy(x.ingested);
    if (x.dITotal) (void)dfree(x.dITotal);
    if (x.sent) (void)hipEventDestroy(x.sent);
  }
  for (auto &r : e->ring)
    for (auto &ev : r)
      if (ev) (void)hipEventDestroy(ev);
  for (auto &x : e->ctx) {
    stage_free(&x.stage, &x.stageDev);
    for (auto &g : x.gPrep)
      if (g) (void)hipGraphExecDestroy(g);
    if (x.gCtl) (void)hipGraphExecDestroy(x.gCtl);
    if (x.gScan) (void)hipGraphExecDestroy(x.gScan);
    if (x.dDesc) (void)dfree(x.dDesc);
  }
  if (e->bounce) (void)hipHostFree(e->bounce);
  if (e->inEv) (void)hipEventDestroy(e->inEv);
  if (e->bktEv) (void)hipEventDestroy(e->bktEv);
  for (hipEvent_t ev : {e->rsSpk, e->rsDec})
    if (ev) (void)hipEventDestroy(ev);
  if (e->sideFork) (void)hipEventDestroy(e->sideFork);
  for (int i = 0; i < 2; i++) {
    if (e->sideDone[i]) (void)hipEventDestroy(e->sideDone[i]);
    if (e->bktDone[i]) (void)hipEventDestroy(e->bktDone[i]);
  }
  for (auto &g : e->ing)
    for (void *p : {static_cast<void *>(g.parsed), static_cast<void *>(g.flows), static_cast<void *>(g.fwd),
                    static_cast<void *>(g.tBegin), static_cast<void *>(g.tEnd), static_cast<void *>(g.list),
                    static_cast<void *>(g.listCnt), static_cast<void *>(g.nackInfo), static_cast<void *>(g.nackPairOff),
                    static_cast<void *>(g.nackPairCnt), static_cast<void *>(g.nackPairs),
                    static_cast<void *>(g.nackIn)})
      if (p) (void)dfree(p);
  if (e->sideS && e->sideS != e->sendS) (void)hipStreamDestroy(e->sideS);
  if (e->emitS) (void)hipStreamDestroy(e->emitS);
  if (e->sendS) (void)hipStreamDestroy(e->sendS);
  if (e->decS) (void)hipStreamDestroy(e->decS);
  if (e->prepS) (void)hipStreamDestroy(e->prepS);
  if (e->ingS && e->ingS != e->prepS) (void)hipStreamDestroy(e->ingS);
  if (e->own) (void)hipStreamDestroy(e->own);
  if (e->d2hS) (void)hipStreamDestroy(e->d2hS);
  delete e;
}

int32_t lkf_add_track(lkf_engine *e, const lkf_track_params *p) {
  if (!e || !p) return LKF_EINVAL;
  if (e->tracks.size() >= e->cfg.max_tracks) return LKF_ENOSPC;
  int32_t h = int32_t(e->tracks.size());
  e->tracks.push_back(*p);
  uint32_t ddIdx = 0xffffffffu;
  if (track_has_dd(*p)) ddIdx = e->nDDTracks++;
  e->trackDD.push_back(ddIdx);
  e->trackActive.push_back(1);
  e->trkSR.emplace_back();
  std::memcpy(e->trkSR.back().offs, p->layer_offsets, 9 * sizeof(uint32_t));
  e->pendTracks.push_back(to_dev_track(*p, ddIdx));  // uploaded by flush_topology
  e->schedDirty = true;
  return h;
}

int lkf_set_layer_offsets_at(lkf_engine *e, int32_t track, const uint32_t offsets[9], uint32_t at_pkt) {
  if (!e || !offsets || track < 0 || track >= int32_t(e->tracks.size())) return LKF_EINVAL;
  lkf_engine::TrackOp op;
  op.track = uint32_t(track);
  op.at = at_pkt;
  std::memcpy(op.offs, offsets, sizeof(op.offs));
  std::memcpy(e->trkSR[size_t(track)].offs, offsets, sizeof(op.offs));
  e->trkOps.push_back(op);
  return LKF_OK;
}

int lkf_set_layer_offsets(lkf_engine *e, int32_t track, const uint32_t offsets[9]) {
  return lkf_set_layer_offsets_at(e, track, offsets, 0);
}

// mediatransportutil v0.0.0-20231213075826-cccbf2b93d3f NtpTime.Duration (the
// offset of NtpTime.Time from the NTP epoch): seconds, and the 32-bit fraction
// in nanoseconds rounded half up
static int64_t ntp_ns(uint64_t t) {
  const uint64_t sec = (t >> 32) * 1000000000ull;
  const uint64_t frac = (t & 0xffffffffull) * 1000000000ull;
  uint64_t nsec = frac >> 32;
  if (uint32_t(frac) >= 0x80000000u) nsec++;
  return int64_t(sec + nsec);
}

// StreamTrackerManager.updateLayerOffsetLocked (streamtrackermanager.go:561-601)
static bool sr_layer_offset(lkf_engine::TrackSR &s, uint32_t clockRate, int ref, int other) {
  if (!s.have[ref] || s.ntp[ref] == 0 || !s.have[other] || s.ntp[other] == 0) return false;
  const int64_t d = ntp_ns(s.ntp[ref]) - ntp_ns(s.ntp[other]);  // srRef.Time().Sub(srOther.Time())
  const double secs = double(d / 1000000000) + double(d % 1000000000) / 1e9;  // Duration.Seconds
  if (std::fabs(secs) > 60.0) return false;  // senderReportThresholdSeconds :36
  const int64_t rtpDiff = d * int64_t(clockRate) / 1000000000;
  const uint32_t norm = s.rtp[other] + uint32_t(rtpDiff);
  uint32_t off = s.rtp[ref] - norm;
  if (off == 0) off = 1;
  const bool changed = s.offs[ref * 3 + other] != off;
  s.offs[ref * 3 + other] = off;
  return changed;
}

// SetRTCPSenderReportData (streamtrackermanager.go:603-627)
int lkf_sender_report(lkf_engine *e, int32_t track, int32_t layer, uint64_t ntp_timestamp, uint32_t rtp_timestamp,
                      uint32_t at_pkt) {
  if (!e || track < 0 || track >= int32_t(e->tracks.size())) return LKF_EINVAL;
  if (layer < 0 || layer > 2) return LKF_OK;  // (invalid layer: ignored, as the reference)
  lkf_engine::TrackSR &s = e->trkSR[size_t(track)];
  s.ntp[layer] = ntp_timestamp;
  s.rtp[layer] = rtp_timestamp;
  s.have[layer] = 1;
  bool changed = false;
  for (int i = 0; i < 3; i++) {
    if (i == layer) continue;
    changed |= sr_layer_offset(s, e->tracks[size_t(track)].clock_rate, layer, i);
    changed |= sr_layer_offset(s, e->tracks[size_t(track)].clock_rate, i, layer);
  }
  if (!changed) return LKF_OK;
  lkf_engine::TrackOp op;
  op.track = uint32_t(track);
  op.at = at_pkt;
  std::memcpy(op.offs, s.offs, sizeof(op.offs));
  e->trkOps.push_back(op);
  return LKF_OK;
}

int32_t lkf_add_downtrack(lkf_engine *e, const lkf_downtrack_params *p) {
  if (!e || !p) return LKF_EINVAL;
  if (p->track < 0 || p->track >= int32_t(e->tracks.size())) return LKF_EINVAL;
  if (e->dtp.size() >= e->cfg.max_downtracks) return LKF_ENOSPC;
  int32_t h = int32_t(e->dtp.size());
  e->dtp.push_back(*p);
  e->active.push_back(1);
  e->seqRM.push_back(0);
  {  // DD selector and VP9 SVC DownTracks: k_decide_dt<true> (svc_run)
    const lkf_track_params &tp = e->tracks[p->track];
    const bool vp9 = tp.kind == LKF_KIND_VIDEO && tp.codec == LKF_CODEC_VP9;
    e->dtIsDD.push_back((track_has_dd(tp) || vp9) ? 1 : 0);
  }
  e->pendHot.emplace_back();
  init_hot(e->pendHot.back(), e->tracks[p->track], *p);
  DevDT d;
  std::memset(&d, 0, sizeof(d));
  d.track = uint32_t(p->track);
  d.ssrc = p->ssrc;
  d.pt = p->payload_type;
  d.extPlayout = p->ext_playout;
  d.extAbs = p->ext_abs_send_time;
  d.extDD = p->ext_dd;
  d.extTcc = p->ext_transport_cc;
  d.twccGroup = uint32_t(h);  // its own counter until bound to a transport
  std::memcpy(d.playout, p->playout_delay, 3);
  d.active = 1;
  e->dtTransport.push_back(-1);
  if (p->ext_transport_cc) e->anyTwcc = e->twccDirty = true;
  e->pendDTs.push_back(d);  // uploaded by flush_topology (one copy per batch of adds)
  e->schedDirty = true;
  return h;
}

int lkf_remove_downtrack(lkf_engine *e, int32_t dt) {
  if (!e || dt < 0 || dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  e->active[dt] = 0;
  e->topoGen++;
  uint8_t zero = 0;
  HIPCHK(hipMemcpy(reinterpret_cast<uint8_t *>(e->dDTs + dt) + offsetof(DevDT, active), &zero, 1,
                   hipMemcpyHostToDevice),
         "remove copy");
  e->schedDirty = true;
  return upload_done(e);
}

int lkf_remove_track(lkf_engine *e, int32_t track) {
  if (!e || track < 0 || track >= int32_t(e->tracks.size())) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  if (!e->trackActive[track]) return LKF_OK;
  e->trackActive[track] = 0;
  const uint8_t zero = 0, one = 1;
  for (size_t d = 0; d < e->dtp.size(); d++)  // closeTracks: every DownTrack of the receiver
    if (e->dtp[d].track == track && e->active[d]) {
      e->active[d] = 0;
      e->topoGen++;
      HIPCHK(hipMemcpy(reinterpret_cast<uint8_t *>(e->dDTs + d) + offsetof(DevDT, active), &zero, 1,
                       hipMemcpyHostToDevice),
             "remove copy");
    }
  for (size_t sid = 0; sid < e->streams.size(); sid++)  // Buffer.Close of its streams
    if (e->streams[sid].track == track)
      HIPCHK(hipMemcpy(reinterpret_cast<uint8_t *>(e->dStreams + sid) + offsetof(DevStream, closed), &one, 1,
                       hipMemcpyHostToDevice),
             "close copy");
  e->schedDirty = true;
  e->spkDirty = true;
  return upload_done(e);
}

int lkf_ctl(lkf_engine *e, int32_t dt, int32_t op, int64_t a0, int64_t a1, int64_t a2, int64_t a3, uint32_t at_pkt) {
  if (!e || dt < 0 || dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
  if (op < LKF_CTL_MUTE || op > LKF_CTL_PLAYOUT_ACKED) return LKF_EINVAL;
  lkf_engine::Pend p;
  p.dt = uint32_t(dt);
  std::memset(&p.ev, 0, sizeof(p.ev));
  p.ev.at = at_pkt;
  p.ev.op = op;
  p.ev.a[0] = a0;
  p.ev.a[1] = a1;
  p.ev.a[2] = a2;
  p.ev.a[3] = a3;
  e->pending.push_back(p);
  return LKF_OK;
}

int lkf_ctl_batch(lkf_engine *e, const lkf_ctl_event *evs, uint32_t n) {
  if (!e || (n && !evs)) return LKF_EINVAL;
  const int32_t nd = int32_t(e->dtp.size());
  for (uint32_t i = 0; i < n; i++)
    if (evs[i].dt < 0 || evs[i].dt >= nd || evs[i].op < LKF_CTL_MUTE || evs[i].op > LKF_CTL_PLAYOUT_ACKED)
      return LKF_EINVAL;
  e->pending.reserve(e->pending.size() + n);
  for (uint32_t i = 0; i < n; i++) {
    lkf_engine::Pend p;
    p.dt = uint32_t(evs[i].dt);
    std::memset(&p.ev, 0, sizeof(p.ev));
    p.ev.at = evs[i].at_pkt;
    p.ev.op = evs[i].op;
    for (int j = 0; j < 4; j++) p.ev.a[j] = evs[i].a[j];
    e->pending.push_back(p);
  }
  return LKF_OK;
}

int lkf_submit(lkf_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len) {
  if (!e || (n && !pkts)) return LKF_EINVAL;
  if (n > e->cfg.max_batch_pkts || arena_len > e->cfg.max_batch_arena) return LKF_ENOSPC;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  BatchCtx &x = e->ctx[e->nRuns % lkf_engine::kCtx];
  if (x.used) HIPCHK(hipEventSynchronize(x.emitted), "wait emit");  // batch n-2 still reads these buffers
  if (n) HIPCHK(hipMemcpyAsync(x.dPktsOwn, pkts, size_t(n) * sizeof(lkf_pkt), hipMemcpyHostToDevice, e->own), "pkts");
  if (arena_len) HIPCHK(hipMemcpyAsync(x.dArenaOwn, arena, arena_len, hipMemcpyHostToDevice, e->own), "arena");
  HIPCHK(hipStreamSynchronize(e->own), "submit sync");
  x.prepByIngest = false;
  e->curPkts = x.dPktsOwn;
  e->curArena = x.dArenaOwn;
  e->curN = n;
  e->curNDev = nullptr;
  e->curDD = nullptr;
  e->curOwned = true;
  e->curDDOwned = true;
  e->ingestStarted = false;
  e->curArenaLen = arena_len;
  e->haveBatch = true;
  return LKF_OK;
}

int lkf_submit_device(lkf_engine *e, const lkf_pkt *d_pkts, uint32_t n, const uint8_t *d_arena, uint64_t arena_len) {
  if (!e || (n && !d_pkts)) return LKF_EINVAL;
  if (n > e->cfg.max_batch_pkts) return LKF_ENOSPC;
  e->ctx[e->nRuns % lkf_engine::kCtx].prepByIngest = false;
  e->curPkts = d_pkts;
  e->curArena = d_arena;
  e->curN = n;
  e->curNDev = nullptr;
  e->curDD = nullptr;
  e->curOwned = false;
  e->curDDOwned = true;
  e->ingestStarted = false;
  e->curArenaLen = arena_len;
  e->haveBatch = true;
  return LKF_OK;
}

int lkf_submit_dd(lkf_engine *e, const lkf_pkt_dd *dd, uint32_t n) {
  if (!e || (n && !dd)) return LKF_EINVAL;
  if (!e->haveBatch || n != e->curN) return LKF_EINVAL;  // parallel to the batch just submitted
  int rc = flush_topology(e);
  if (rc) return rc;
  if (!e->ddAlloc) return LKF_OK;  // no DD track: nothing reads it
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  BatchCtx &x = e->ctx[e->nRuns % lkf_engine::kCtx];
  if (x.used) HIPCHK(hipEventSynchronize(x.emitted), "wait emit");  // batch n-3 may still read it
  if (n) HIPCHK(hipMemcpyAsync(x.dDDIn, dd, size_t(n) * sizeof(lkf_pkt_dd), hipMemcpyHostToDevice, e->own), "dd");
  HIPCHK(hipStreamSynchronize(e->own), "submit dd sync");
  e->curDD = x.dDDIn;
  e->curDDOwned = true;
  return LKF_OK;
}

int lkf_submit_dd_device(lkf_engine *e, const lkf_pkt_dd *d_dd, uint32_t n) {
  if (!e || (n && !d_dd)) return LKF_EINVAL;
  if (!e->haveBatch || n != e->curN) return LKF_EINVAL;
  e->curDD = d_dd;
  e->curDDOwned = false;
  return LKF_OK;
}

// Lane schedule: one wave per (track, up to 64 of its DownTracks), idle lanes
// padded with kIdle.  Video tracks first (longest packet lists).
static int rebuild_sched(lkf_engine *e) {
  const uint32_t nd = uint32_t(e->dtp.size());
  const uint32_t nt = uint32_t(e->tracks.size());
  std::vector<std::vector<uint32_t>> byTrack(nt);
  for (uint32_t d = 0; d < nd; d++)
    if (e->active[d]) byTrack[e->dtp[d].track].push_back(d);
  std::vector<uint32_t> order(nt);
  for (uint32_t t = 0; t < nt; t++) order[t] = t;
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t b) { return e->tracks[a].kind > e->tracks[b].kind; });
  // Two parts: DownTracks of the plain selectors (k_decide_dt<false>), then
  // the SVC ones (dependency-descriptor or VP9 selector) and those whose
  // sequencer holds padding exclusions (k_decide_dt<true>), each interleaved
  // per XCD.
  std::vector<uint32_t> sched, waveTrack;
  e->ddLanes = 0;
  for (int part = 0; part < 2; part++) {
    std::vector<uint32_t> ps, pt;
    for (uint32_t t : order) {
      for (uint32_t d : byTrack[t]) {  // one wave per DownTrack (interleaved per XCD below)
        if ((e->dtIsDD[d] || e->seqRM[d]) != (part == 1)) continue;
        ps.push_back(d);
        pt.push_back(t);
      }
    }
    if (ps.empty()) continue;
    // Waves are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8).
    // Give all DownTracks of a track the same XCD, consecutive in its order,
    // so the 8-9 waves reading one track's packet descriptors share an L2.
    // Tracks go to the XCD with the fewest waves so far (video first, so the
    // long waves spread evenly); idle slots pad the shorter XCD lists.
    constexpr int kX = 8;
    std::vector<std::vector<uint32_t>> lst(kX), lstT(kX);
    std::vector<double> load(kX, 0.0);
    size_t i = 0;
    while (i < ps.size()) {
      const uint32_t t = pt[i];
      size_t j = i;
      while (j < ps.size() && pt[j] == t) j++;
      int bx = 0;
      for (int x = 1; x < kX; x++)
        if (load[x] < load[bx]) bx = x;
      const double w = e->tracks[t].kind == LKF_KIND_VIDEO ? 7.0 : 1.0;  // ~packets per wave
      for (size_t q = i; q < j; q++) {
        lst[bx].push_back(ps[q]);
        lstT[bx].push_back(t);
        load[bx] += w;
      }
      i = j;
    }
    size_t mx = 0;
    for (auto &l : lst) mx = std::max(mx, l.size());
    const size_t base = sched.size();
    sched.resize(base + mx * kX, kIdle);
    waveTrack.resize(base + mx * kX, 0);
    for (int x = 0; x < kX; x++)
      for (size_t q = 0; q < lst[x].size(); q++) {
        sched[base + q * kX + x] = lst[x][q];
        waveTrack[base + q * kX + x] = lstT[x][q];
      }
    if (part == 1) e->ddLanes = uint32_t(mx * kX);
  }
  e->sched.swap(sched);
  e->waveTrack.swap(waveTrack);
  e->dtLane.assign(nd, -1);
  for (uint32_t l = 0; l < e->sched.size(); l++)
    if (e->sched[l] != kIdle) e->dtLane[e->sched[l]] = int32_t(l);
  const size_t nl = e->sched.size();
  int rc = drain_streams(e);  // queued runs still read the previous schedule
  if (rc) return rc;
  if (nl + 1 > e->schedCap) {
    if (e->dSched) HIPCHK(dfree(e->dSched), "free sched");
    if (e->dWaveTrack) HIPCHK(dfree(e->dWaveTrack), "free wavetrack");
    e->schedCap = nl + 1 + 4096;
    HIPCHK(dalloc(&e->dSched, e->schedCap), "alloc sched");
    HIPCHK(dalloc(&e->dWaveTrack, e->schedCap + 1), "alloc wavetrack");
  }
  // output order: by track, then DownTrack handle (every DownTrack, active or not)
  {
    std::vector<uint32_t> perm(nd);
    for (uint32_t d = 0; d < nd; d++) perm[d] = d;
    std::stable_sort(perm.begin(), perm.end(),
                     [&](uint32_t a, uint32_t b) { return e->dtp[a].track < e->dtp[b].track; });
    if (nd) HIPCHK(hipMemcpy(e->dPerm, perm.data(), nd * sizeof(uint32_t), hipMemcpyHostToDevice), "perm copy");
  }
  if (nl) {
    HIPCHK(hipMemcpy(e->dSched, e->sched.data(), nl * sizeof(uint32_t), hipMemcpyHostToDevice), "sched copy");
    HIPCHK(hipMemcpy(e->dWaveTrack, e->waveTrack.data(), e->waveTrack.size() * sizeof(uint32_t),
                     hipMemcpyHostToDevice),
           "wavetrack copy");
  }
  e->schedDirty = false;
  e->epoch++;
  return upload_done(e);
}

// Per transport, its transport-cc DownTracks in record order (track, then
// DownTrack handle) for k_twcc_base; the counters of transports added since
// the last rebuild start at 0 (pion's interceptor starts at 0 per
// PeerConnection).  Queued runs read the lists: drained first.
static int rebuild_twcc(lkf_engine *e) {
  int rc = drain_streams(e);
  if (rc) return rc;
  const uint32_t nt = uint32_t(e->transports.size());
  std::vector<std::vector<uint32_t>> lst(nt);
  std::vector<uint32_t> order(e->dtp.size());
  for (uint32_t d = 0; d < order.size(); d++) order[d] = d;
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t b) { return e->dtp[a].track < e->dtp[b].track; });
  for (uint32_t d : order)
    if (e->dtp[d].ext_transport_cc && e->dtTransport[d] >= 0) lst[size_t(e->dtTransport[d])].push_back(d);
  std::vector<uint32_t> off(nt + 1, 0), flat;
  for (uint32_t t = 0; t < nt; t++) {
    off[t] = uint32_t(flat.size());
    flat.insert(flat.end(), lst[t].begin(), lst[t].end());
  }
  off[nt] = uint32_t(flat.size());
  if (nt > e->twccTCap || !e->dTwccCtrT) {  // grow the transport counters (first: before any transport), keeping the old ones
    const uint32_t cap = std::max<uint32_t>(nt, 2 * e->twccTCap + 64);
    uint32_t *c = nullptr, *o = nullptr;
    HIPCHK(dalloc(&c, cap), "alloc twcc counters");
    HIPCHK(hipMemset(c, 0, size_t(cap) * sizeof(uint32_t)), "twcc counters reset");
    if (e->dTwccCtrT) {
      HIPCHK(hipMemcpy(c, e->dTwccCtrT, size_t(e->twccTCap) * sizeof(uint32_t), hipMemcpyDeviceToDevice),
             "twcc counters move");
      HIPCHK(dfree(e->dTwccCtrT), "free twcc counters");
    }
    if (e->dTwccTOff) HIPCHK(dfree(e->dTwccTOff), "free twcc offsets");
    HIPCHK(dalloc(&o, cap + 1), "alloc twcc offsets");
    e->dTwccCtrT = c;
    e->dTwccTOff = o;
    e->twccTCap = cap;
  }
  if (flat.size() > e->twccListCap || !e->dTwccTList) {
    if (e->dTwccTList) HIPCHK(dfree(e->dTwccTList), "free twcc lists");
    e->twccListCap = uint32_t(std::max<size_t>(flat.size(), 1024));
    HIPCHK(dalloc(&e->dTwccTList, e->twccListCap), "alloc twcc lists");
  }
  HIPCHK(hipMemcpy(e->dTwccTOff, off.data(), off.size() * sizeof(uint32_t), hipMemcpyHostToDevice), "twcc offsets");
  if (!flat.empty())
    HIPCHK(hipMemcpy(e->dTwccTList, flat.data(), flat.size() * sizeof(uint32_t), hipMemcpyHostToDevice), "twcc lists");
  e->nTwccT = nt;
  e->twccDirty = false;
  return upload_done(e);
}

int lkf_run(lkf_engine *e, void *stream) {
  if (!e) return LKF_EINVAL;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  {
    int rc = flush_topology(e);
    if (rc) return rc;
  }
  if (e->schedDirty) {
    int rc = rebuild_sched(e);
    if (rc) return rc;
  }
  if (e->twccDirty) {
    int rc = rebuild_twcc(e);
    if (rc) return rc;
  }
  const int ci = int(e->nRuns % lkf_engine::kCtx);
  BatchCtx &x = e->ctx[ci];
  if (!e->haveBatch) {  // control-only run: an empty batch applies queued ops
    e->curPkts = x.dPktsOwn;
    e->curArena = x.dArenaOwn;
    e->curOwned = e->curDDOwned = true;
    e->curN = 0;
    e->curNDev = nullptr;
    e->curArenaLen = 0;
  }
  // The caller's stream orders the batch's inputs; the stages themselves run
  // on the engine's decide/emit streams (completion: lkf_sync).
  using clk = std::chrono::steady_clock;
  const auto tp0 = clk::now();
  auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  hipStream_t us = stream ? reinterpret_cast<hipStream_t>(stream) : e->own;
  e->cur = us;
  // prep stream: control-op CSR, per-batch init, track ranges, slot scan,
  // layer index (and, before lkf_run, the ingest).  It runs ahead: batch n+1
  // is prepared while batch n decides, so decide(n+1) starts as soon as
  // decide(n) ends.
  hipStream_t ps = e->prepS;
  hipStream_t s = e->decS;
  HIPCHK(hipEventRecord(e->inEv, us), "event");
  HIPCHK(hipStreamWaitEvent(ps, e->inEv, 0), "wait caller stream");
  const uint32_t nt = uint32_t(e->tracks.size());
  const uint32_t nd = uint32_t(e->dtp.size());
  const uint32_t nl = uint32_t(e->sched.size());
  // this context's previous batch (run n-2) must have finished its emit stage
  if (x.used) HIPCHK(hipStreamWaitEvent(ps, x.emitted, 0), "wait emit");
  if (x.fromIngest && e->haveBatch) HIPCHK(hipStreamWaitEvent(ps, x.ingested, 0), "wait ingest");
  const bool prepDone = x.fromIngest && e->haveBatch && x.prepByIngest && x.prepNT == nt && x.prepND == nd &&
                        e->curPkts == x.dPktsOwn;
  const bool ingestFed = x.fromIngest && e->haveBatch;  // (emit's residency, below)
  x.fromIngest = false;
  x.prepByIngest = false;

  // Per-lane control-op CSR (stable: queue order within a lane, then by
  // at_pkt).  The host sorts only the ops: an LSD radix sort on the lane
  // (8-bit digits, stable), then a stable insertion by at_pkt inside a lane
  // with several ops; it stages the run's RunDesc, the sorted ops and their
  // lanes in this context's page-locked cached buffer.  The prep stage's
  // first kernel pulls them and k_ev_offsets derives the dense per-lane
  // offsets on the GPU (no host pass over all lanes).
  const auto tp1 = clk::now();
  if (x.used) HIPCHK(hipEventSynchronize(x.pulled), "stage wait");  // run n-3's pull of this staging is done
  const auto tp2 = clk::now();
  if (!e->trkOps.empty()) {  // a track's layer-offset changes: one op per active DownTrack of it
    std::stable_sort(e->trkOps.begin(), e->trkOps.end(), [](const lkf_engine::TrackOp &a, const lkf_engine::TrackOp &b) {
      return a.track != b.track ? a.track < b.track : a.at < b.at;
    });
    std::vector<std::vector<uint32_t>> byT(nt);
    for (uint32_t d = 0; d < nd; d++)
      if (e->active[d]) byT[e->dtp[d].track].push_back(d);
    for (const auto &op : e->trkOps) {
      lkf_engine::Pend q;
      std::memset(&q.ev, 0, sizeof(q.ev));
      q.ev.at = op.at;
      q.ev.op = kOpLayerOffsets;
      for (int k = 0; k < 4; k++) q.ev.a[k] = int64_t(uint64_t(op.offs[2 * k]) | (uint64_t(op.offs[2 * k + 1]) << 32));
      q.ev.pad = int64_t(op.offs[8]);
      for (uint32_t d : byT[op.track]) {
        q.dt = d;
        e->pending.push_back(q);
      }
      std::memcpy(e->tracks[op.track].layer_offsets, op.offs, sizeof(op.offs));  // as of the end of this run
    }
    e->trkOps.clear();
  }
  auto &ka = e->sortA, &kb = e->sortB;  // (lane, pending index)
  ka.clear();
  for (uint32_t i = 0; i < uint32_t(e->pending.size()); i++) {
    const int l = e->dtLane[e->pending[i].dt];
    if (l >= 0) ka.push_back({uint32_t(l), i});  // ops for removed DownTracks are dropped
  }
  const size_t nev = ka.size();
  kb.resize(nev);
  for (uint32_t shift = 0; shift < 32 && (nl >> shift) > 0; shift += 8) {  // stable LSD passes
    uint32_t cnt[257] = {0};
    for (auto &k : ka) cnt[((k.first >> shift) & 0xff) + 1]++;
    for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
    for (auto &k : ka) kb[cnt[(k.first >> shift) & 0xff]++] = k;
    ka.swap(kb);
  }
  if (nev > x.stageCap || !x.stage) {  // (graphs captured with the old staging are re-captured)
    // the queued pull of this context's previous run may still read the old
    // staging, and its graphs are destroyed when re-captured: drain first
    if (x.stage) {
      if (int rc = drain_streams(e)) return rc;
    }
    stage_free(&x.stage, &x.stageDev);
    x.stageCap = uint32_t(std::max<size_t>(2 * nev, 4096));
    HIPCHK(stage_alloc(&x.stage, &x.stageDev, sizeof(RunDesc) + size_t(x.stageCap) * (sizeof(DevEvent) + 4)),
           "alloc stage");
    x.gPrepEpoch[0] = x.gPrepEpoch[1] = 0;
    x.gCtlEpoch = 0;
  }
  DevEvent *evs = reinterpret_cast<DevEvent *>(x.stage + sizeof(RunDesc));
  uint32_t *lanes = reinterpret_cast<uint32_t *>(x.stage + sizeof(RunDesc) + size_t(x.stageCap) * sizeof(DevEvent));
  for (size_t i = 0; i < nev; i++) {
    evs[i] = e->pending[ka[i].second].ev;
    lanes[i] = ka[i].first;
    if (i && ka[i - 1].first == ka[i].first && evs[i].at < evs[i - 1].at) {
      const DevEvent v = evs[i];  // queued out of at_pkt order: stable insertion within the lane
      size_t j = i;
      while (j > 0 && lanes[j - 1] == ka[i].first && evs[j - 1].at > v.at) {
        evs[j] = evs[j - 1];
        j--;
      }
      evs[j] = v;
    }
  }
  e->pending.clear();
  {
    RunDesc &h = *reinterpret_cast<RunDesc *>(x.stage);
    std::memset(&h, 0, sizeof(h));
    h.pkts = reinterpret_cast<uint64_t>(e->curPkts);
    h.arena = reinterpret_cast<uint64_t>(e->curArena);
    h.dd = reinterpret_cast<uint64_t>(e->curDD);
    h.nDev = reinterpret_cast<uint64_t>(e->curNDev);
    h.n = e->curN;
    h.nev = uint32_t(nev);
    h.evCap = x.stageCap;
  }
  const auto tp25 = clk::now();
  if (nev > x.evCap || size_t(nl) + 1 > x.evOffCap || nev > x.evLaneCap) {
    // this context's op buffers: its previous run (n-3) must be done with them.
    // ps waits on that run's "emitted" event above, so draining ps covers its
    // prep, decide and emit stages (the lane list is read by k_ev_offsets on ps,
    // the ops and offsets by the decide stage).
    // (every stream: the pull graph on the engine's own stream reads them too,
    // and the graphs captured with them are destroyed below)
    if (int rc = drain_streams(e)) return rc;
    if (nev > x.evCap) {
      if (x.dEvents) HIPCHK(dfree(x.dEvents), "free events");
      x.evCap = std::max<uint64_t>(2 * nev, 4096);
      HIPCHK(dalloc(&x.dEvents, x.evCap), "alloc events");
    }
    if (size_t(nl) + 1 > x.evOffCap) {
      if (x.dEvOff) HIPCHK(dfree(x.dEvOff), "free evoff");
      x.evOffCap = size_t(nl) + 1 + 4096;
      HIPCHK(dalloc(&x.dEvOff, x.evOffCap), "alloc evoff");
    }
    if (nev > x.evLaneCap) {
      if (x.dEvLane) HIPCHK(dfree(x.dEvLane), "free evlane");
      x.evLaneCap = std::max<uint64_t>(2 * nev, 4096);
      HIPCHK(dalloc(&x.dEvLane, x.evLaneCap), "alloc evlane");
    }
    x.gPrepEpoch[0] = x.gPrepEpoch[1] = 0;
    x.gCtlEpoch = 0;
  }
  const auto tp3 = clk::now();

  // ---- prep stage (prep stream): the pull, per-batch init, track ranges,
  // slot scan, layer index, tracker observe, DD decode
  hipEvent_t *rg = e->ring[e->nRuns % lkf_engine::kRing];
  if (!e->ingestStarted) HIPCHK(hipEventRecord(rg[0], ps), "event");  // else: recorded ahead of the ingest
  e->ingestStarted = false;
  // the control-op pull (k_h2d: the run descriptor and the ops from the
  // pinned staging; k_ev_offsets) on the engine's own stream: it does not
  // depend on the batch, so it runs beside a preceding ingest instead of after
  // it on the prep stream
  hipStream_t cs = e->own;
  if (x.used) HIPCHK(hipStreamWaitEvent(cs, x.emitted, 0), "wait emit (pull)");
  auto ctl = [&]() -> int {
    HIPCHK(launch_h2d(cs, x.stageDev, x.dDesc, x.dEvents, x.dEvLane), "event pull");
    HIPCHK(launch_ev_offsets(cs, x.dEvLane, x.dDesc, nl, x.dEvOff), "event offsets");
    return LKF_OK;
  };
  auto prep = [&]() -> int {
    if (!prepDone) {  // (an ingest's k_ing_out did both)
      HIPCHK(launch_batch_init(ps, nt, nd, kStatsWords * (1 + kStatCopies), x.dTBegin, x.dTEnd, x.dTRuns, x.dErr,
                               x.dStats, x.dFwdCnt, x.dFwdBytes),
             "batch init");
      HIPCHK(launch_track_ranges(ps, x.dDesc, e->cfg.max_batch_pkts, nt, x.dTBegin, x.dTEnd, x.dTRuns, x.dErr),
             "track_ranges");
    }
    HIPCHK(launch_scan(ps, 0, e->dDTs, x.dTBegin, x.dTEnd, nullptr, nullptr, nd, x.dPartA, x.dPartB, x.dSlotBase,
                       nullptr, x.dTot + 0, nullptr, nullptr),
           "slot scan");
    HIPCHK(launch_layer_index(ps, x.dDesc, x.dTBegin, x.dTEnd, nt, e->cfg.max_batch_pkts, x.dLayerList,
                              x.dLayerBefore, x.dLayerCnt, e->ddAlloc ? x.dDDUsed : nullptr),
           "layer index");
    if (e->nTrk)  // StreamTracker.Observe of every (track, spatial layer) tracker (receiver.go:686-695)
      HIPCHK(launch_tracker_observe(ps, e->dTrk, e->nTrk, x.dDesc, x.dTBegin, x.dTEnd), "tracker observe");
    if (e->ddAlloc) {  // dependency descriptors of this batch (track structure rings advance in order)
      HIPCHK(launch_dd_decode(ps, x.dDesc, x.dTBegin, x.dTEnd, e->dTracks, nt, e->dDDStruct, e->dDDTrack, x.dDDPkt,
                              x.dErr, e->nDDTrk ? e->dTrackDDTrk : nullptr, e->dDDTrk, x.dDDSpill,
                              reinterpret_cast<uint32_t *>(x.dDDUsed + 1), e->ddSpillCap),
             "dd decode");
    }
    return LKF_OK;
  };
  auto scanTail = [&](hipStream_t st) -> int {
    // counters and the output scan stay on the (high-priority) decide stream:
    // on the low-priority emit stream these small kernels queued behind the
    // next batch's decide waves and were on the emit chain's critical path
    HIPCHK(launch_stats_reduce(st, x.dStats), "stats reduce");
    HIPCHK(launch_scan(st, 1, e->dDTs, nullptr, nullptr, x.dFwdCnt, x.dFwdBytes, nd, x.dPartA, x.dPartB, x.dRecBase,
                       x.dByteBase, x.dTot + 2, x.dTot + 3, e->dPerm, x.dGFirst, e->cfg.max_out_pkts),
           "out scan");
    return LKF_OK;
  };
  // (re)captures a stage as a graph on stream st: the captured launches are the
  // same as the direct ones
  auto capture = [&](hipStream_t st, hipGraphExec_t &g, auto body) -> int {
    // an exec is destroyed only once its last launch (on st, this context's
    // previous run) has finished: HIP may release its kernel arguments at once
    if (g) {
      HIPCHK(hipStreamSynchronize(st), "graph idle");
      HIPCHK(hipGraphExecDestroy(g), "graph destroy");
    }
    g = nullptr;
    HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed), "begin capture");
    const int rc = body();
    hipGraph_t graph = nullptr;
    const hipError_t r = hipStreamEndCapture(st, &graph);
    if (rc) return rc;
    HIPCHK(r, "end capture");
    const hipError_t ri = hipGraphInstantiate(&g, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    HIPCHK(ri, "graph instantiate");
    return LKF_OK;
  };
  if (e->useGraph) {
    if (x.gCtlEpoch != e->epoch || !x.gCtl) {
      const int rc = capture(cs, x.gCtl, ctl);
      if (rc) return rc;
      x.gCtlEpoch = e->epoch;
    }
    HIPCHK(hipGraphLaunch(x.gCtl, cs), "pull graph");
  } else {
    const int rc = ctl();
    if (rc) return rc;
  }
  HIPCHK(hipEventRecord(x.pulled, cs), "event");
  HIPCHK(hipStreamWaitEvent(ps, x.pulled, 0), "wait pull");
  if (e->useGraph) {
    const int fi = prepDone ? 1 : 0;
    if (x.gPrepEpoch[fi] != e->epoch || !x.gPrep[fi]) {
      const int rc = capture(ps, x.gPrep[fi], prep);
      if (rc) return rc;
      x.gPrepEpoch[fi] = e->epoch;
    }
    HIPCHK(hipGraphLaunch(x.gPrep[fi], ps), "prep graph");
  } else {
    const int rc = prep();
    if (rc) return rc;
  }
  HIPCHK(hipEventRecord(x.prepped, ps), "event");
  if (e->debugDD && e->ddAlloc) {  // LKF_DEBUG_DD=1 (diagnostic): the context's DD cursor after its prep
    HIPCHK(hipStreamSynchronize(ps), "debug sync");
    uint64_t u[2] = {0, 0};
    HIPCHK(hipMemcpy(u, x.dDDUsed, sizeof(u), hipMemcpyDeviceToHost), "debug copy");
    fprintf(stderr, "[lkf dd] run %llu ctx %d after prep: cursor %llu spill %llu graph %d epoch %llu/%llu\n",
            (unsigned long long)e->nRuns, ci, (unsigned long long)u[0], (unsigned long long)u[1], int(e->useGraph),
            (unsigned long long)x.gPrepEpoch[prepDone ? 1 : 0], (unsigned long long)e->epoch);
  }
  HIPCHK(hipStreamWaitEvent(s, x.prepped, 0), "wait prep");
  DecideLaunch d;
  d.layerList = x.dLayerList;
  d.layerBefore = x.dLayerBefore;
  d.layerCnt = x.dLayerCnt;
  d.pktStride = e->cfg.max_batch_pkts;
  d.sched = e->dSched;
  d.waveTrack = e->dWaveTrack;
  d.nlanes = nl;
  d.hot = e->dHot;
  d.dts = e->dDTs;
  d.tracks = e->dTracks;
  d.rm = e->dRm;
  d.vc = e->dVc;
  d.seq = e->dSeq;
  d.seqSize = e->cfg.seq_size;
  d.srm = e->dSrm;
  d.srmStride = e->srmStride;
  d.srmCap = e->srmCap;
  d.pkts = e->curPkts;
  d.tBegin = x.dTBegin;
  d.tEnd = x.dTEnd;
  d.slotBase = x.dSlotBase;
  d.recs = x.dRecs;
  d.fbase = x.dFBase;
  d.wide = x.dWide;
  d.ss = e->dSS;
  d.ssRing = e->dSSRing;
  d.ssGap = e->dSSGap;
  d.dtOffs = e->dDTOffs;
  d.tupleCap = e->cfg.max_batch_tuples;
  d.err = x.dErr;
  d.events = x.dEvents;
  d.evOff = x.dEvOff;
  d.fwdCnt = x.dFwdCnt;
  d.fwdBytes = x.dFwdBytes;
  d.dtCum = e->dDTCum;
  d.stats = x.dStats;
  d.ddLanes = e->ddLanes;
  // Several DownTracks per decide wave when the batch is short (a 10-20 ms
  // tick has a few packets per track): the per-DownTrack prologue then
  // dominates and one workgroup per DownTrack is dispatch-rate bound.
  if (e->decideK) {
    d.perWave = e->decideK;
  } else {
    // (round 6: 2 below 48 packets per track — 4 at the shortest ticks measured
    // slower since the stream wave and the NACK queues changed: 10-ms ticks at
    // 1,000 rooms 0.555 -> 0.533 ms ingress, 0.338 -> 0.331 ms ExtPacket, at 100
    // rooms 0.130 -> 0.106 ms; 1: 0.557 / 0.346 ms; profiles/r6_ab_runs.txt)
    // Many DownTracks: one wave each is bound by the dispatch rate (≈240 waves
    // per µs over the 8 XCDs: configs[2]'s 337 k DownTracks ≈ 1.4 ms), so a
    // wave serves one more DownTrack per 100 k (configs[2] 2.74 -> 2.54 ms at
    // 4; configs[1]'s 18 k stay at one: 2 costs 0.74 -> 0.87 ms there;
    // configs[3]'s 100 k measured alike at 1 and 2)
    const uint64_t per = uint64_t(e->curN) / std::max<uint32_t>(1, nt);  // (ingest: the datagram count bound)
    const uint32_t byCount = uint32_t(std::min<uint64_t>(8, (uint64_t(nd) + 99999) / 100000));
    d.perWave = std::max<uint32_t>(per >= 48 ? 1 : 2, byCount);
  }
  d.ddPkts = e->ddAlloc ? x.dDDPkt : nullptr;
  d.ddStructs = e->dDDStruct;
  d.ddState = e->ddAlloc ? e->dDDState : nullptr;
  d.ddArena = x.dDDArena;
  d.ddUsed = x.dDDUsed;
  d.ddSpill = e->ddAlloc ? x.dDDSpill : nullptr;
  d.ddCap = e->ddArenaCap;
  d.maxDts = e->cfg.max_downtracks;
  d.maxTracks = e->cfg.max_tracks;
  d.npkts = e->curN;  // (an ingest-produced batch: the launch bound)
  d.nev = uint32_t(nev);
  HIPCHK(hipEventRecord(rg[1], s), "event");
  HIPCHK(launch_decide(s, d), "decide");
  HIPCHK(hipEventRecord(rg[2], s), "event");
  if (e->useGraph) {
    if (x.gScanEpoch != e->epoch || !x.gScan) {
      const int rc = capture(s, x.gScan, [&]() { return scanTail(s); });
      if (rc) return rc;
      x.gScanEpoch = e->epoch;
    }
    HIPCHK(hipGraphLaunch(x.gScan, s), "scan graph");
  } else {
    const int rc = scanTail(s);
    if (rc) return rc;
  }
  if (e->anyTwcc)  // the transports' sequence ranges of this batch (after the forwarded counts)
    HIPCHK(launch_twcc_base(s, e->dDTs, nd, x.dFwdCnt, e->dTwccCtrD, e->dTwccCtrT, e->dTwccTOff, e->dTwccTList,
                            e->nTwccT, x.dTwccBase),
           "twcc base");
  HIPCHK(hipEventRecord(x.decided, s), "event");
  if (e->nSeqDD && e->ddAlloc) {  // sequencer ddBytes (decide stream: before the next batch's decide)
    SeqDDLaunch q;
    q.list = e->dSeqDDList;
    q.n = e->nSeqDD;
    q.hot = e->dHot;
    q.seq = e->dSeq;
    q.seqSize = e->cfg.seq_size;
    q.srm = e->dSrm;
    q.srmStride = e->srmStride;
    q.srmCap = e->srmCap;
    q.ddIdx = e->dSeqDDIdx;
    q.seqDD = e->dSeqDD;
    q.recs = x.dRecs;
    q.fbase = x.dFBase;
    q.wide = x.dWide;
    q.slotBase = x.dSlotBase;
    q.fwdCnt = x.dFwdCnt;
    q.pkts = e->curPkts;
    q.ddArena = x.dDDArena;
    HIPCHK(launch_seq_dd(s, q), "sequencer dd");
  }

  // ---- emit stage (emit stream): wire bytes.  The decide stream goes
  // straight on to the next batch's decide.
  hipStream_t es = e->emitS;
  HIPCHK(hipStreamWaitEvent(es, x.decided, 0), "wait decided");
  HIPCHK(hipEventRecord(rg[3], es), "event");
  EmitLaunch m;
  m.perm = e->dPerm;
  m.recBase = x.dRecBase;
  m.byteBase = x.dByteBase;
  m.gFirst = x.dGFirst;
  m.slotBase = x.dSlotBase;
  m.totals = x.dTot + 2;
  m.recs = x.dRecs;
  m.fbase = x.dFBase;
  m.wide = x.dWide;
  m.pkts = e->curPkts;
  m.arena = e->curArena;
  m.dts = e->dDTs;
  m.ndts = nd;
  m.out = x.dOut;
  m.outArena = x.dOutArena;
  m.outCap = e->cfg.max_out_pkts;
  m.outByteCap = e->cfg.max_out_bytes;
  m.err = x.dErr;
  m.ddArena = e->ddAlloc ? x.dDDArena : nullptr;
  m.maxDts = e->cfg.max_downtracks;
  m.npkts = e->curN;
  m.tupleCap = e->cfg.max_batch_tuples;
  m.arenaLen = e->curArenaLen;
  m.ddCap = e->ddArenaCap;
  m.twccBase = e->anyTwcc ? x.dTwccBase : nullptr;
  m.gCap = e->cfg.max_out_pkts / 64 + 2;
  // One workgroup per 64-record group (grid = the capacity bound; workgroups
  // past the batch's records exit at once).  Short-lived workgroups free their
  // slots as they finish, so the next batch's decide stage (higher-priority
  // stream) interleaves with this emit instead of waiting for a persistent grid.
  m.grid = e->emitPersistent ? e->emitGrid
                             : uint32_t(((e->cfg.max_out_pkts + 63) / 64 + 7) / 8 * 8);
  // An ingest-fed batch's emit runs beside the next ingest chain: at a low
  // fan-out (fewer than emitCapFanout DownTracks per track) its workgroups are
  // capped at 12 per CU (LDS reserved at launch), which keeps the payload lines
  // its DownTracks re-read in L2 and leaves CUs to the ingest (configs[1], 9 per
  // track: 0.78 -> 0.74 ms per step).  A submitted batch's emit, or one with a
  // high fan-out, is most of the step and runs uncapped (the cap: ExtPacket
  // configs[1] 0.455 -> 0.54 ms, configs[2] 2.51 -> 2.83 ms, configs[3] 3.35 ->
  // 3.47 ms; profiles/r6_ab_runs.txt).
  m.ldsPad = (ingestFed && uint64_t(nd) < uint64_t(e->emitCapFanout) * std::max<uint32_t>(1, nt)) ? e->emitLdsPad : 0;
  if (nd) HIPCHK(launch_emit(e->emitS, m), "emit");
  HIPCHK(hipEventRecord(rg[4], e->emitS), "event");
  HIPCHK(launch_accumulate(e->emitS, x.dStats, x.dTot, e->dCum, x.dErr, e->dSticky), "accumulate");
  // (sendingPacket -> RTPStatsSender.Update of every forwarded tuple runs inside
  // decide, ss_fold.)  This batch's bucket copies (sender stream) finish before
  // its context counts as done.
  if (e->bktStorePending) {
    HIPCHK(hipEventRecord(x.sent, e->sendS), "event");
    HIPCHK(hipStreamWaitEvent(e->emitS, x.sent, 0), "wait bucket store");
  }
  e->bktStorePending = false;
  HIPCHK(hipEventRecord(x.emitted, e->emitS), "event");
  if (e->hostProf && e->nRuns >= 3) {  // steady state: skip the first runs (initial control ops, first touch)
    e->hp[0] += std::chrono::duration<double, std::milli>(tp1 - tp0).count();
    e->hp[1] += std::chrono::duration<double, std::milli>(tp2 - tp1).count();
    e->hp[2] += std::chrono::duration<double, std::milli>(tp25 - tp2).count();
    e->hp[6] += std::chrono::duration<double, std::milli>(tp3 - tp25).count();
    e->hp[3] += ms_since(tp3);
    e->hp[4] += ms_since(tp0);
    e->hp[5] += 1;
  }
  x.used = true;
  x.protectedRun = false;
  if (!e->protRun.empty()) e->protRun[e->nRuns % 256] = 0;
  e->lastCtx = ci;
  e->nRuns++;
  e->haveBatch = false;
  e->curNDev = nullptr;
  e->curDD = nullptr;
  return LKF_OK;
}

// Waits for all queued batches; reports (and clears) the sticky error word:
// every error of every batch and ingest since the last lkf_sync.
int lkf_sync(lkf_engine *e) {
  if (!e) return LKF_EINVAL;
  int rc = drain_streams(e);
  if (rc) return rc;
  uint32_t acc = 0;
  D2H(&acc, e->dSticky, sizeof(acc), "err copy");
  if (e->debugDD && e->ddAlloc) {
    for (int c = 0; c < lkf_engine::kCtx; c++) {
      uint64_t u[2] = {0, 0};
      if (hipMemcpy(u, e->ctx[c].dDDUsed, sizeof(u), hipMemcpyDeviceToHost) == hipSuccess)
        fprintf(stderr, "[lkf dd] sync after run %llu: ctx %d cursor %llu (%p)\n", (unsigned long long)e->nRuns, c,
                (unsigned long long)u[0], static_cast<void *>(e->ctx[c].dDDUsed));
    }
  }
  if (!acc) return LKF_OK;
  HIPCHK(hipMemset(e->dSticky, 0, sizeof(uint32_t)), "err reset");
  HIPCHK(hipDeviceSynchronize(), "err reset sync");  // null-stream memset vs the engine's streams
  if (acc & (3u << 8)) {
    e->err = "raw batch not grouped by track / bad stream handle";
    return LKF_EORDER;
  }
  if (acc & (4u << 8)) {
    e->err = "dependency descriptor beyond an engine limit (templates, frame diffs, chains)";
    return LKF_ENOSPC;
  }
  if (acc & (8u << 8)) {
    e->err = "RTCP NACK pair capacity of an ingest exceeded";
    return LKF_ENOSPC;
  }
  if (acc & 32u) {
    e->err = "internal: a DownTrack with padding exclusions was decided by the plain kernel";
    return LKF_EINVAL;
  }
  if (acc & 16u) {
    e->err = "dependency descriptor unreadable, missing its lkf_pkt_dd entry, or beyond an engine limit";
    return LKF_EINVAL;
  }
  if (acc & 3u) {
    e->err = "batch not grouped by track / bad track handle";
    return LKF_EORDER;
  }
  if (acc & 64u) {
    e->err = "output or tuple capacity exceeded (decide: the batch's DD arena)";
    if (e->ddAlloc) {  // (the contexts' cursors, for the report)
      char buf[192];
      size_t o = 0;
      for (auto &x : e->ctx) {
        uint64_t u[2] = {0, 0};
        if (x.dDDUsed && hipMemcpy(u, x.dDDUsed, sizeof(u), hipMemcpyDeviceToHost) == hipSuccess && o < sizeof(buf))
          o += size_t(snprintf(buf + o, sizeof(buf) - o, " %llu/%llu", (unsigned long long)u[0],
                               (unsigned long long)e->ddArenaCap));
      }
      e->err += " used/cap:";
      e->err += buf;
      // (diagnostic) the live allocations around context 0's cursor, and the
      // contexts' small buffers by name
      const uintptr_t c0 = reinterpret_cast<uintptr_t>(e->ctx[0].dDDUsed);
      {
        std::lock_guard<std::mutex> g(dreg().m);
        for (auto it = dreg().a.lower_bound(c0 > (1u << 20) ? c0 - (1u << 20) : 0);
             it != dreg().a.end() && it->first < c0 + (1u << 20); ++it) {
          char t[64];
          snprintf(t, sizeof(t), " [%+lld:%zu]", (long long)(intptr_t(it->first) - intptr_t(c0)), it->second);
          e->err += t;
        }
      }
      for (int c = 0; c < lkf_engine::kCtx; c++) {
        const BatchCtx &x = e->ctx[c];
        const void *ps[] = {x.dTBegin, x.dTEnd, x.dTRuns, x.dErr, x.dTot, x.dDesc, x.dEvents, x.dEvOff, x.dEvLane,
                            x.dDDUsed, x.dStats, x.dPartA, x.dFBase, x.dLayerCnt, x.dTwccBase};
        const char *nm[] = {"tB", "tE", "tR", "err", "tot", "desc", "ev", "evoff", "evlane", "ddu", "stats",
                            "partA", "fbase", "lcnt", "twcc"};
        for (size_t k = 0; k < sizeof(ps) / sizeof(ps[0]); k++) {
          const intptr_t dlt = intptr_t(reinterpret_cast<uintptr_t>(ps[k])) - intptr_t(c0);
          if (ps[k] && dlt > -(1 << 20) && dlt < (1 << 20)) {
            char t[48];
            snprintf(t, sizeof(t), " %d.%s%+lld", c, nm[k], (long long)dlt);
            e->err += t;
          }
        }
      }
    }
    return LKF_ENOSPC;
  }
  if (acc & 12u) {
    e->err = (acc & 8u) ? "output or tuple capacity exceeded (decide: tuple slots)"
                        : "output or tuple capacity exceeded (emit: output records or bytes)";
    return LKF_ENOSPC;
  }
  return LKF_OK;
}

int lkf_get_stats(lkf_engine *e, lkf_stats *out) {
  if (!e || !out) return LKF_EINVAL;
  std::memset(out, 0, sizeof(*out));
  int rc = lkf_sync(e);
  if (e->lastCtx < 0) return rc;
  BatchCtx &x = e->ctx[e->lastCtx];
  uint64_t st[kStatsWords];
  uint64_t tot[4];
  D2H(st, x.dStats, sizeof(st), "stats copy");
  D2H(tot, x.dTot, sizeof(tot), "tot copy");
  out->tuples = st[0];
  out->forwarded = st[1];
  out->out_bytes = st[2];
  out->arena_bytes = tot[3];
  for (int i = 0; i < LKF_DROP_NREASONS; i++) out->drops[i] = st[4 + i];
  return rc;
}

int lkf_output_device(lkf_engine *e, const lkf_out **d_out, uint64_t *n_out, const uint8_t **d_arena,
                      uint64_t *arena_len) {
  if (!e) return LKF_EINVAL;
  int rc = lkf_sync(e);
  if (rc) return rc;
  if (e->lastCtx < 0) {
    if (d_out) *d_out = e->ctx[0].dOut;
    if (d_arena) *d_arena = e->ctx[0].dOutArena;
    if (n_out) *n_out = 0;
    if (arena_len) *arena_len = 0;
    return LKF_OK;
  }
  BatchCtx &x = e->ctx[e->lastCtx];
  uint64_t tot[4];
  D2H(tot, x.dTot, sizeof(tot), "tot copy");
  // a batch whose output exceeded the engine's capacity wrote nothing (k_emit
  // flags it; lkf_sync reported it once): never hand out a range beyond the
  // output buffers, whatever the caller did with that report
  if (tot[2] > e->cfg.max_out_pkts || tot[3] > e->cfg.max_out_bytes) {
    e->err = "output or tuple capacity exceeded";
    return LKF_ENOSPC;
  }
  if (d_out) *d_out = x.dOut;
  if (d_arena) *d_arena = x.dOutArena;
  if (n_out) *n_out = tot[2];
  if (arena_len) *arena_len = tot[3];
  return LKF_OK;
}

int lkf_drain(lkf_engine *e, lkf_out *out, uint64_t cap, uint8_t *arena, uint64_t arena_cap, uint64_t *n_out,
              uint64_t *arena_len) {
  const lkf_out *dOut = nullptr;
  const uint8_t *dAr = nullptr;
  uint64_t n = 0, len = 0;
  int rc = lkf_output_device(e, &dOut, &n, &dAr, &len);
  if (rc) return rc;
  if (n_out) *n_out = n;
  if (arena_len) *arena_len = len;
  if (n > cap || len > arena_cap) return LKF_ENOSPC;
  if (out && n) {
    const int r = copy_to_host(e, out, dOut, n * sizeof(lkf_out), "drain recs");
    if (r) return r;
  }
  if (arena && len) return copy_to_host(e, arena, dAr, len, "drain bytes");
  return LKF_OK;
}

int lkf_drain_run(lkf_engine *e, uint32_t age, lkf_out *out, uint64_t cap, uint8_t *arena, uint64_t arena_cap,
                  uint64_t *n_out, uint64_t *arena_len) {
  if (!e || age >= uint32_t(lkf_engine::kCtx) || uint64_t(age) >= e->nRuns) return LKF_EINVAL;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  BatchCtx &x = e->ctx[(e->nRuns - 1 - age) % lkf_engine::kCtx];
  HIPCHK(hipEventSynchronize(x.emitted), "wait emitted");
  uint64_t tot[4];
  D2H(tot, x.dTot, sizeof(tot), "tot copy");
  if (n_out) *n_out = tot[2];
  if (arena_len) *arena_len = tot[3];
  if (tot[2] > e->cfg.max_out_pkts || tot[3] > e->cfg.max_out_bytes) {  // (see lkf_output_device)
    e->err = "output or tuple capacity exceeded";
    return LKF_ENOSPC;
  }
  if (tot[2] > cap || tot[3] > arena_cap) return LKF_ENOSPC;
  if (out && tot[2]) {
    const int r = copy_to_host(e, out, x.dOut, tot[2] * sizeof(lkf_out), "drain recs");
    if (r) return r;
  }
  if (arena && tot[3]) {
    const int r = copy_to_host(e, arena, x.dOutArena, tot[3], "drain bytes");
    if (r) return r;
  }
  return LKF_OK;
}

int lkf_drain_run_async(lkf_engine *e, uint32_t age, lkf_out *out, uint64_t cap, uint8_t *arena, uint64_t arena_cap,
                        uint64_t *n_out, uint64_t *arena_len) {
  if (!e || age >= uint32_t(lkf_engine::kCtx) || uint64_t(age) >= e->nRuns) return LKF_EINVAL;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  if (!e->d2hS) HIPCHK(hipStreamCreateWithFlags(&e->d2hS, hipStreamNonBlocking), "copy stream");
  BatchCtx &x = e->ctx[(e->nRuns - 1 - age) % lkf_engine::kCtx];
  HIPCHK(hipEventSynchronize(x.emitted), "wait emitted");
  uint64_t tot[4];
  D2H(tot, x.dTot, sizeof(tot), "tot copy");
  if (n_out) *n_out = tot[2];
  if (arena_len) *arena_len = tot[3];
  if (tot[2] > e->cfg.max_out_pkts || tot[3] > e->cfg.max_out_bytes) {  // (see lkf_output_device)
    e->err = "output or tuple capacity exceeded";
    return LKF_ENOSPC;
  }
  if (tot[2] > cap || tot[3] > arena_cap) return LKF_ENOSPC;
  // (the context is reused only after run n + 3 is enqueued, which the caller
  // does after lkf_drain_wait: the source stays valid while the copies run)
  if (out && tot[2]) {
    CHKRANGE(x.dOut, tot[2] * sizeof(lkf_out), "async d2h");
    HIPCHK(hipMemcpyAsync(out, x.dOut, tot[2] * sizeof(lkf_out), hipMemcpyDeviceToHost, e->d2hS), "drain recs");
  }
  if (arena && tot[3]) {
    CHKRANGE(x.dOutArena, tot[3], "async d2h");
    HIPCHK(hipMemcpyAsync(arena, x.dOutArena, tot[3], hipMemcpyDeviceToHost, e->d2hS), "drain bytes");
  }
  return LKF_OK;
}

int lkf_drain_wait(lkf_engine *e) {
  if (!e) return LKF_EINVAL;
  if (e->d2hS) HIPCHK(hipStreamSynchronize(e->d2hS), "copy stream sync");
  return LKF_OK;
}

// ---- SRTP protect ---------------------------------------------------------
static int srtp_init(lkf_engine *e) {
  if (e->dAesTab) return LKF_OK;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  HIPCHK(dalloc(&e->dAesTab, 256 + 64), "alloc aes tables");
  HIPCHK(dalloc(&e->dSrtpDT, e->cfg.max_downtracks), "alloc srtp dt");
  HIPCHK(hipMemsetAsync(e->dSrtpDT, 0, sizeof(SrtpDT) * e->cfg.max_downtracks, e->own), "srtp dt init");
  HIPCHK(launch_aes_tables(e->own, e->dAesTab), "aes tables");
  HIPCHK(hipStreamSynchronize(e->own), "srtp init sync");
  for (auto &r : e->protRing)
    for (auto &ev : r) HIPCHK(hipEventCreate(&ev), "protect event");
  e->protRun.assign(256, 0);
  return LKF_OK;
}

int32_t lkf_add_transport(lkf_engine *e, const lkf_transport_params *p) {
  if (!e || !p || (p->profile != LKF_SRTP_AES128_CM_HMAC_SHA1_80 && p->profile != LKF_SRTP_AEAD_AES_128_GCM))
    return LKF_EINVAL;
  int rc = srtp_init(e);
  if (rc) return rc;
  const uint32_t t = uint32_t(e->transports.size());
  if (t + 1 > e->transportCap) {  // grow; queued protect stages read the keys
    rc = drain_streams(e);
    if (rc) return rc;
    const uint32_t cap = std::max<uint32_t>(64, 2 * e->transportCap);
    lkf_transport_params *np = nullptr;
    SrtpKeys *nk = nullptr;
    HIPCHK(dalloc(&np, cap), "alloc transports");
    HIPCHK(dalloc(&nk, cap), "alloc srtp keys");
    if (t) {
      HIPCHK(hipMemcpy(np, e->dTransports, t * sizeof(*np), hipMemcpyDeviceToDevice), "copy transports");
      HIPCHK(hipMemcpy(nk, e->dSrtpKeys, t * sizeof(*nk), hipMemcpyDeviceToDevice), "copy keys");
    }
    if (e->dTransports) HIPCHK(dfree(e->dTransports), "free transports");
    if (e->dSrtpKeys) HIPCHK(dfree(e->dSrtpKeys), "free keys");
    e->dTransports = np;
    e->dSrtpKeys = nk;
    e->transportCap = cap;
  }
  e->transports.push_back(*p);
  HIPCHK(hipMemcpyAsync(e->dTransports + t, &e->transports.back(), sizeof(*p), hipMemcpyHostToDevice, e->own),
         "transport copy");
  HIPCHK(launch_srtp_keys(e->own, e->dTransports + t, t, 1, e->dAesTab, e->dSrtpKeys), "srtp keys");
  HIPCHK(hipStreamSynchronize(e->own), "srtp keys sync");
  return int32_t(t);
}

int lkf_set_downtrack_transport(lkf_engine *e, int32_t dt, int32_t t) {
  if (!e || dt < 0 || dt >= int32_t(e->dtp.size()) || t < -1 || t >= int32_t(e->transports.size()))
    return LKF_EINVAL;
  int rc = srtp_init(e);
  if (rc) return rc;
  rc = flush_topology(e);  // (the DownTrack's static parameters are on the device)
  if (rc) return rc;
  rc = drain_streams(e);  // queued protect stages read the binding
  if (rc) return rc;
  SrtpDT v{uint32_t(t + 1), 0, 0};
  HIPCHK(hipMemcpy(e->dSrtpDT + dt, &v, sizeof(v), hipMemcpyHostToDevice), "srtp bind");
  // its transport-wide sequence numbers: the transport's counter from now on
  e->dtTransport[size_t(dt)] = t;
  const uint32_t grp = t >= 0 ? (0x80000000u | uint32_t(t)) : uint32_t(dt);
  HIPCHK(hipMemcpy(reinterpret_cast<uint8_t *>(e->dDTs + dt) + offsetof(DevDT, twccGroup), &grp, sizeof(grp),
                   hipMemcpyHostToDevice),
         "twcc group");
  if (e->dtp[size_t(dt)].ext_transport_cc) e->twccDirty = true;
  return upload_done(e);
}

// pion/rtp NewAbsSendTimeExtension(t).Marshal(): NTP time >> 14, 24 bits
static uint32_t abs_send_time(int64_t unixNs) {
  const uint64_t u = uint64_t(unixNs);
  const uint64_t sec = u / 1000000000ull + 0x83AA7E80ull;
  const uint64_t frac = ((u % 1000000000ull) << 32) / 1000000000ull;
  return uint32_t((((sec << 32) | frac) >> 14) & 0xFFFFFF);
}

int lkf_protect(lkf_engine *e, int64_t send_time_ns) {
  if (!e || e->lastCtx < 0) return LKF_EINVAL;
  int rc = srtp_init(e);
  if (rc) return rc;
  BatchCtx &x = e->ctx[e->lastCtx];
  if (!x.dProt)
    HIPCHK(dalloc(&x.dProt, e->cfg.max_out_bytes + 16 * uint64_t(e->cfg.max_out_pkts)), "alloc protected arena");
  SrtpProtectArgs a;
  a.tab = e->dAesTab;
  a.totals = x.dTot + 2;
  a.out = x.dOut;
  a.arena = x.dOutArena;
  a.prot = x.dProt;
  a.dts = e->dDTs;
  a.sd = e->dSrtpDT;
  a.keys = e->dSrtpKeys;
  a.cap = e->cfg.max_out_pkts;
  a.absVal = abs_send_time(send_time_ns);
  // after the run's emit stage on the emit stream; the context's "emitted"
  // event (what its next reuse waits for) moves behind the protect stage
  const size_t slot = (e->nRuns - 1) % 256;
  HIPCHK(hipEventRecord(e->protRing[slot][0], e->emitS), "event");
  HIPCHK(launch_srtp_protect(e->emitS, a, uint32_t(e->dtp.size()), e->dPerm, x.dRecBase, x.dFwdCnt), "protect");
  HIPCHK(hipEventRecord(e->protRing[slot][1], e->emitS), "event");
  HIPCHK(hipEventRecord(x.emitted, e->emitS), "event");
  e->protRun[slot] = 1;
  x.protectedRun = true;
  return LKF_OK;
}

int lkf_output_protected_device(lkf_engine *e, const uint8_t **d_arena, uint64_t *arena_len) {
  if (!e || e->lastCtx < 0) return LKF_EINVAL;
  int rc = lkf_sync(e);
  if (rc) return rc;
  BatchCtx &x = e->ctx[e->lastCtx];
  if (!x.protectedRun) {
    e->err = "the last run was not protected (lkf_protect)";
    return LKF_EINVAL;
  }
  uint64_t tot[4];
  D2H(tot, x.dTot, sizeof(tot), "tot copy");
  if (d_arena) *d_arena = x.dProt;
  if (arena_len) *arena_len = tot[3] + 16 * tot[2];
  return LKF_OK;
}

int lkf_protect_timing_window(lkf_engine *e, uint32_t n, float *protect_ms) {
  if (!e || !e->dAesTab || n == 0 || n > 256 || n > e->nRuns) return LKF_EINVAL;
  float sum = 0;
  for (uint64_t r = e->nRuns - n; r < e->nRuns; r++) {
    if (!e->protRun[r % 256]) return LKF_EINVAL;
    HIPCHK(hipEventSynchronize(e->protRing[r % 256][1]), "evsync");
    float a = 0;
    HIPCHK(hipEventElapsedTime(&a, e->protRing[r % 256][0], e->protRing[r % 256][1]), "elapsed");
    sum += a;
  }
  if (protect_ms) *protect_ms = sum;
  return LKF_OK;
}

int lkf_drain_protected(lkf_engine *e, uint8_t *arena, uint64_t cap, uint64_t *arena_len) {
  const uint8_t *d = nullptr;
  uint64_t len = 0;
  int rc = lkf_output_protected_device(e, &d, &len);
  if (rc) return rc;
  if (arena_len) *arena_len = len;
  if (len > cap) return LKF_ENOSPC;
  if (arena && len) D2H(arena, d, len, "drain protected");
  return LKF_OK;
}

int lkf_sender_stats_get(lkf_engine *e, int32_t dt, lkf_sender_stats *out) {
  if (!e || !out || dt < 0 || dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  SenderStats s;
  D2H(&s, e->dSS + dt, sizeof(s), "sender stats copy");
  std::memset(out, 0, sizeof(*out));
  out->ext_start_sn = s.extStartSN;
  out->ext_highest_sn = s.extHighestSN;
  out->ext_start_ts = s.extStartTS;
  out->ext_highest_ts = s.extHighestTS;
  out->first_time_ns = s.firstTime;
  out->highest_time_ns = s.highestTime;
  out->last_transit = s.lastTransit;
  out->last_jitter_ext_ts = s.lastJitterExtTimestamp;
  out->bytes = s.bytes;
  out->header_bytes = s.headerBytes;
  out->bytes_duplicate = s.bytesDuplicate;
  out->header_bytes_duplicate = s.headerBytesDuplicate;
  out->bytes_padding = s.bytesPadding;
  out->header_bytes_padding = s.headerBytesPadding;
  out->packets_duplicate = s.packetsDuplicate;
  out->packets_padding = s.packetsPadding;
  out->packets_out_of_order = s.packetsOutOfOrder;
  out->packets_lost = s.packetsLost;
  out->jitter = s.jitter;
  out->max_jitter = s.maxJitter;
  out->frames = s.frames;
  out->key_frames = s.keyFrames;
  out->initialized = s.initialized;
  out->clock_rate = s.clockRate;
  D2H(out->gap_histogram, e->dSSGap + size_t(dt) * kGapWords, kGapBins * sizeof(uint32_t), "sender gap copy");
  return LKF_OK;
}

int lkf_sender_sninfo(lkf_engine *e, int32_t dt, uint64_t esn, uint32_t *out) {
  if (!e || !out || dt < 0 || dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  D2H(out, e->dSSRing + size_t(dt) * kSnInfoSize + (esn & (kSnInfoSize - 1)), sizeof(uint32_t), "sninfo copy");
  return LKF_OK;
}

int lkf_sender_stats_seed(lkf_engine *e, int32_t dt, int32_t from_dt) {
  if (!e || dt < 0 || dt >= int32_t(e->dtp.size()) || from_dt < 0 || from_dt >= int32_t(e->dtp.size()))
    return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  SenderStats from, to;
  D2H(&from, e->dSS + from_dt, sizeof(from), "sender stats copy");
  if (!from.initialized) return LKF_OK;  // rtpStatsBase.seed: from must be initialized
  D2H(&to, e->dSS + dt, sizeof(to), "sender stats copy");
  from.clockRate = to.clockRate;  // params are not seeded
  HIPCHK(hipMemcpy(e->dSS + dt, &from, sizeof(from), hipMemcpyHostToDevice), "sender stats seed");
  HIPCHK(hipMemcpy(e->dSSGap + size_t(dt) * kGapWords, e->dSSGap + size_t(from_dt) * kGapWords,
                   kGapWords * sizeof(uint32_t), hipMemcpyDeviceToDevice),
         "sender gap seed");
  HIPCHK(hipMemcpy(e->dSSRing + size_t(dt) * kSnInfoSize, e->dSSRing + size_t(from_dt) * kSnInfoSize,
                   kSnInfoSize * sizeof(uint32_t), hipMemcpyDeviceToDevice),
         "sender ring seed");
  return upload_done(e);
}

int lkf_get_state(lkf_engine *e, int32_t dt, lkf_fwd_state *o) {
  if (!e || !o || dt < 0 || dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  DTHot h;
  D2H(&h, e->dHot + dt, sizeof(h), "state copy");
  std::memset(o, 0, sizeof(*o));
  if (!(h.flags & F_STARTED)) return LKF_OK;  // GetState forwarder.go:344-346
  o->started = 1;
  o->reference_layer_spatial = h.referenceLayerSpatial;
  o->pre_start_time_ns = h.preStartTime;
  o->ext_first_ts = h.extFirstTS;
  o->ref_ts_offset = h.refTSOffset;
  o->ext_last_sn = h.extLastSN;
  o->ext_second_last_sn = h.extSecondLastSN;
  o->ext_last_ts = h.extLastTS;
  o->ext_second_last_ts = h.extSecondLastTS;
  o->last_marker = (h.flags & F_LAST_MARKER) ? 1 : 0;
  o->second_last_marker = (h.flags & F_SECOND_LAST_MARKER) ? 1 : 0;
  o->has_vp8 = (h.flags & F_VP8) ? 1 : 0;
  o->vp8_ext_last_picture_id = h.extLastPictureId;
  o->vp8_picture_id_used = (h.flags & F_PICID_USED) ? 1 : 0;
  o->vp8_last_tl0picidx = h.lastTl0;
  o->vp8_tl0picidx_used = (h.flags & F_TL0_USED) ? 1 : 0;
  o->vp8_tid_used = (h.flags & F_TID_USED) ? 1 : 0;
  o->vp8_last_keyidx = h.lastKeyIdx;
  o->vp8_keyidx_used = (h.flags & F_KEYIDX_USED) ? 1 : 0;
  return LKF_OK;
}

int lkf_seed_state(lkf_engine *e, int32_t dt, const lkf_fwd_state *i) {
  if (!e || !i || dt < 0 || dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
  if (!i->started) return LKF_OK;  // SeedState forwarder.go:360-362
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  DTHot h;
  D2H(&h, e->dHot + dt, sizeof(h), "state copy");
  auto setf = [&](uint32_t f, bool v) { h.flags = v ? (h.flags | f) : (h.flags & ~f); };
  // RTPMunger.SeedLast rtpmunger.go:126-133
  h.extLastSN = i->ext_last_sn;
  h.extSecondLastSN = i->ext_second_last_sn;
  h.extLastTS = i->ext_last_ts;
  h.extSecondLastTS = i->ext_second_last_ts;
  setf(F_LAST_MARKER, i->last_marker);
  setf(F_SECOND_LAST_MARKER, i->second_last_marker);
  // codecMunger.SeedState vp8.go:99-109 (only a VP8 munger takes VP8State)
  if ((h.flags & F_VP8) && i->has_vp8) {
    h.extLastPictureId = i->vp8_ext_last_picture_id;
    setf(F_PICID_USED, i->vp8_picture_id_used);
    h.lastTl0 = i->vp8_last_tl0picidx;
    setf(F_TL0_USED, i->vp8_tl0picidx_used);
    setf(F_TID_USED, i->vp8_tid_used);
    h.lastKeyIdx = i->vp8_last_keyidx;
    setf(F_KEYIDX_USED, i->vp8_keyidx_used);
  }
  setf(F_STARTED, true);
  h.referenceLayerSpatial = i->reference_layer_spatial;
  h.preStartTime = i->pre_start_time_ns;
  h.extFirstTS = i->ext_first_ts;
  h.refTSOffset = i->ref_ts_offset;
  HIPCHK(hipMemcpy(e->dHot + dt, &h, sizeof(h), hipMemcpyHostToDevice), "seed copy");
  return upload_done(e);
}

int lkf_seq_lookup(lkf_engine *e, int32_t dt, const uint16_t *sns, uint32_t n, int64_t now_ns, lkf_seq_meta *out,
                   uint32_t *n_out) {
  if (!e || dt < 0 || dt >= int32_t(e->dtp.size()) || (n && (!sns || !out))) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  if (n > e->seqScratchCap) {
    if (e->dSns) (void)dfree(e->dSns);
    if (e->dSeqOut) (void)dfree(e->dSeqOut);
    e->seqScratchCap = std::max<uint32_t>(n, 256);
    HIPCHK(dalloc(&e->dSns, e->seqScratchCap), "alloc");
    HIPCHK(dalloc(&e->dSeqOut, e->seqScratchCap), "alloc");
  }
  if (!e->dSeqN) HIPCHK(dalloc(&e->dSeqN, 1), "alloc");
  if (n) HIPCHK(hipMemcpy(e->dSns, sns, n * sizeof(uint16_t), hipMemcpyHostToDevice), "sns copy");
  rc = upload_done(e);
  if (rc) return rc;
  HIPCHK(launch_seq_lookup(e->own, e->dHot, e->dSeq, e->cfg.seq_size, e->dSrm, e->srmStride, e->srmCap, uint32_t(dt),
                           e->dSns, n, now_ns / 1000000,
                           e->dSeqOut, e->dSeqN),
         "seq lookup");
  HIPCHK(hipStreamSynchronize(e->own), "sync");
  uint32_t cnt = 0;
  D2H(&cnt, e->dSeqN, sizeof(cnt), "n copy");
  if (cnt) D2H(out, e->dSeqOut, cnt * sizeof(lkf_seq_meta), "out copy");
  if (n_out) *n_out = cnt;
  return LKF_OK;
}

static int rtx_reserve(lkf_engine *e, uint32_t n) {
  if (n <= e->rtxCap) return LKF_OK;
  for (void *p : {static_cast<void *>(e->dNacks), static_cast<void *>(e->dNackG), static_cast<void *>(e->dNackValid),
                  static_cast<void *>(e->dRtx), static_cast<void *>(e->dRtxSrc), static_cast<void *>(e->dRtxLen),
                  static_cast<void *>(e->dRtxOff)})
    if (p) (void)dfree(p);
  e->rtxCap = std::max<uint32_t>(n, 1024);
  HIPCHK(dalloc(&e->dNacks, e->rtxCap), "alloc nacks");
  HIPCHK(dalloc(&e->dNackG, e->rtxCap + 1), "alloc nack groups");
  HIPCHK(dalloc(&e->dNackValid, e->rtxCap), "alloc nack valid");
  HIPCHK(dalloc(&e->dRtx, e->rtxCap), "alloc rtx");
  HIPCHK(dalloc(&e->dRtxSrc, e->rtxCap), "alloc rtx src");
  HIPCHK(dalloc(&e->dRtxLen, e->rtxCap), "alloc rtx len");
  HIPCHK(dalloc(&e->dRtxOff, e->rtxCap), "alloc rtx off");
  return LKF_OK;
}

int lkf_rtx_lookup(lkf_engine *e, const lkf_nack *nacks, uint32_t n, int64_t now_ns, lkf_rtx *out, uint32_t cap,
                   uint32_t *n_out) {
  if (!e || !n_out || (n && !nacks)) return LKF_EINVAL;
  *n_out = 0;
  // groups: one per DownTrack's contiguous NACK list (a DownTrack must not reappear)
  std::vector<uint32_t> gStart;
  std::vector<uint8_t> seen(e->dtp.size(), 0);
  for (uint32_t i = 0; i < n; i++) {
    const int32_t dt = nacks[i].dt;
    if (dt < 0 || dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
    if (i == 0 || nacks[i - 1].dt != dt) {
      if (seen[dt]) return LKF_EORDER;
      seen[dt] = 1;
      if (e->active[dt]) gStart.push_back(i);  // a removed DownTrack answers no NACK
    }
  }
  e->rtxNow = now_ns;  // retransmitPackets' time.Now() for the RTX sendingPacket (lkf_rtx_emit)
  if (gStart.empty()) return LKF_OK;
  // group ends: the next group's start or the end of its DownTrack's run
  std::vector<uint32_t> gb(gStart.size() + 1);
  std::vector<lkf_nack> packed;
  packed.reserve(n);
  for (size_t g = 0; g < gStart.size(); g++) {
    gb[g] = uint32_t(packed.size());
    uint32_t i = gStart[g];
    const int32_t dt = nacks[i].dt;
    while (i < n && nacks[i].dt == dt) packed.push_back(nacks[i++]);
  }
  gb[gStart.size()] = uint32_t(packed.size());
  const uint32_t m = uint32_t(packed.size());
  int rc = flush_topology(e);
  if (rc) return rc;
  // The lookup reads and updates the sequencer records and the DownTracks'
  // hot state, which between runs only the decide stream touches: ordered on
  // that stream behind the queued decides (their emits keep running), as the
  // allocation calls.
  hipStream_t s = e->decS;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  if (m > e->rtxCap) HIPCHK(hipStreamSynchronize(s), "sync decide stream");  // (rtx_reserve reallocates)
  rc = rtx_reserve(e, m);
  if (rc) return rc;
  HIPCHK(hipEventRecord(e->inEv, e->own), "event");
  HIPCHK(hipStreamWaitEvent(s, e->inEv, 0), "wait own stream");
  HIPCHK(hipMemcpyAsync(e->dNacks, packed.data(), m * sizeof(lkf_nack), hipMemcpyHostToDevice, s), "nacks copy");
  HIPCHK(hipMemcpyAsync(e->dNackG, gb.data(), gb.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s),
         "groups copy");
  HIPCHK(launch_rtx_lookup(s, e->dHot, e->dSeq, e->cfg.seq_size, e->dSrm, e->srmStride, e->srmCap, e->dNacks,
                           e->dNackG, uint32_t(gStart.size()), now_ns / 1000000, e->dRtx, e->dNackValid),
         "rtx lookup");
  std::vector<lkf_rtx> r(m);
  std::vector<uint32_t> v(m);
  CHKRANGE(e->dRtx, m * sizeof(lkf_rtx), "async d2h");
  HIPCHK(hipMemcpyAsync(r.data(), e->dRtx, m * sizeof(lkf_rtx), hipMemcpyDeviceToHost, s), "rtx copy");
  CHKRANGE(e->dNackValid, m * sizeof(uint32_t), "async d2h");
  HIPCHK(hipMemcpyAsync(v.data(), e->dNackValid, m * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "valid copy");
  HIPCHK(hipStreamSynchronize(s), "sync");
  uint32_t k = 0;
  for (uint32_t i = 0; i < m; i++) k += v[i];
  *n_out = k;
  if (cap < k) return LKF_ENOSPC;
  k = 0;
  for (uint32_t i = 0; i < m; i++)
    if (v[i]) out[k++] = r[i];
  return LKF_OK;
}

static int rtx_emit_common(lkf_engine *e, const lkf_rtx *rtx, uint32_t n, const uint8_t *srcArena,
                           const std::vector<uint16_t> &srcHdr, lkf_out *out, uint8_t *out_arena, uint64_t out_cap,
                           uint32_t *n_out, uint64_t *out_len);
// The retransmissions run on the sender stream, after every queued stage that
// touches what they read or update: the decides and sequencer DD bytes
// (decide stream), the sender statistics (sender stream for long batches,
// emit stream for short ones — the RTX sendingPacket updates the same
// RTPStatsSender) and the bucket copies (sender stream).  The host then waits
// for that point: the scratch buffers below are rewritten from the host.
static int rtx_order(lkf_engine *e, uint32_t n) {
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  if (e->twccDirty) {  // a transport-cc DownTrack added / bound since the last run: its counters first
    const int rt = rebuild_twcc(e);
    if (rt) return rt;
  }
  const int rc = sender_after_queued(e);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(e->sendS), "sync sender stream");
  return rtx_reserve(e, n);
}
int lkf_rtx_emit(lkf_engine *e, const lkf_rtx *rtx, uint32_t n, const lkf_raw_pkt *src, const uint8_t *src_arena,
                 uint64_t src_len, lkf_out *out, uint8_t *out_arena, uint64_t out_cap, uint32_t *n_out,
                 uint64_t *out_len) {
  if (!e || !n_out || !out_len || (n && (!rtx || !src))) return LKF_EINVAL;
  *n_out = 0;
  *out_len = 0;
  if (!n) return LKF_OK;
  for (uint32_t i = 0; i < n; i++) {
    if (rtx[i].dt < 0 || rtx[i].dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
    if (src[i].len && (!src_arena || uint64_t(src[i].off) + src[i].len > src_len)) return LKF_EINVAL;
  }
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = rtx_order(e, n);
  if (rc) return rc;
  if (src_len + 64 > e->rtxInCap) {
    if (e->dRtxIn) (void)dfree(e->dRtxIn);
    e->rtxInCap = std::max<uint64_t>(src_len + 64, 1 << 20);
    HIPCHK(dalloc(&e->dRtxIn, e->rtxInCap), "alloc rtx in");
  }
  // uploads ordered on the sender stream ahead of the kernels that read them
  // (a pageable hipMemcpy may return before its DMA lands, and the engine's
  // streams do not order against the null stream)
  HIPCHK(hipMemcpyAsync(e->dRtx, rtx, n * sizeof(lkf_rtx), hipMemcpyHostToDevice, e->sendS), "rtx copy");
  HIPCHK(hipMemcpyAsync(e->dRtxSrc, src, n * sizeof(lkf_raw_pkt), hipMemcpyHostToDevice, e->sendS), "src copy");
  if (src_len)
    HIPCHK(hipMemcpyAsync(e->dRtxIn, src_arena, src_len, hipMemcpyHostToDevice, e->sendS), "src arena copy");
  std::vector<uint16_t> hdr(n, 0);
  for (uint32_t i = 0; i < n; i++) {
    if (!src[i].len) continue;
    const uint8_t *b = src_arena + src[i].off;
    uint32_t h = 12 + 4 * (b[0] & 0xf);
    if ((b[0] & 0x10) && h + 4 <= src[i].len) h += 4 + 4 * ((uint32_t(b[h + 2]) << 8) | b[h + 3]);
    hdr[i] = uint16_t(h);
  }
  return rtx_emit_common(e, rtx, n, e->dRtxIn, hdr, out, out_arena, out_cap, n_out, out_len);
}

// The retransmissions from device-side sources (dRtx / dRtxSrc filled; srcArena:
// the bytes they index): sizes, offsets, wire bytes, then sendingPacket per
// retransmission (srcHdr[i]: the source header's size).
static int rtx_emit_common(lkf_engine *e, const lkf_rtx *rtx, uint32_t n, const uint8_t *srcArena,
                           const std::vector<uint16_t> &srcHdr, lkf_out *out, uint8_t *out_arena, uint64_t out_cap,
                           uint32_t *n_out, uint64_t *out_len) {
  int rc = LKF_OK;
  const uint8_t *rtxDD = nullptr;
  if (e->nSeqDD) {  // epm.ddBytes of each record (its sequencer slot)
    if (n > e->rtxDDCap) {
      if (e->dRtxDD) (void)dfree(e->dRtxDD);
      e->rtxDDCap = std::max<uint32_t>(n, 1024);
      HIPCHK(dalloc(&e->dRtxDD, size_t(e->rtxDDCap) * kSeqDDBytes), "alloc rtx dd");
    }
    HIPCHK(launch_rtx_dd(e->sendS, n, e->dRtx, e->dDTs, e->dSeq, e->cfg.seq_size, e->dSeqDDIdx, e->dSeqDD,
                         e->dRtxDD),
           "rtx dd");
    rtxDD = e->dRtxDD;
  }
  HIPCHK(launch_rtx_emit(e->sendS, false, n, e->dRtx, e->dRtxSrc, srcArena, e->dDTs, e->dTracks, e->dRtxLen,
                         nullptr, nullptr, rtxDD),
         "rtx size");
  std::vector<uint32_t> len(n);
  CHKRANGE(e->dRtxLen, n * sizeof(uint32_t), "async d2h");
  HIPCHK(hipMemcpyAsync(len.data(), e->dRtxLen, n * sizeof(uint32_t), hipMemcpyDeviceToHost, e->sendS), "len copy");
  HIPCHK(hipStreamSynchronize(e->sendS), "sync");
  std::vector<uint64_t> off(n, 0);
  uint64_t tot = 0;
  uint32_t k = 0;
  for (uint32_t i = 0; i < n; i++) {
    off[i] = tot;
    if (len[i]) {
      tot += (uint64_t(len[i]) + 15) & ~uint64_t(15);
      k++;
    }
  }
  *n_out = k;
  *out_len = tot;
  if (tot > out_cap || (k && (!out || !out_arena))) return LKF_ENOSPC;
  if (tot + 64 > e->rtxOutCap) {
    if (e->dRtxOut) (void)dfree(e->dRtxOut);
    e->rtxOutCap = std::max<uint64_t>(tot + 64, 1 << 20);
    HIPCHK(dalloc(&e->dRtxOut, e->rtxOutCap), "alloc rtx out");
  }
  HIPCHK(hipMemcpyAsync(e->dRtxOff, off.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, e->sendS), "off copy");
  HIPCHK(launch_rtx_emit(e->sendS, true, n, e->dRtx, e->dRtxSrc, srcArena, e->dDTs, e->dTracks, e->dRtxLen,
                         e->dRtxOff, e->dRtxOut, rtxDD),
         "rtx write");
  if (e->anyTwcc)  // transport-cc numbers in record (send) order
    HIPCHK(launch_twcc_stamp(e->sendS, e->dDTs, e->dTwccCtrD, e->dTwccCtrT, n, nullptr, nullptr, nullptr, e->dRtx,
                             e->dRtxOff, e->dRtxLen, e->dRtxOut),
           "twcc stamp");
  if (tot) {
    CHKRANGE(e->dRtxOut, tot, "async d2h");
    HIPCHK(hipMemcpyAsync(out_arena, e->dRtxOut, tot, hipMemcpyDeviceToHost, e->sendS), "rtx bytes copy");
  }
  HIPCHK(hipStreamSynchronize(e->sendS), "sync");
  {  // sendingPacket (downtrack.go:1671-1681): the bucket packet's header as
     // unmarshalled (CSRCs and extensions kept), the forwarded payload
    std::vector<SenderUpd> ul;
    for (uint32_t i = 0; i < n; i++) {
      if (!len[i]) continue;
      const uint32_t h = srcHdr[i];
      const uint8_t *w = out_arena + off[i];  // the RTX header as written (CSRCs, pacer extension block)
      uint32_t outHdr = 12 + 4 * uint32_t(w[0] & 0xf);
      if (w[0] & 0x10) outHdr += 4 + 4 * ((uint32_t(w[outHdr + 2]) << 8) | w[outHdr + 3]);
      SenderUpd u;
      std::memset(&u, 0, sizeof(u));
      u.esn = rtx[i].meta.ext_sn;
      u.ets = rtx[i].meta.ext_ts;
      u.t = e->rtxNow;
      u.dt = uint32_t(rtx[i].dt);
      u.hdr = uint16_t(h);
      u.pay = uint16_t(len[i] - outHdr);
      u.marker = rtx[i].meta.marker ? 1 : 0;
      ul.push_back(u);
    }
    rc = sender_list(e, ul);
    if (rc) return rc;
  }
  k = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (!len[i]) continue;
    lkf_out &o = out[k++];
    std::memset(&o, 0, sizeof(o));
    o.ext_sn = rtx[i].meta.ext_sn;
    o.ext_ts = rtx[i].meta.ext_ts;
    o.out_off = off[i];
    o.dt = uint32_t(rtx[i].dt);
    o.pkt = i;
    o.out_len = uint16_t(len[i]);
    o.flags = rtx[i].meta.marker ? LKF_OUT_MARKER : 0;
    o.layer = rtx[i].meta.layer;
  }
  return LKF_OK;
}

// Receiver.ReadRTP(layer, sourceSeqNo) (receiver.go:559-566) from the GPU
// buckets: the DownTrack's track buffer of the record's layer (an SVC track's
// single buffer; a closed buffer returns io.EOF), Bucket.GetPacket on the
// device, then the retransmissions as lkf_rtx_emit.
int lkf_rtx_emit_bucket(lkf_engine *e, const lkf_rtx *rtx, uint32_t n, lkf_out *out, uint8_t *out_arena,
                        uint64_t out_cap, uint32_t *n_out, uint64_t *out_len) {
  if (!e || !n_out || !out_len || (n && !rtx)) return LKF_EINVAL;
  *n_out = 0;
  *out_len = 0;
  if (!n) return LKF_OK;
  for (uint32_t i = 0; i < n; i++)
    if (rtx[i].dt < 0 || rtx[i].dt >= int32_t(e->dtp.size())) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = rtx_order(e, n);
  if (rc) return rc;
  std::vector<int32_t> sid(n, -1);
  std::vector<uint16_t> sn(n);
  {
    std::vector<std::vector<int32_t>> byTrack(e->tracks.size());
    for (size_t s = 0; s < e->streams.size(); s++) byTrack[size_t(e->streams[s].track)].push_back(int32_t(s));
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t t = e->dtp[size_t(rtx[i].dt)].track;
      sn[i] = rtx[i].meta.source_sn;
      if (!e->trackActive[t]) continue;
      const auto &v = byTrack[t];
      const int layer = rtx[i].meta.layer < 0 ? 0 : rtx[i].meta.layer;
      if (v.size() == 1) {
        sid[i] = v[0];
      } else {
        for (int32_t s : v)
          if (e->streams[size_t(s)].layer == layer) sid[i] = s;
      }
    }
  }
  if (!e->bktSlots) std::fill(sid.begin(), sid.end(), -1);
  if (n > e->bktReadCap) {
    if (e->dBktStream) (void)dfree(e->dBktStream);
    if (e->dBktSn) (void)dfree(e->dBktSn);
    e->bktReadCap = std::max<uint32_t>(n, 1024);
    HIPCHK(dalloc(&e->dBktStream, e->bktReadCap), "alloc bucket reads");
    HIPCHK(dalloc(&e->dBktSn, e->bktReadCap), "alloc bucket read sns");
  }
  // (uploads on the sender stream, ahead of k_bkt_read / k_rtx: see lkf_rtx_emit)
  HIPCHK(hipMemcpyAsync(e->dRtx, rtx, n * sizeof(lkf_rtx), hipMemcpyHostToDevice, e->sendS), "rtx copy");
  HIPCHK(hipMemcpyAsync(e->dBktStream, sid.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, e->sendS),
         "bucket read copy");
  HIPCHK(hipMemcpyAsync(e->dBktSn, sn.data(), n * sizeof(uint16_t), hipMemcpyHostToDevice, e->sendS),
         "bucket sn copy");
  if (uint64_t(n) * kBktSlot + 64 > e->rtxInCap) {
    if (e->dRtxIn) (void)dfree(e->dRtxIn);
    e->rtxInCap = std::max<uint64_t>(uint64_t(n) * kBktSlot + 64, 1 << 20);
    HIPCHK(dalloc(&e->dRtxIn, e->rtxInCap), "alloc rtx in");
  }
  HIPCHK(launch_bucket_read(e->sendS, n, e->dBktStream, e->dBktSn, e->dBkt, e->dBktTag, e->dBktRing, e->dRtxIn,
                            e->dRtxSrc),
         "bucket read");
  std::vector<lkf_raw_pkt> src(n);
  CHKRANGE(e->dRtxSrc, n * sizeof(lkf_raw_pkt), "async d2h");
  HIPCHK(hipMemcpyAsync(src.data(), e->dRtxSrc, n * sizeof(lkf_raw_pkt), hipMemcpyDeviceToHost, e->sendS),
         "src back");
  HIPCHK(hipStreamSynchronize(e->sendS), "sync");
  std::vector<uint16_t> hdr(n, 0);
  for (uint32_t i = 0; i < n; i++) hdr[i] = uint16_t(src[i].len ? src[i].reserved : 0);
  return rtx_emit_common(e, rtx, n, e->dRtxIn, hdr, out, out_arena, out_cap, n_out, out_len);
}

// ---- padding / blank frames (downtrack.go:764-859, :1307-1401) -------------
// Worst-case space per request is reserved (padding: ceil(bytes / 275)
// packets of at most 12 + 8 + 255 bytes; blank: two packets of at most
// 12 + 8 + 80), the kernel fills what it sends, the host packs it.
// sendingPacket -> RTPStatsSender.Update for host-listed packets (padding,
// blank frames, RTX): grouped by DownTrack in call order, one thread per
// DownTrack (k_sender_updates).  Runs on e->own after the producing kernel.
static int sender_list(lkf_engine *e, std::vector<SenderUpd> &list) {
  if (list.empty()) return LKF_OK;
  std::stable_sort(list.begin(), list.end(), [](const SenderUpd &a, const SenderUpd &b) { return a.dt < b.dt; });
  std::vector<uint32_t> g;
  for (uint32_t i = 0; i < list.size(); i++)
    if (i == 0 || list[i].dt != list[i - 1].dt) g.push_back(i);
  g.push_back(uint32_t(list.size()));
  if (list.size() > e->ssListCap || g.size() > e->ssListCap + 1) {
    if (e->dSSList) (void)dfree(e->dSSList);
    if (e->dSSGroups) (void)dfree(e->dSSGroups);
    e->ssListCap = uint32_t(std::max<size_t>(2 * list.size(), 4096));
    HIPCHK(dalloc(&e->dSSList, e->ssListCap), "alloc sender list");
    HIPCHK(dalloc(&e->dSSGroups, e->ssListCap + 1), "alloc sender groups");
  }
  // on the sender stream, after the queued runs' sender statistics (sender or
  // emit stream), which update the same DownTracks' RTPStatsSender
  hipStream_t st = e->sendS;
  {
    const int rc = sender_after_queued(e);
    if (rc) return rc;
  }
  HIPCHK(hipMemcpyAsync(e->dSSList, list.data(), list.size() * sizeof(SenderUpd), hipMemcpyHostToDevice, st),
         "sender list copy");
  HIPCHK(hipMemcpyAsync(e->dSSGroups, g.data(), g.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st),
         "sender groups copy");
  SenderListLaunch a;
  a.list = e->dSSList;
  a.gBegin = e->dSSGroups;
  a.ngroups = uint32_t(g.size() - 1);
  a.ss = e->dSS;
  a.ring = e->dSSRing;
  a.gap = e->dSSGap;
  HIPCHK(launch_sender_updates(st, a), "sender updates");
  HIPCHK(hipStreamSynchronize(st), "sync");
  return LKF_OK;
}

// a padding / blank packet's header with the pacer's extension block
// (abs-send-time) and the TWCC interceptor's element (k_pad pad_hdr_len)
static uint32_t pad_hdr_bytes(const lkf_downtrack_params &p) {
  const uint32_t eb = (p.ext_abs_send_time ? 4u : 0u) + (p.ext_transport_cc ? 3u : 0u);
  return eb ? 16u + ((eb + 3) & ~3u) : 12u;
}

static int pad_common(lkf_engine *e, int blank, const lkf_pad_req *reqs, uint32_t n, int64_t now_ns, lkf_out *out,
                      uint8_t *arena, uint64_t out_cap, uint64_t arena_cap, uint32_t *n_out, uint64_t *arena_len,
                      uint32_t *bytes_sent) {
  if (!e || !n_out || !arena_len || (n && !reqs)) return LKF_EINVAL;
  *n_out = 0;
  *arena_len = 0;
  if (!n) return LKF_OK;
  std::vector<uint8_t> seen(e->dtp.size(), 0);
  std::vector<uint64_t> off(2 * size_t(n));
  uint64_t recs = 0, bytes = 0;
  for (uint32_t i = 0; i < n; i++) {
    const int32_t dt = reqs[i].dt;
    if (dt < 0 || dt >= int32_t(e->dtp.size()) || seen[dt]) return LKF_EINVAL;
    seen[dt] = 1;
    const uint64_t np = !e->active[dt] ? 0 : blank ? 2 : (uint64_t(reqs[i].bytes_to_send) + 274) / 275;
    off[i] = recs;
    off[n + i] = bytes;
    recs += np;
    bytes += np * (blank ? 112 : 288);
  }
  int rc = flush_topology(e);
  if (rc) return rc;
  if (e->twccDirty) {  // a transport-cc DownTrack added / bound since the last run: its counters first
    rc = rebuild_twcc(e);
    if (rc) return rc;
  }
  // k_pad reads and writes the DownTracks' Forwarder / sequencer state, which
  // between runs only the decide stream touches: it runs there, behind the
  // queued decides (their emits keep running); its sendingPacket updates go to
  // the sender stream (sender_list)
  const hipStream_t ds = e->decS;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  if (n > e->padCap) {
    for (void *p : {static_cast<void *>(e->dPadReq), static_cast<void *>(e->dPadOff), static_cast<void *>(e->dPadCnt)})
      if (p) (void)dfree(p);
    e->padCap = std::max<uint32_t>(n, 1024);
    HIPCHK(dalloc(&e->dPadReq, e->padCap), "alloc pad reqs");
    HIPCHK(dalloc(&e->dPadOff, 2 * size_t(e->padCap)), "alloc pad offsets");
    HIPCHK(dalloc(&e->dPadCnt, 2 * size_t(e->padCap)), "alloc pad counts");
  }
  if (recs > e->padOutCap) {
    if (e->dPadOut) (void)dfree(e->dPadOut);
    e->padOutCap = std::max<uint64_t>(recs, 4096);
    HIPCHK(dalloc(&e->dPadOut, e->padOutCap), "alloc pad out");
  }
  if (bytes > e->padArenaCap) {
    if (e->dPadArena) (void)dfree(e->dPadArena);
    e->padArenaCap = std::max<uint64_t>(bytes, 1 << 20);
    HIPCHK(dalloc(&e->dPadArena, e->padArenaCap), "alloc pad arena");
  }
  // a removed DownTrack sends nothing: its request is dropped before the kernel
  std::vector<lkf_pad_req> q(reqs, reqs + n);
  std::vector<uint32_t> live;
  for (uint32_t i = 0; i < n; i++)
    if (e->active[q[i].dt]) live.push_back(i);
  std::vector<lkf_pad_req> lq(live.size());
  std::vector<uint64_t> loff(2 * live.size());
  for (size_t j = 0; j < live.size(); j++) {
    lq[j] = q[live[j]];
    loff[j] = off[live[j]];
    loff[live.size() + j] = off[n + live[j]];
  }
  const uint32_t m = uint32_t(live.size());
  std::vector<uint32_t> cnt(2 * size_t(m), 0);
  if (m) {
    HIPCHK(hipEventRecord(e->inEv, e->own), "event");
    HIPCHK(hipStreamWaitEvent(ds, e->inEv, 0), "wait own stream");
    // the request uploads on the decide stream, ordered ahead of k_pad (see lkf_rtx_emit)
    HIPCHK(hipMemcpyAsync(e->dPadReq, lq.data(), m * sizeof(lkf_pad_req), hipMemcpyHostToDevice, ds), "pad req copy");
    HIPCHK(hipMemcpyAsync(e->dPadOff, loff.data(), 2 * size_t(m) * sizeof(uint64_t), hipMemcpyHostToDevice, ds),
           "pad off copy");
    PadLaunch a;
    a.blank = blank;
    a.n = m;
    a.reqs = e->dPadReq;
    a.nowNs = now_ns;
    a.hot = e->dHot;
    a.dts = e->dDTs;
    a.tracks = e->dTracks;
    a.rm = e->dRm;
    a.seq = e->dSeq;
    a.seqSize = e->cfg.seq_size;
    a.srm = e->dSrm;
    a.srmStride = e->srmStride;
    a.srmCap = e->srmCap;
    a.dtCum = e->dDTCum;
    a.recOff = e->dPadOff;
    a.byteOff = e->dPadOff + m;
    a.out = e->dPadOut;
    a.arena = e->dPadArena;
    a.cnt = e->dPadCnt;
    a.bytes = e->dPadCnt + m;
    HIPCHK(launch_pad(ds, a), "pad");
    if (e->anyTwcc)  // transport-cc numbers in request (send) order
      HIPCHK(launch_twcc_stamp(ds, e->dDTs, e->dTwccCtrD, e->dTwccCtrT, m, e->dPadOut, e->dPadOff, e->dPadCnt, nullptr,
                               nullptr, nullptr, e->dPadArena),
             "twcc stamp");
    HIPCHK(hipStreamSynchronize(ds), "sync");
    D2H(cnt.data(), e->dPadCnt, 2 * size_t(m) * sizeof(uint32_t), "pad cnt copy");
  }
  if (bytes_sent)
    for (uint32_t i = 0; i < n; i++) bytes_sent[i] = 0;
  uint64_t k = 0, tot = 0;
  for (uint32_t j = 0; j < m; j++) {
    k += cnt[j];
    if (bytes_sent) bytes_sent[live[j]] = cnt[m + j];
    if (!blank && cnt[j] && !e->seqRM[lq[j].dt]) {  // pushPadding ran: reschedule (rebuild_sched)
      e->seqRM[lq[j].dt] = 1;
      e->schedDirty = true;
    }
  }
  std::vector<lkf_out> recv(recs ? recs : 1);
  std::vector<uint8_t> arv(bytes ? bytes : 1);
  if (k) {
    D2H(recv.data(), e->dPadOut, recs * sizeof(lkf_out), "pad out copy");
    D2H(arv.data(), e->dPadArena, bytes, "pad arena copy");
    // sendingPacket (downtrack.go:835-846, :1377-1386): isPadding, a 12-B
    // header (the pacer adds the extensions later), the payload as padding
    std::vector<SenderUpd> ul;
    for (uint32_t j = 0; j < m; j++)
      for (uint32_t c = 0; c < cnt[j]; c++) {
        const lkf_out &o = recv[loff[j] + c];
        SenderUpd u;
        std::memset(&u, 0, sizeof(u));
        u.esn = o.ext_sn;
        u.ets = o.ext_ts;
        u.t = now_ns;
        u.dt = o.dt;
        u.hdr = 12;
        u.pay = 0;
        u.pad = uint16_t(o.out_len - pad_hdr_bytes(e->dtp[o.dt]));
        u.marker = (o.flags & LKF_OUT_MARKER) ? 1 : 0;
        ul.push_back(u);
      }
    rc = sender_list(e, ul);
    if (rc) return rc;
  }
  for (uint32_t j = 0; j < m; j++)
    for (uint32_t c = 0; c < cnt[j]; c++) tot += (uint64_t(recv[loff[j] + c].out_len) + 15) & ~uint64_t(15);
  *n_out = uint32_t(k);
  *arena_len = tot;
  if (k > out_cap || tot > arena_cap || (k && (!out || !arena))) return LKF_ENOSPC;
  uint64_t w = 0, pos = 0;
  for (uint32_t j = 0; j < m; j++)
    for (uint32_t c = 0; c < cnt[j]; c++) {
      lkf_out o = recv[loff[j] + c];
      const uint64_t al = (uint64_t(o.out_len) + 15) & ~uint64_t(15);
      std::memcpy(arena + pos, arv.data() + o.out_off, al);
      o.out_off = pos;
      o.pkt = live[j];
      out[w++] = o;
      pos += al;
    }
  return LKF_OK;
}

// ---- the dependency-descriptor stream tracker (streamtracker_dd.go) --------
int32_t lkf_add_stream_tracker_dd(lkf_engine *e, int32_t track) {
  if (!e || track < 0 || track >= int32_t(e->tracks.size()) || !track_has_dd(e->tracks[track])) return LKF_EINVAL;
  if (e->trackDDTrk.size() < e->tracks.size()) e->trackDDTrk.resize(e->tracks.size(), -1);
  if (e->trackDDTrk[track] >= 0) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  if (!e->dTrackDDTrk) {
    HIPCHK(dalloc(&e->dTrackDDTrk, e->cfg.max_tracks), "alloc track dd trackers");
    HIPCHK(hipMemset(e->dTrackDDTrk, 0xff, size_t(e->cfg.max_tracks) * sizeof(uint32_t)), "track dd trackers reset");
  }
  if (e->nDDTrk + 1 > e->ddTrkCap) {
    const uint32_t cap = std::max<uint32_t>(2 * e->ddTrkCap, 256);
    DDTrkState *n = nullptr;
    HIPCHK(dalloc(&n, cap), "alloc dd trackers");
    if (e->nDDTrk) HIPCHK(hipMemcpy(n, e->dDDTrk, e->nDDTrk * sizeof(DDTrkState), hipMemcpyDeviceToDevice), "dd trackers move");
    if (e->dDDTrk) HIPCHK(dfree(e->dDDTrk), "free dd trackers");
    e->dDDTrk = n;
    e->ddTrkCap = cap;
  }
  DDTrkState t;
  std::memset(&t, 0, sizeof(t));
  t.maxS = t.maxT = -1;
  for (int l = 0; l < 3; l++) t.lastNotified[l] = -1;
  t.track = uint32_t(track);
  const uint32_t id = e->nDDTrk++;
  HIPCHK(hipMemcpy(e->dDDTrk + id, &t, sizeof(t), hipMemcpyHostToDevice), "dd tracker init");
  HIPCHK(hipMemcpy(e->dTrackDDTrk + track, &id, sizeof(id), hipMemcpyHostToDevice), "track dd tracker");
  e->trackDDTrk[track] = int32_t(id);
  e->epoch++;  // the prep graph's k_dd_decode observes the trackers
  return upload_done(e) ? LKF_EHIP : int32_t(id);
}

// SetPaused / Stop (streamtracker_dd.go:57-68, :123-137) on the host copy
int lkf_dd_tracker_ctl(lkf_engine *e, int32_t tracker, int32_t op, int32_t arg) {
  if (!e || tracker < 0 || uint32_t(tracker) >= e->nDDTrk) return LKF_EINVAL;
  if (op != LKF_TRACKER_PAUSE && op != LKF_TRACKER_STOP) return LKF_EINVAL;
  int rc = drain_streams(e);
  if (rc) return rc;
  DDTrkState t;
  D2H(&t, e->dDDTrk + tracker, sizeof(t), "dd tracker read");
  if (op == LKF_TRACKER_STOP) {
    if (!(t.flags & DT_STOPPED)) t.flags = (t.flags | DT_STOPPED) & ~DT_WORKER;
  } else {
    const bool p = arg != 0;
    if (bool(t.flags & DT_PAUSED) != p) {
      if (p) {
        t.flags |= DT_PAUSED | DT_WORKER;  // a worker drains the bitrates while paused
      } else {  // resetLocked :108-121
        t.flags &= ~(DT_PAUSED | DT_WORKER);
        std::memset(t.bytes, 0, sizeof(t.bytes));
        std::memset(t.bitrate, 0, sizeof(t.bitrate));
      }
    }
  }
  HIPCHK(hipMemcpy(e->dDDTrk + tracker, &t, sizeof(t), hipMemcpyHostToDevice), "dd tracker write");
  return upload_done(e);
}

int lkf_dd_trackers_tick(lkf_engine *e, const int32_t *trackers, uint32_t n, int64_t bitrate_elapsed_ns,
                         lkf_dd_tracker_status *out) {
  if (!e || (n && (!trackers || !out))) return LKF_EINVAL;
  std::vector<uint8_t> seen(e->nDDTrk, 0);
  for (uint32_t i = 0; i < n; i++) {
    if (trackers[i] < 0 || uint32_t(trackers[i]) >= e->nDDTrk || seen[trackers[i]]) return LKF_EINVAL;
    seen[trackers[i]] = 1;
  }
  if (!n) return LKF_OK;
  int rc = drain_streams(e);
  if (rc) return rc;
  HIPCHK(grow(&e->dDDTrkIds, e->ddTrkIdsCap, n), "alloc dd tracker ids");
  HIPCHK(grow(&e->dDDTrkOut, e->ddTrkOutCap, n), "alloc dd tracker out");
  HIPCHK(hipMemcpy(e->dDDTrkIds, trackers, n * sizeof(int32_t), hipMemcpyHostToDevice), "dd tracker ids copy");
  rc = upload_done(e);
  if (rc) return rc;
  HIPCHK(launch_dd_tracker_tick(e->own, e->dDDTrk, e->dDDTrkIds, n, bitrate_elapsed_ns, e->dDDTrkOut), "dd tracker tick");
  HIPCHK(hipStreamSynchronize(e->own), "sync");
  D2H(out, e->dDDTrkOut, n * sizeof(lkf_dd_tracker_status), "dd tracker out copy");
  return LKF_OK;
}

// ---- stream trackers (streamtracker.go, streamtracker_packet.go) ------------
int32_t lkf_add_stream_tracker(lkf_engine *e, int32_t track, int32_t layer, uint32_t samples_required,
                               uint32_t cycles_required) {
  if (!e || track < 0 || track >= int32_t(e->tracks.size()) || layer < 0) return LKF_EINVAL;
  int rc = drain_streams(e);
  if (rc) return rc;
  if (e->nTrk + 1 > e->trkCap) {
    const uint32_t cap = std::max<uint32_t>(2 * e->trkCap, 1024);
    TrackerState *n = nullptr;
    HIPCHK(dalloc(&n, cap), "alloc trackers");
    if (e->nTrk) HIPCHK(hipMemcpy(n, e->dTrk, e->nTrk * sizeof(TrackerState), hipMemcpyDeviceToDevice), "trackers move");
    if (e->dTrk) HIPCHK(dfree(e->dTrk), "free trackers");
    e->dTrk = n;
    e->trkCap = cap;
  }
  e->epoch++;  // the prep graph observes every tracker
  TrackerState t = {};
  t.track = uint32_t(track);
  t.layer = layer;
  t.samples = samples_required;
  t.cycles = cycles_required;
  HIPCHK(hipMemcpy(e->dTrk + e->nTrk, &t, sizeof(t), hipMemcpyHostToDevice), "tracker init");
  rc = upload_done(e);
  if (rc) return rc;
  return int32_t(e->nTrk++);
}

// a StreamTrackerFrame (streamtracker_frame.go:39-211) with the source's
// StreamTrackerFrameConfig.MinFPS (config.go:413-458)
int32_t lkf_add_stream_tracker_frame(lkf_engine *e, int32_t track, int32_t layer, uint32_t clock_rate,
                                     double min_fps) {
  if (!e || track < 0 || track >= int32_t(e->tracks.size()) || layer < 0 || clock_rate == 0) return LKF_EINVAL;
  const int32_t id = lkf_add_stream_tracker(e, track, layer, 0, 0);
  if (id < 0) return id;
  TrackerState t;
  D2H(&t, e->dTrk + id, sizeof(t), "tracker read");
  t.frame = 1;
  t.clockRate = clock_rate;
  t.minFPS = min_fps;
  tracker_frame_reset_fps(t);
  HIPCHK(hipMemcpy(e->dTrk + id, &t, sizeof(t), hipMemcpyHostToDevice), "tracker write");
  const int rc = upload_done(e);
  return rc ? rc : id;
}

// Reset / SetPaused / Stop (streamtracker.go:127-185) on the host copy of the state
int lkf_stream_tracker_ctl(lkf_engine *e, int32_t tracker, int32_t op, int32_t arg) {
  if (!e || tracker < 0 || uint32_t(tracker) >= e->nTrk) return LKF_EINVAL;
  int rc = drain_streams(e);
  if (rc) return rc;
  TrackerState t;
  D2H(&t, e->dTrk + tracker, sizeof(t), "tracker read");
  auto resetLocked = [&]() {
    t.workerLive = 0;  // generation bump: the worker exits
    t.status = 0;
    for (int i = 0; i < 4; i++) t.bytes[i] = t.bitrate[i] = 0;
    t.countSinceLast = t.cycleCount = 0;
    t.initialized = 0;
    if (t.frame) {  // StreamTrackerFrame.Reset
      tracker_frame_reset_fps(t);
      t.lastCheckSet = 0;
      t.lastCheckNs = 0;
    }
  };
  auto notify = [&]() {
    if (t.status != t.lastNotified) {
      t.lastNotified = t.status;
      t.notifications++;
    }
  };
  switch (op) {
    case LKF_TRACKER_RESET:
      if (t.stopped) return LKF_OK;
      resetLocked();
      notify();
      break;
    case LKF_TRACKER_PAUSE:
      t.paused = arg != 0;
      if (!t.paused) {
        resetLocked();
      } else {
        t.workerLive = 0;
        t.status = 0;
      }
      notify();
      break;
    case LKF_TRACKER_STOP:
      if (t.stopped) return LKF_OK;
      t.stopped = 1;
      t.workerLive = 0;
      break;
    default:
      return LKF_EINVAL;
  }
  HIPCHK(hipMemcpy(e->dTrk + tracker, &t, sizeof(t), hipMemcpyHostToDevice), "tracker write");
  return upload_done(e);
}

int lkf_stream_trackers_tick(lkf_engine *e, const int32_t *trackers, uint32_t n, int check, int64_t bitrate_elapsed_ns,
                             lkf_tracker_status *out) {
  return lkf_stream_trackers_tick_at(e, trackers, n, check, bitrate_elapsed_ns, 0, out);
}
int lkf_stream_trackers_tick_at(lkf_engine *e, const int32_t *trackers, uint32_t n, int check,
                                int64_t bitrate_elapsed_ns, int64_t now_ns, lkf_tracker_status *out) {
  if (!e || (n && (!trackers || !out))) return LKF_EINVAL;
  if (!n) return LKF_OK;
  std::vector<uint8_t> seen(e->nTrk, 0);
  for (uint32_t i = 0; i < n; i++) {
    if (trackers[i] < 0 || uint32_t(trackers[i]) >= e->nTrk || seen[trackers[i]]) return LKF_EINVAL;
    seen[trackers[i]] = 1;
  }
  int rc = drain_streams(e);
  if (rc) return rc;
  HIPCHK(grow(&e->dTrkIds, e->trkIdsCap, n), "alloc tracker ids");
  HIPCHK(grow(&e->dTrkOut, e->trkOutCap, n), "alloc tracker out");
  HIPCHK(hipMemcpy(e->dTrkIds, trackers, n * sizeof(int32_t), hipMemcpyHostToDevice), "tracker ids copy");
  rc = upload_done(e);
  if (rc) return rc;
  HIPCHK(launch_tracker_tick(e->own, e->dTrk, e->dTrkIds, n, check, bitrate_elapsed_ns, now_ns, e->dTrkOut), "tracker tick");
  HIPCHK(hipStreamSynchronize(e->own), "sync");
  D2H(out, e->dTrkOut, n * sizeof(lkf_tracker_status), "tracker out copy");
  return LKF_OK;
}

// ---- RED for Opus (redreceiver.go, redprimaryreceiver.go) -------------------
static int red_common(lkf_engine *e, bool decode, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena,
                      uint64_t arena_len, const int32_t *map, uint32_t map_len, lkf_pkt *out, uint32_t out_cap,
                      uint8_t *out_arena, uint64_t out_arena_cap, uint32_t *n_out, uint64_t *out_arena_len) {
  if (!e || !n_out || !out_arena_len || (n && (!pkts || !arena)) || (map_len && !map)) return LKF_EINVAL;
  *n_out = 0;
  *out_arena_len = 0;
  const uint32_t nt = uint32_t(e->tracks.size());
  if (map_len > nt) return LKF_EINVAL;
  for (uint32_t t = 0; t < map_len; t++)
    if (map[t] >= int32_t(nt) || map[t] < -1) return LKF_EINVAL;
  // groups: the mapped tracks' contiguous packet runs (each track once)
  std::vector<uint32_t> gb, ge;
  std::vector<uint8_t> seen(nt, 0);
  std::vector<uint64_t> off(2 * size_t(n) + 1, 0);
  uint64_t recs = 0, bytes = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t t = pkts[i].track;
    if (t >= nt || uint64_t(pkts[i].arena_off) + pkts[i].payload_off + pkts[i].payload_len > arena_len)
      return LKF_EINVAL;
    if (i == 0 || pkts[i - 1].track != t) {
      if (seen[t]) return LKF_EORDER;
      seen[t] = 1;
      if (t < map_len && map[t] >= 0) {
        gb.push_back(i);
        ge.push_back(i);
      }
    }
    const bool mapped = t < map_len && map[t] >= 0;
    if (mapped) ge.back() = i + 1;
    off[i] = recs;
    off[n + i] = bytes;
    if (mapped) {
      const uint64_t hdr = pkts[i].payload_off, pl = pkts[i].payload_len;
      recs += decode ? 3 : 1;
      bytes += decode ? 3 * ((hdr + pl + 15) & ~15ull) : ((hdr + std::max<uint64_t>(1500, pl + 1) + 15) & ~15ull);
    }
  }
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  if (!gb.empty()) {
    auto &r = e->red;
    if (decode && !e->dRedDec) {
      HIPCHK(dalloc(&e->dRedDec, e->cfg.max_tracks), "alloc red dec");
      HIPCHK(hipMemset(e->dRedDec, 0, size_t(e->cfg.max_tracks) * sizeof(RedDecState)), "red dec reset");
    }
    if (!decode && !e->dRedEnc) {
      HIPCHK(dalloc(&e->dRedEnc, e->cfg.max_tracks), "alloc red enc");
      HIPCHK(hipMemset(e->dRedEnc, 0, size_t(e->cfg.max_tracks) * sizeof(RedEncState)), "red enc reset");
    }
    HIPCHK(grow(&r.in, r.inCap, n), "alloc red in");
    HIPCHK(grow(&r.inArena, r.inArenaCap, arena_len + 64), "alloc red in arena");
    HIPCHK(grow(&r.out, r.outCap, recs), "alloc red out");
    HIPCHK(grow(&r.outArena, r.outArenaCap, bytes), "alloc red out arena");
    HIPCHK(grow(&r.g, r.gCap, 2 * gb.size()), "alloc red groups");
    HIPCHK(grow(&r.cnt, r.cntCap, n), "alloc red counts");
    HIPCHK(grow(&r.map, r.mapCap, nt), "alloc red map");
    HIPCHK(grow(&r.off, r.offCap, 2 * uint64_t(n) + 1), "alloc red offsets");
    std::vector<int32_t> mp(nt, -1);
    for (uint32_t t = 0; t < map_len; t++) mp[t] = map[t];
    std::vector<uint32_t> g(gb);
    g.insert(g.end(), ge.begin(), ge.end());
    HIPCHK(hipMemcpy(r.in, pkts, n * sizeof(lkf_pkt), hipMemcpyHostToDevice), "red in copy");
    HIPCHK(hipMemcpy(r.inArena, arena, arena_len, hipMemcpyHostToDevice), "red arena copy");
    HIPCHK(hipMemcpy(r.g, g.data(), g.size() * sizeof(uint32_t), hipMemcpyHostToDevice), "red groups copy");
    HIPCHK(hipMemcpy(r.map, mp.data(), nt * sizeof(int32_t), hipMemcpyHostToDevice), "red map copy");
    HIPCHK(hipMemcpy(r.off, off.data(), 2 * size_t(n) * sizeof(uint64_t), hipMemcpyHostToDevice), "red off copy");
    HIPCHK(hipMemset(r.cnt, 0, n * sizeof(uint32_t)), "red counts reset");
    rc = upload_done(e);
    if (rc) return rc;
    RedLaunch a;
    a.in = r.in;
    a.inArena = r.inArena;
    a.gBegin = r.g;
    a.gEnd = r.g + gb.size();
    a.ngroups = uint32_t(gb.size());
    a.map = r.map;
    a.enc = e->dRedEnc;
    a.dec = e->dRedDec;
    a.recOff = r.off;
    a.byteOff = r.off + n;
    a.out = r.out;
    a.outArena = r.outArena;
    a.cnt = r.cnt;
    HIPCHK(launch_red(e->own, decode, a), "red");
    HIPCHK(hipStreamSynchronize(e->own), "sync");
  }
  std::vector<uint32_t> cnt(n, 0);
  std::vector<lkf_pkt> rec(recs ? recs : 1);
  std::vector<uint8_t> ar(bytes ? bytes : 1);
  if (!gb.empty()) {
    D2H(cnt.data(), e->red.cnt, n * sizeof(uint32_t), "red cnt copy");
    if (recs) D2H(rec.data(), e->red.out, recs * sizeof(lkf_pkt), "red out copy");
    if (bytes) D2H(ar.data(), e->red.outArena, bytes, "red arena copy");
  }
  uint64_t k = 0, tot = 0;
  for (uint32_t i = 0; i < n; i++)
    for (uint32_t c = 0; c < cnt[i]; c++) {
      const lkf_pkt &o = rec[off[i] + c];
      tot += (uint64_t(o.payload_off) + o.payload_len + 15) & ~15ull;
      k++;
    }
  *n_out = uint32_t(k);
  *out_arena_len = tot;
  if (k > out_cap || tot > out_arena_cap || (k && (!out || !out_arena))) return LKF_ENOSPC;
  uint64_t w = 0, pos = 0;
  for (uint32_t i = 0; i < n; i++)
    for (uint32_t c = 0; c < cnt[i]; c++) {
      lkf_pkt o = rec[off[i] + c];
      const uint64_t len = uint64_t(o.payload_off) + o.payload_len, al = (len + 15) & ~15ull;
      std::memcpy(out_arena + pos, ar.data() + o.arena_off, len);
      std::memset(out_arena + pos + len, 0, al - len);
      o.arena_off = uint32_t(pos);
      out[w++] = o;
      pos += al;
    }
  return LKF_OK;
}

int lkf_red_encode(lkf_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len,
                   const int32_t *map, uint32_t map_len, lkf_pkt *out, uint32_t out_cap, uint8_t *out_arena,
                   uint64_t out_arena_cap, uint32_t *n_out, uint64_t *out_arena_len) {
  return red_common(e, false, pkts, n, arena, arena_len, map, map_len, out, out_cap, out_arena, out_arena_cap, n_out,
                    out_arena_len);
}
int lkf_red_decode(lkf_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len,
                   const int32_t *map, uint32_t map_len, lkf_pkt *out, uint32_t out_cap, uint8_t *out_arena,
                   uint64_t out_arena_cap, uint32_t *n_out, uint64_t *out_arena_len) {
  return red_common(e, true, pkts, n, arena, arena_len, map, map_len, out, out_cap, out_arena, out_arena_cap, n_out,
                    out_arena_len);
}

// ---- Forwarder allocation: AllocateOptimal (forwarder.go:591-725),
// AllocateNextHigher (:1107-1217), GetNextHigherTransition (:1219-1306),
// Pause (:1308-1351) ------------------------------------------------------
static int alloc_common(lkf_engine *e, int mode, const lkf_alloc_req *reqs, const int64_t *capacity, uint32_t n,
                        void *out, size_t outSize) {
  if (!e || (n && (!reqs || !out || (mode == ALLOC_NEXT_HIGHER && !capacity)))) return LKF_EINVAL;
  if (!n) return LKF_OK;
  std::vector<uint8_t> seen(e->dtp.size(), 0);
  for (uint32_t i = 0; i < n; i++) {
    const int32_t dt = reqs[i].dt;
    if (dt < 0 || dt >= int32_t(e->dtp.size()) || seen[dt]) return LKF_EINVAL;
    if (!e->active[dt]) {  // a removed DownTrack has no allocation (its state stays as it was)
      e->err = "allocation request for a removed DownTrack";
      return LKF_EINVAL;
    }
    seen[dt] = 1;
  }
  int rc = flush_topology(e);
  if (rc) return rc;
  // The allocation reads and writes the DownTracks' hot state and last
  // allocation, which between runs only the decide stream touches: it is
  // ordered on that stream after the queued runs' decides, and the host waits
  // for it alone, not for their emits, sender statistics or protect stages
  // (those keep overlapping the call).
  hipStream_t s = e->decS;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  if (n > e->allocCap) {
    HIPCHK(hipStreamSynchronize(s), "sync before alloc buffers realloc");
    if (e->dAllocReq) (void)dfree(e->dAllocReq);
    if (e->dAllocOut) (void)dfree(e->dAllocOut);
    if (e->dAllocCapacity) (void)dfree(e->dAllocCapacity);
    e->allocCap = std::max<uint32_t>(n, 1024);
    HIPCHK(dalloc(&e->dAllocReq, e->allocCap), "alloc alloc reqs");
    HIPCHK(dalloc(&e->dAllocOut, e->allocCap), "alloc alloc out");
    HIPCHK(dalloc(&e->dAllocCapacity, e->allocCap), "alloc alloc capacity");
  }
  static_assert(sizeof(lkf_video_transition) <= sizeof(lkf_allocation), "transition fits the out buffer");
  // (the engine's own stream: anything an earlier control call left there)
  HIPCHK(hipEventRecord(e->inEv, e->own), "event");
  HIPCHK(hipStreamWaitEvent(s, e->inEv, 0), "wait own stream");
  HIPCHK(hipMemcpyAsync(e->dAllocReq, reqs, n * sizeof(lkf_alloc_req), hipMemcpyHostToDevice, s), "alloc req copy");
  if (mode == ALLOC_NEXT_HIGHER)
    HIPCHK(hipMemcpyAsync(e->dAllocCapacity, capacity, n * sizeof(int64_t), hipMemcpyHostToDevice, s),
           "capacity copy");
  HIPCHK(launch_allocate(s, mode, e->dAllocReq, e->dAllocCapacity, n, e->dHot, e->dDTs, e->dTracks, e->dLastAlloc,
                         e->dAllocOut),
         "allocate");
  CHKRANGE(e->dAllocOut, n * outSize, "async d2h");
  HIPCHK(hipMemcpyAsync(out, e->dAllocOut, n * outSize, hipMemcpyDeviceToHost, s), "alloc out copy");
  HIPCHK(hipStreamSynchronize(s), "sync");
  return LKF_OK;
}
int lkf_allocate_optimal(lkf_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_allocation *out) {
  return alloc_common(e, ALLOC_OPTIMAL, reqs, nullptr, n, out, sizeof(lkf_allocation));
}
int lkf_allocate_next_higher(lkf_engine *e, const lkf_alloc_req *reqs, const int64_t *capacity, uint32_t n,
                             lkf_allocation *out) {
  return alloc_common(e, ALLOC_NEXT_HIGHER, reqs, capacity, n, out, sizeof(lkf_allocation));
}
int lkf_next_higher_transition(lkf_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_video_transition *out) {
  return alloc_common(e, ALLOC_TRANSITION, reqs, nullptr, n, out, sizeof(lkf_video_transition));
}
int lkf_pause(lkf_engine *e, const lkf_alloc_req *reqs, uint32_t n, lkf_allocation *out) {
  return alloc_common(e, ALLOC_PAUSE, reqs, nullptr, n, out, sizeof(lkf_allocation));
}

// ---- the cooperative allocation pass (Provisional*, allocateAllTracks) ------
// distinct, active, video DownTracks (the reference's selector is nil for audio)
static int prov_check(lkf_engine *e, const int32_t *dts, uint32_t n, size_t stride) {
  std::vector<uint8_t> seen(e->dtp.size(), 0);
  for (uint32_t i = 0; i < n; i++) {
    const int32_t dt = *reinterpret_cast<const int32_t *>(reinterpret_cast<const uint8_t *>(dts) + i * stride);
    if (dt < 0 || dt >= int32_t(e->dtp.size()) || seen[dt] || !e->active[dt] ||
        e->tracks[e->dtp[dt].track].kind != LKF_KIND_VIDEO) {
      e->err = "provisional allocation: DownTracks must be distinct, active and video";
      return LKF_EINVAL;
    }
    seen[dt] = 1;
  }
  return LKF_OK;
}
static int prov_reserve(lkf_engine *e, uint32_t n, uint32_t ngroups) {
  const lkf_cfg &c = e->cfg;
  if (!e->dProv) {
    HIPCHK(dalloc(&e->dProv, c.max_downtracks), "alloc provisional");
    HIPCHK(hipMemset(e->dProv, 0, size_t(c.max_downtracks) * sizeof(ProvState)), "provisional reset");
  }
  if (n > e->provCap) {
    if (e->dProvReq) (void)dfree(e->dProvReq);
    if (e->dProvOut) (void)dfree(e->dProvOut);
    if (e->dAllocReq) (void)dfree(e->dAllocReq);
    if (e->dAllocOut) (void)dfree(e->dAllocOut);
    if (e->dAllocCapacity) (void)dfree(e->dAllocCapacity);
    e->provCap = std::max<uint32_t>(n, 1024);
    e->allocCap = std::max<uint32_t>(e->allocCap, e->provCap);
    HIPCHK(dalloc(&e->dProvReq, e->provCap), "alloc prov reqs");
    HIPCHK(dalloc(&e->dProvOut, size_t(e->provCap) * sizeof(lkf_allocation)), "alloc prov out");
    HIPCHK(dalloc(&e->dAllocReq, e->allocCap), "alloc alloc reqs");
    HIPCHK(dalloc(&e->dAllocOut, e->allocCap), "alloc alloc out");
    HIPCHK(dalloc(&e->dAllocCapacity, e->allocCap), "alloc alloc capacity");
  }
  if (ngroups > e->provGroupCap) {
    if (e->dProvGroups) (void)dfree(e->dProvGroups);
    e->provGroupCap = std::max<uint32_t>(ngroups, 256);
    HIPCHK(dalloc(&e->dProvGroups, e->provGroupCap), "alloc prov groups");
  }
  return LKF_OK;
}
static int prov_common(lkf_engine *e, int mode, const lkf_prov_req *reqs, const lkf_alloc_req *alloc, uint32_t n,
                       void *out, size_t outSize) {
  if (!e || (n && !reqs && !alloc) || (n && outSize && !out)) return LKF_EINVAL;
  if (!n) return LKF_OK;
  int rc = alloc ? prov_check(e, &alloc[0].dt, n, sizeof(lkf_alloc_req)) : prov_check(e, &reqs[0].dt, n, sizeof(lkf_prov_req));
  if (rc) return rc;
  rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  rc = prov_reserve(e, n, 0);
  if (rc) return rc;
  if (alloc)
    HIPCHK(hipMemcpy(e->dAllocReq, alloc, n * sizeof(lkf_alloc_req), hipMemcpyHostToDevice), "prov req copy");
  else
    HIPCHK(hipMemcpy(e->dProvReq, reqs, n * sizeof(lkf_prov_req), hipMemcpyHostToDevice), "prov req copy");
  rc = upload_done(e);
  if (rc) return rc;
  ProvLaunch a;
  a.mode = mode;
  a.n = n;
  a.reqs = e->dProvReq;
  a.alloc = e->dAllocReq;
  a.hot = e->dHot;
  a.dts = e->dDTs;
  a.tracks = e->dTracks;
  a.last = e->dLastAlloc;
  a.prov = e->dProv;
  a.out = e->dProvOut;
  HIPCHK(launch_prov(e->own, a), "provisional");
  HIPCHK(hipStreamSynchronize(e->own), "sync");
  if (outSize) D2H(out, e->dProvOut, n * outSize, "prov out copy");
  return LKF_OK;
}
static int prov_dts(lkf_engine *e, int mode, const int32_t *dts, uint32_t n, void *out, size_t outSize) {
  if (n && !dts) return LKF_EINVAL;
  std::vector<lkf_prov_req> r(n);
  for (uint32_t i = 0; i < n; i++) {
    std::memset(&r[i], 0, sizeof(r[i]));
    r[i].dt = dts[i];
  }
  return prov_common(e, mode, r.data(), nullptr, n, out, outSize);
}
int lkf_provisional_prepare(lkf_engine *e, const lkf_alloc_req *reqs, uint32_t n) {
  return prov_common(e, PROV_PREPARE, nullptr, reqs, n, nullptr, 0);
}
int lkf_provisional_reset(lkf_engine *e, const int32_t *dts, uint32_t n) {
  return prov_dts(e, PROV_RESET, dts, n, nullptr, 0);
}
int lkf_provisional_allocate(lkf_engine *e, const lkf_prov_req *reqs, uint32_t n, lkf_prov_result *out) {
  return prov_common(e, PROV_ALLOCATE, reqs, nullptr, n, out, sizeof(lkf_prov_result));
}
int lkf_provisional_cooperative(lkf_engine *e, const lkf_prov_req *reqs, uint32_t n, lkf_video_transition *out) {
  return prov_common(e, PROV_COOPERATIVE, reqs, nullptr, n, out, sizeof(lkf_video_transition));
}
int lkf_provisional_best_weighted(lkf_engine *e, const int32_t *dts, uint32_t n, lkf_video_transition *out) {
  return prov_dts(e, PROV_BEST_WEIGHTED, dts, n, out, sizeof(lkf_video_transition));
}
int lkf_provisional_commit(lkf_engine *e, const int32_t *dts, uint32_t n, lkf_allocation *out) {
  return prov_dts(e, PROV_COMMIT, dts, n, out, sizeof(lkf_allocation));
}
int lkf_allocate_all(lkf_engine *e, const lkf_alloc_group *groups, uint32_t ngroups, const lkf_alloc_req *reqs,
                     uint32_t n, lkf_allocation *out) {
  if (!e || (ngroups && !groups) || (n && (!reqs || !out))) return LKF_EINVAL;
  std::vector<uint8_t> cover(n, 0);  // groups are disjoint ranges of reqs
  for (uint32_t g = 0; g < ngroups; g++) {
    if (uint64_t(groups[g].first) + groups[g].count > n) return LKF_EINVAL;
    for (uint32_t k = 0; k < groups[g].count; k++)
      if (cover[groups[g].first + k]++) return LKF_EINVAL;
  }
  if (!ngroups || !n) return LKF_OK;
  int rc = prov_check(e, &reqs[0].dt, n, sizeof(lkf_alloc_req));
  if (rc) return rc;
  rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  rc = prov_reserve(e, n, ngroups);
  if (rc) return rc;
  HIPCHK(hipMemcpy(e->dAllocReq, reqs, n * sizeof(lkf_alloc_req), hipMemcpyHostToDevice), "alloc req copy");
  HIPCHK(hipMemcpy(e->dProvGroups, groups, ngroups * sizeof(lkf_alloc_group), hipMemcpyHostToDevice), "groups copy");
  HIPCHK(hipMemset(e->dProvOut, 0, n * sizeof(lkf_allocation)), "alloc out reset");
  rc = upload_done(e);
  if (rc) return rc;
  HIPCHK(launch_allocate_all(e->own, e->dProvGroups, ngroups, e->dAllocReq, e->dHot, e->dDTs, e->dTracks,
                             e->dLastAlloc, e->dProv, reinterpret_cast<lkf_allocation *>(e->dProvOut)),
         "allocate all");
  HIPCHK(hipStreamSynchronize(e->own), "sync");
  D2H(out, e->dProvOut, n * sizeof(lkf_allocation), "alloc out copy");
  return LKF_OK;
}

int lkf_padding(lkf_engine *e, const lkf_pad_req *reqs, uint32_t n, int64_t now_ns, lkf_out *out, uint8_t *arena,
                uint64_t out_cap, uint64_t arena_cap, uint32_t *n_out, uint64_t *arena_len, uint32_t *bytes_sent) {
  return pad_common(e, 0, reqs, n, now_ns, out, arena, out_cap, arena_cap, n_out, arena_len, bytes_sent);
}

int lkf_blank_frames(lkf_engine *e, const lkf_pad_req *reqs, uint32_t n, int64_t now_ns, lkf_out *out, uint8_t *arena,
                     uint64_t out_cap, uint64_t arena_cap, uint32_t *n_out, uint64_t *arena_len) {
  return pad_common(e, 1, reqs, n, now_ns, out, arena, out_cap, arena_cap, n_out, arena_len, nullptr);
}

int lkf_last_timings(lkf_engine *e, float *decide_ms, float *emit_ms, float *total_ms) {
  return lkf_timing_window(e, 1, decide_ms, emit_ms, total_ms);
}

// decide = sum of the decide-kernel spans, emit = sum of the k_emit spans,
// total = GPU span from the first run's start to the last run's emit end
// (stages overlap across batches, so total < decide + emit).
int lkf_timing_window(lkf_engine *e, uint32_t n, float *decide_ms, float *emit_ms, float *total_ms) {
  if (!e || n == 0 || n > uint32_t(lkf_engine::kRing) || n > e->nRuns) return LKF_EINVAL;
  float sa = 0, sb = 0;
  const uint64_t first = e->nRuns - n;
  for (uint64_t r = first; r < e->nRuns; r++) {
    hipEvent_t *rg = e->ring[r % lkf_engine::kRing];
    HIPCHK(hipEventSynchronize(rg[4]), "evsync");
    float a = 0, b = 0;
    HIPCHK(hipEventElapsedTime(&a, rg[1], rg[2]), "elapsed");
    HIPCHK(hipEventElapsedTime(&b, rg[3], rg[4]), "elapsed");
    sa += a;
    sb += b;
  }
  float c = 0;
  HIPCHK(hipEventElapsedTime(&c, e->ring[first % lkf_engine::kRing][0],
                             e->ring[(e->nRuns - 1) % lkf_engine::kRing][4]),
         "elapsed");
  if (decide_ms) *decide_ms = sa;
  if (emit_ms) *emit_ms = sb;
  if (total_ms) *total_ms = c;
  return LKF_OK;
}

// ---- ingress ------------------------------------------------------------------

// NewBuffer + Bind (buffer.go:124-215); AudioLevelParams defaults config.go:380-385.
int32_t lkf_add_stream(lkf_engine *e, const lkf_stream_params *p) {
  if (!e || !p || p->track < 0 || p->track >= int32_t(e->tracks.size())) return LKF_EINVAL;
  if (e->streams.size() >= e->maxStreams) return LKF_ENOSPC;
  const lkf_track_params &tp = e->tracks[p->track];
  DevStream d;
  std::memset(&d, 0, sizeof(d));
  d.track = uint32_t(p->track);
  d.layer = p->layer;
  d.ssrc = p->ssrc;
  d.clockRate = tp.clock_rate;
  d.codec = tp.codec;
  d.levelExt = p->audio_level_ext;
  d.ddExt = p->dd_ext;
  d.twccExt = p->twcc_ext;
  d.ddIdx = p->dd_ext ? e->nDDStreams++ : 0xffffffffu;  // its DependencyDescriptorParser (buffer.go:193-201)
  d.nack = p->nack ? 1 : 0;  // its NackQueue (buffer.go:248-256)
  const bool dflt = !p->active_level && !p->min_percentile && !p->observe_duration_ms && !p->smooth_intervals;
  d.activeLevel = dflt ? 35 : p->active_level;
  d.minPercentile = dflt ? 40 : p->min_percentile;
  d.observeDuration = dflt ? 400 : p->observe_duration_ms;
  const uint32_t smooth = dflt ? 2 : p->smooth_intervals;
  d.minActiveDuration = uint32_t(d.minPercentile) * d.observeDuration / 100;  // audiolevel.go:55
  d.smoothFactor = smooth > 0 ? double(2) / double(smooth + 1) : 1.0;
  d.activeThreshold = std::pow(10.0, double(d.activeLevel) * (-1.0 / 20));  // ConvertAudioLevel
  e->streams.push_back(*p);
  e->pendStreams.push_back(d);
  e->spkDirty = true;
  return int32_t(e->streams.size() - 1);
}

// Enqueued on the decide stream ahead of the batch's decide stage (no host
// sync): the ExtPacket count stays on the device (k_track_ranges reads it).
// the d* names of the ingest scratch point at set `par` (the last ingest's)
static void IngSetSelect(lkf_engine *e, int par) {
  const lkf_engine::IngSet &g = e->ing[par];
  e->ingPar = par;
  e->dParsed = g.parsed;
  e->dFlows = g.flows;
  e->dFwdFlag = g.fwd;
  e->dITBegin = g.tBegin;
  e->dITEnd = g.tEnd;
  e->dIList = g.list;
  e->dIListCnt = g.listCnt;
  e->dNackInfo = g.nackInfo;
  e->dNackPairOff = g.nackPairOff;
  e->dNackPairCnt = g.nackPairCnt;
  e->dNackPairs = g.nackPairs;
}

static int ingest_common(lkf_engine *e, BatchCtx &x, const lkf_raw_pkt *dRaws, uint32_t n, const uint8_t *dRaw,
                         uint64_t rawLen) {
  const uint32_t nt = uint32_t(e->tracks.size());
  hipStream_t s = e->ingS;
  // the batch's GPU span (lkf_timing_window total) starts before its ingest
  HIPCHK(hipEventRecord(e->ring[e->nRuns % lkf_engine::kRing][0], s), "event");
  e->ingestStarted = true;
  // this ingest's scratch set: the ingest two back used it, and its NACK
  // queues (side stream) and bucket copies (sender stream) read it
  const int par = e->ingPar ^ 1;
  IngSetSelect(e, par);
  if (e->sidePending[par]) HIPCHK(hipStreamWaitEvent(s, e->sideDone[par], 0), "wait nack queues");
  e->sidePending[par] = false;
  if (e->bktPending[par]) HIPCHK(hipStreamWaitEvent(s, e->bktDone[par], 0), "wait bucket copies");
  e->bktPending[par] = false;
  IngestLaunch a;
  a.raws = dRaws;
  a.n = n;
  a.raw = dRaw;
  a.streams = e->dStreams;
  a.nstreams = uint32_t(e->streams.size());
  a.ntracks = nt;
  a.hot = e->dStreamHot;
  a.hist = e->dHist;
  a.rxGap = e->dRxGap;
  a.rings = e->dStreamRings;
  a.parsed = e->dParsed;
  a.tBegin = e->dITBegin;
  a.tEnd = e->dITEnd;
  a.tRuns = e->dITRuns;
  a.err = e->dIErr;
  a.flows = e->dFlows;
  a.fwd = e->dFwdFlag;
  a.twcc = e->dTwcc;
  a.pos = e->dPos;
  a.partA = e->dIPartA;
  a.partB = e->dIPartB;
  a.total = x.dITotal;
  a.out = x.dPktsOwn;
  a.list = e->dIList;
  a.listCnt = e->dIListCnt;
  a.listStride = e->cfg.max_batch_pkts;
  a.nack = e->dNack;
  a.nackInfo = e->dNackInfo;
  a.nackPairOff = e->dNackPairOff;
  a.nackPairCnt = e->dNackPairCnt;
  a.nackPairs = e->dNackPairs;
  a.nackPairCap = e->nackPairCap;
  a.nackIn = e->ing[e->ingPar].nackIn;
  BucketLaunch bl;
  if (e->bktSlots && e->bktStorePending) {  // a second ingest before lkf_run: the first one's copies read this
                                            // context's store list first
    HIPCHK(hipEventRecord(e->bktEv, e->sendS), "event");
    HIPCHK(hipStreamWaitEvent(s, e->bktEv, 0), "wait bucket store");
  }
  if (e->bktSlots) {
    bl.raws = dRaws;
    bl.raw = dRaw;
    bl.n = n;
    bl.streams = e->dStreams;
    bl.nstreams = uint32_t(e->streams.size());
    bl.tBegin = e->dITBegin;
    bl.tEnd = e->dITEnd;
    bl.list = e->dIList;
    bl.listCnt = e->dIListCnt;
    bl.listStride = e->cfg.max_batch_pkts;
    bl.flows = e->dFlows;
    bl.fwd = e->dFwdFlag;
    bl.state = e->dBkt;
    bl.tag = e->dBktTag;
    bl.owner = e->dBktOwner;
    bl.store = x.dBktStore;
    bl.ring = e->dBktRing;
    bl.epoch = ++e->bktEpoch;
    a.bucket = &bl;
  }
  // the forwarding context's preparation for lkf_run (k_ing_out)
  a.fwdPrep.tBegin = x.dTBegin;
  a.fwdPrep.tEnd = x.dTEnd;
  a.fwdPrep.err = x.dErr;
  a.fwdPrep.fwdCnt = x.dFwdCnt;
  a.fwdPrep.stats = x.dStats;
  a.fwdPrep.fwdBytes = x.dFwdBytes;
  a.fwdPrep.nstats = kStatsWords * (1 + kStatCopies);
  a.fwdPrep.ndts = uint32_t(e->dtp.size());
  const bool dd = e->nDDStreams != 0;
  a.ddStates = dd ? e->dDDIng : nullptr;
  a.ddStructs = dd ? e->dDDIngStruct : nullptr;
  a.ingDD = dd ? e->dIngDD : nullptr;
  a.outDD = dd ? x.dDDIn : nullptr;
  {
    bool side = false;
    HIPCHK(launch_ingest(s, a, e->sideS, e->sideFork, e->sideDone[par], &side), "ingest");
    e->sidePending[par] = side;
  }
  if (a.bucket && n) {  // the bucket copies, off the forwarding path: the sender stream (the
                        // batch context counts as done only after it, like the sender statistics)
    HIPCHK(hipEventRecord(e->bktEv, s), "event");
    HIPCHK(hipStreamWaitEvent(e->sendS, e->bktEv, 0), "wait ingest (bucket store)");
    static const bool skipStore = [] {  // (measurement only: LKF_SKIP_BKT_STORE=1 leaves the rings stale)
      const char *v = getenv("LKF_SKIP_BKT_STORE");
      return v && atoi(v) != 0;
    }();
    if (!skipStore) HIPCHK(launch_bucket_store(e->sendS, bl), "bucket store");
    HIPCHK(hipEventRecord(e->bktDone[par], e->sendS), "event");
    e->bktPending[par] = true;
    e->bktStorePending = true;
  }
  HIPCHK(launch_err_fold(s, e->dIErr, e->dSticky, 8), "ingest error fold");
  HIPCHK(hipEventRecord(x.ingested, s), "event");  // the run's preparation (prep stream) waits for it
  x.fromIngest = true;
  x.prepByIngest = n != 0;
  x.prepNT = nt;
  x.prepND = uint32_t(e->dtp.size());
  e->lastIngestN = n;
  e->ingRaws = dRaws;
  e->curPkts = x.dPktsOwn;
  e->curN = n;  // launch bound; the count is x.dITotal
  // (an empty ingest launches nothing, so dITotal still holds an older
  // ingest's count: the batch is empty, with no device-side count)
  e->curNDev = n ? x.dITotal : nullptr;
  e->curDD = a.outDD;  // the ExtPackets' descriptors (nullptr: no DD stream)
  e->curOwned = true;
  e->curDDOwned = true;
  e->curArena = dRaw;
  e->curArenaLen = rawLen;
  e->haveBatch = true;
  return LKF_OK;
}

int lkf_ingest(lkf_engine *e, const lkf_raw_pkt *pkts, uint32_t n, const uint8_t *raw, uint64_t raw_len) {
  if (!e || (n && (!pkts || !raw))) return LKF_EINVAL;
  if (n > e->cfg.max_batch_pkts || raw_len > e->cfg.max_batch_arena) return LKF_ENOSPC;
  int rc = flush_topology(e);
  if (rc) return rc;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  BatchCtx &x = e->ctx[e->nRuns % lkf_engine::kCtx];
  if (x.used) HIPCHK(hipStreamWaitEvent(e->ingS, x.emitted, 0), "wait emit");  // batch n-3 reads these buffers
  if (e->haveBatch && e->curPkts == x.dPktsOwn) {
    // a second ingest into this context before lkf_run: the previous ingest's
    // NACK queues (side stream) and bucket copies (sender stream) still read
    // the datagrams these copies overwrite
    const int lp = e->ingPar;
    if (e->sidePending[lp]) HIPCHK(hipStreamWaitEvent(e->ingS, e->sideDone[lp], 0), "wait nack queues");
    if (e->bktPending[lp]) HIPCHK(hipStreamWaitEvent(e->ingS, e->bktDone[lp], 0), "wait bucket copies");
  }
  if (n) HIPCHK(hipMemcpyAsync(x.dRawPkts, pkts, size_t(n) * sizeof(lkf_raw_pkt), hipMemcpyHostToDevice, e->ingS),
                "raw pkts");
  if (raw_len) HIPCHK(hipMemcpyAsync(x.dArenaOwn, raw, raw_len, hipMemcpyHostToDevice, e->ingS), "raw arena");
  // host buffers are reusable when lkf_ingest returns (the header's contract)
  HIPCHK(hipStreamSynchronize(e->ingS), "ingest copy sync");
  return ingest_common(e, x, x.dRawPkts, n, x.dArenaOwn, raw_len);
}

int lkf_ingest_device(lkf_engine *e, const lkf_raw_pkt *d_pkts, uint32_t n, const uint8_t *d_raw, uint64_t raw_len) {
  if (!e || (n && (!d_pkts || !d_raw))) return LKF_EINVAL;
  if (n > e->cfg.max_batch_pkts) return LKF_ENOSPC;
  const auto t0 = std::chrono::steady_clock::now();
  int rc = flush_topology(e);
  if (rc) return rc;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  BatchCtx &x = e->ctx[e->nRuns % lkf_engine::kCtx];
  if (x.used) HIPCHK(hipStreamWaitEvent(e->ingS, x.emitted, 0), "wait emit");
  rc = ingest_common(e, x, d_pkts, n, d_raw, raw_len);
  if (e->hostProf) {
    e->hp[7] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    e->hp[8] += 1;
  }
  return rc;
}

int lkf_ingest_flows(lkf_engine *e, lkf_flow *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !n_out) return LKF_EINVAL;
  *n_out = e->lastIngestN;
  if (cap < e->lastIngestN) return LKF_ENOSPC;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  HIPCHK(hipStreamSynchronize(e->ingS), "sync");
  if (e->lastIngestN)
    D2H(out, e->dFlows, size_t(e->lastIngestN) * sizeof(lkf_flow), "flows");
  return LKF_OK;
}

int lkf_ingest_twcc(lkf_engine *e, uint32_t *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !n_out) return LKF_EINVAL;
  *n_out = e->lastIngestN;
  if (cap < e->lastIngestN) return LKF_ENOSPC;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  HIPCHK(hipStreamSynchronize(e->ingS), "sync");
  if (e->lastIngestN)
    D2H(out, e->dTwcc, size_t(e->lastIngestN) * sizeof(uint32_t), "twcc");
  return LKF_OK;
}

int lkf_ingested(lkf_engine *e, lkf_pkt *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !n_out) return LKF_EINVAL;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  HIPCHK(hipStreamSynchronize(e->ingS), "sync");
  uint32_t n = 0;
  if (e->haveBatch) {
    n = e->curN;
    if (e->curNDev) {
      uint64_t t = 0;
      D2H(&t, e->curNDev, sizeof(t), "count copy");
      n = uint32_t(t);
    }
  }
  *n_out = n;
  if (cap < n) return LKF_ENOSPC;
  if (n && e->curOwned) D2H(out, e->curPkts, size_t(n) * sizeof(lkf_pkt), "ingested copy");
  if (n && !e->curOwned)  // the caller's device buffer (lkf_submit_device): not an engine allocation
    HIPCHK(hipMemcpy(out, e->curPkts, size_t(n) * sizeof(lkf_pkt), hipMemcpyDeviceToHost), "ingested copy");
  return LKF_OK;
}

int lkf_ingested_dd(lkf_engine *e, lkf_pkt_dd *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !n_out) return LKF_EINVAL;
  uint32_t n = 0;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  HIPCHK(hipStreamSynchronize(e->ingS), "sync");
  if (e->haveBatch) {
    n = e->curN;
    if (e->curNDev) {
      uint64_t t = 0;
      D2H(&t, e->curNDev, sizeof(t), "count copy");
      n = uint32_t(t);
    }
  }
  *n_out = n;
  if (cap < n) return LKF_ENOSPC;
  if (!n) return LKF_OK;
  if (e->curDD && e->curDDOwned)
    D2H(out, e->curDD, size_t(n) * sizeof(lkf_pkt_dd), "ingested dd copy");
  else if (e->curDD)  // the caller's device buffer (lkf_submit_dd_device)
    HIPCHK(hipMemcpy(out, e->curDD, size_t(n) * sizeof(lkf_pkt_dd), hipMemcpyDeviceToHost), "ingested dd copy");
  else
    std::memset(out, 0, size_t(n) * sizeof(lkf_pkt_dd));
  return LKF_OK;
}

int lkf_stream_stats_get(lkf_engine *e, int32_t sid, lkf_stream_stats *o) {
  if (!e || !o || sid < 0 || sid >= int32_t(e->streams.size())) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  StreamHot h;
  D2H(&h, e->dStreamHot + sid, sizeof(h), "stream state copy");
  std::memset(o, 0, sizeof(*o));
  o->initialized = (h.flags & S_INIT) ? 1 : 0;
  o->ext_start_sn = h.snStart;  // WrapAround.GetExtendedStart = ET(start)
  o->ext_highest_sn = h.snExtHighest;
  o->ext_start_ts = h.tsStart;
  o->ext_highest_ts = h.tsExtHighest;
  o->packets_lost = h.packetsLost;
  o->packets_out_of_order = h.packetsOutOfOrder;
  o->packets_duplicate = h.packetsDuplicate;
  o->packets_padding = h.packetsPadding;
  o->bytes = h.bytes;
  o->header_bytes = h.headerBytes;
  o->bytes_duplicate = h.bytesDuplicate;
  o->bytes_padding = h.bytesPadding;
  o->frames = h.frames;
  o->nacks = h.nacks;
  if (e->dNack) {  // (the NACK queues keep the count: see NackState)
    uint64_t nq = 0;
    D2H(&nq, &e->dNack[sid].nacks, sizeof(nq), "stream nacks");
    o->nacks += nq;
  }
  o->first_time_ns = h.firstTime;
  o->highest_time_ns = h.highestTime;
  o->last_transit = h.lastTransit;
  o->last_jitter_ext_ts = h.lastJitterExtTs;
  o->jitter = h.jitter;
  o->max_jitter = h.maxJitter;
  D2H(o->gap_histogram, e->dRxGap + size_t(sid) * kGapWords, kGapBins * sizeof(uint32_t), "stream gap copy");
  return LKF_OK;
}

int lkf_ingest_nacks(lkf_engine *e, lkf_rtcp_nack *out, uint32_t cap, lkf_nack_pair *pairs, uint32_t pair_cap,
                     uint32_t *n_out, uint32_t *n_pairs_out) {
  if (!e || !n_out || !n_pairs_out) return LKF_EINVAL;
  *n_out = *n_pairs_out = 0;
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  if (!e->dNack || !e->lastIngestN) return LKF_OK;
  const uint32_t n = e->lastIngestN;
  hipStream_t ps = e->sideS;  // after the NACK queues of the ingest that produced them (same stream)
  HIPCHK(launch_nack_compact(ps, n, e->ingRaws, e->dStreams, e->dNackInfo, e->dNackPairOff, e->dNackPairs,
                             e->dNackPartA, e->dNackPartB, e->dNackRecPos, e->dNackPairPos, e->dNackTot, e->dNackOut, e->dNackPairsOut),
         "nack compact");
  uint64_t tot[2] = {0, 0};
  CHKRANGE(e->dNackTot, sizeof(tot), "async d2h");
  HIPCHK(hipMemcpyAsync(tot, e->dNackTot, sizeof(tot), hipMemcpyDeviceToHost, ps), "nack totals");
  HIPCHK(hipStreamSynchronize(ps), "nack sync");
  *n_out = uint32_t(tot[0]);
  *n_pairs_out = uint32_t(tot[1]);
  if (tot[0] > cap || tot[1] > pair_cap) return LKF_ENOSPC;
  if (tot[0] && !out) return LKF_EINVAL;
  if (tot[1] && !pairs) return LKF_EINVAL;
  if (tot[0]) D2H(out, e->dNackOut, tot[0] * sizeof(lkf_rtcp_nack), "nack records");
  if (tot[1])
    D2H(pairs, e->dNackPairsOut, tot[1] * sizeof(lkf_nack_pair), "nack pairs");
  return LKF_OK;
}

int lkf_stream_set_rtt(lkf_engine *e, int32_t sid, uint32_t rtt_ms) {
  if (!e || sid < 0 || sid >= int32_t(e->streams.size())) return LKF_EINVAL;
  if (rtt_ms == 0) return LKF_OK;  // Buffer.SetRTT ignores 0
  int rc = flush_topology(e);
  if (rc) return rc;
  if (!e->streams[sid].nack || !e->dNack) return LKF_OK;  // no NackQueue (the rtpStats RTT is out of scope)
  rc = drain_streams(e);  // a queued ingest reads the RTT
  if (rc) return rc;
  e->streams[sid].rtt_ms = rtt_ms;
  HIPCHK(hipMemcpy(&e->dNack[sid].rtt, &rtt_ms, sizeof(rtt_ms), hipMemcpyHostToDevice), "nack rtt");
  return upload_done(e);
}

// Room -> participant -> microphone-stream tables for k_speakers.
static int rebuild_speakers(lkf_engine *e) {
  // primary receiver of a track = its layer-0 stream (first added)
  std::vector<int> primary(e->tracks.size(), -1);
  for (size_t sid = 0; sid < e->streams.size(); sid++) {
    const auto &sp = e->streams[sid];
    if (sp.layer == 0 && primary[sp.track] < 0) primary[sp.track] = int(sid);
  }
  // (room, participant) -> mic streams with an AudioLevel
  std::vector<std::pair<std::pair<uint32_t, uint32_t>, uint32_t>> rows;
  for (size_t t = 0; t < e->tracks.size(); t++) {
    const auto &tp = e->tracks[t];
    if (!tp.is_mic || !e->trackActive[t] || primary[t] < 0 || !e->streams[primary[t]].audio_level_ext) continue;
    rows.push_back({{tp.room, tp.publisher}, uint32_t(primary[t])});
  }
  std::stable_sort(rows.begin(), rows.end(),
                   [](const auto &a, const auto &b) { return a.first < b.first; });
  std::vector<uint32_t> roomOff, roomId, partId, partMicOff, mics;
  for (size_t i = 0; i < rows.size();) {
    const uint32_t room = rows[i].first.first;
    roomId.push_back(room);
    roomOff.push_back(uint32_t(partId.size()));
    while (i < rows.size() && rows[i].first.first == room) {
      const uint32_t part = rows[i].first.second;
      partId.push_back(part);
      partMicOff.push_back(uint32_t(mics.size()));
      while (i < rows.size() && rows[i].first.first == room && rows[i].first.second == part) mics.push_back(rows[i++].second);
    }
    if (partId.size() - roomOff.back() > 64) {
      e->err = "more than 64 microphone participants in a room";
      return LKF_ENOSPC;
    }
  }
  roomOff.push_back(uint32_t(partId.size()));
  partMicOff.push_back(uint32_t(mics.size()));
  e->nRooms = uint32_t(roomId.size());
  e->spkRoomIds = roomId;
  e->topoGen++;
  uint32_t **bufs[] = {&e->dRoomPartOff, &e->dPartId, &e->dPartMicOff, &e->dMics, &e->dRoomId};
  const std::vector<uint32_t> *src[] = {&roomOff, &partId, &partMicOff, &mics, &roomId};
  for (int i = 0; i < 5; i++) {
    if (*bufs[i]) HIPCHK(dfree(*bufs[i]), "free");
    HIPCHK(dalloc(bufs[i], std::max<size_t>(src[i]->size(), 1)), "alloc speakers table");
    if (!src[i]->empty())
      HIPCHK(hipMemcpy(*bufs[i], src[i]->data(), src[i]->size() * sizeof(uint32_t), hipMemcpyHostToDevice),
             "speakers table copy");
  }
  if (e->spkCap < size_t(e->nRooms) * 64) {
    if (e->dSpkSlots) HIPCHK(dfree(e->dSpkSlots), "free");
    if (e->dSpkCounts) HIPCHK(dfree(e->dSpkCounts), "free");
    e->spkCap = std::max<size_t>(size_t(e->nRooms) * 64, 64);
    HIPCHK(dalloc(&e->dSpkSlots, e->spkCap), "alloc slots");
    HIPCHK(dalloc(&e->dSpkCounts, e->spkCap / 64 + 1), "alloc counts");
  }
  e->spkDirty = false;
  return LKF_OK;
}

// The speaker tick without a host wait: the ranking of every room at now_ns
// is enqueued on the prep stream (after the ingest that updated the levels)
// and stays in HBM (the per-room slots an all-gather reads); lkf_speakers
// reads a ranking back.
int lkf_speakers_enqueue(lkf_engine *e, int64_t now_ns) {
  if (!e) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  if (e->spkDirty) {
    rc = drain_streams(e);
    if (rc) return rc;
    rc = rebuild_speakers(e);
    if (rc) return rc;
  }
  if (e->nRooms == 0) return LKF_OK;
  SpeakersLaunch a;
  a.nrooms = e->nRooms;
  a.roomPartOff = e->dRoomPartOff;
  a.partId = e->dPartId;
  a.partMicOff = e->dPartMicOff;
  a.mics = e->dMics;
  a.roomId = e->dRoomId;
  a.streams = e->dStreams;
  a.hot = e->dStreamHot;
  a.nowNs = now_ns;
  a.slots = e->dSpkSlots;
  a.counts = e->dSpkCounts;
  HIPCHK(launch_speakers(e->ingS, a), "speakers");
  return LKF_OK;
}

int lkf_speakers(lkf_engine *e, int64_t now_ns, lkf_speaker *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !n_out) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  if (e->spkDirty) {
    rc = rebuild_speakers(e);
    if (rc) return rc;
  }
  *n_out = 0;
  if (e->nRooms == 0) return LKF_OK;
  SpeakersLaunch a;
  a.nrooms = e->nRooms;
  a.roomPartOff = e->dRoomPartOff;
  a.partId = e->dPartId;
  a.partMicOff = e->dPartMicOff;
  a.mics = e->dMics;
  a.roomId = e->dRoomId;
  a.streams = e->dStreams;
  a.hot = e->dStreamHot;
  a.nowNs = now_ns;
  a.slots = e->dSpkSlots;
  a.counts = e->dSpkCounts;
  // the ingest stream: ordered after the ingest that updated the levels
  HIPCHK(launch_speakers(e->ingS, a), "speakers");
  std::vector<uint32_t> counts(e->nRooms);
  std::vector<lkf_speaker> slots(size_t(e->nRooms) * 64);
  CHKRANGE(e->dSpkCounts, counts.size() * sizeof(uint32_t), "async d2h");
  HIPCHK(hipMemcpyAsync(counts.data(), e->dSpkCounts, counts.size() * sizeof(uint32_t), hipMemcpyDeviceToHost,
                        e->ingS),
         "counts copy");
  CHKRANGE(e->dSpkSlots, slots.size() * sizeof(lkf_speaker), "async d2h");
  HIPCHK(hipMemcpyAsync(slots.data(), e->dSpkSlots, slots.size() * sizeof(lkf_speaker), hipMemcpyDeviceToHost,
                        e->ingS),
         "slots copy");
  HIPCHK(hipStreamSynchronize(e->ingS), "speakers sync");
  uint32_t k = 0;
  for (uint32_t r = 0; r < e->nRooms; r++) k += counts[r];
  *n_out = k;
  if (cap < k) return LKF_ENOSPC;
  k = 0;
  for (uint32_t r = 0; r < e->nRooms; r++)
    for (uint32_t j = 0; j < counts[r]; j++) out[k++] = slots[size_t(r) * 64 + j];
  return LKF_OK;
}

// The room manager's periodic summary without a host wait (see lkfwd.h).
// The ranking and its pack run on the ingest stream after the last enqueued
// ingest; the totals' pack on the decide stream after the last enqueued
// decide (the DownTracks' sendingPacket totals); the caller's stream waits
// for both.  The engine never waits for the caller: the caller keeps `spk` /
// `bwe` unread by earlier work of its own until this tick's writes land
// (bench.py: a ring of buffers, each reused after its gather's event).
int lkf_room_summaries_enqueue(lkf_engine *e, int64_t now_ns, const uint32_t *room_ids, uint32_t rows, int32_t *spk,
                               uint32_t k, int64_t *bwe, uint32_t s, void *stream) {
  if (!e || (rows && !room_ids) || !spk || !bwe || k == 0 || k > 64 || s == 0) return LKF_EINVAL;
  for (uint32_t r = 1; r < rows; r++)
    if (room_ids[r] <= room_ids[r - 1]) return LKF_EINVAL;  // ascending, distinct
  int rc = flush_topology(e);
  if (rc) return rc;
  if (e->spkDirty) {
    rc = drain_streams(e);
    if (rc) return rc;
    rc = rebuild_speakers(e);
    if (rc) return rc;
  }
  HIPCHK(hipSetDevice(e->dev), "hipSetDevice");
  if (!e->rsSpk) {
    HIPCHK(hipEventCreateWithFlags(&e->rsSpk, hipEventDisableTiming), "event");
    HIPCHK(hipEventCreateWithFlags(&e->rsDec, hipEventDisableTiming), "event");
  }
  const uint32_t nd = uint32_t(e->dtp.size());
  if (rows != e->rsRooms.size() || !std::equal(room_ids, room_ids + rows, e->rsRooms.begin()) || k != e->rsK ||
      s != e->rsS || e->topoGen != e->rsGen) {
    std::vector<uint32_t> rooms(room_ids, room_ids + rows);
    auto rowOf = [&](uint32_t room) -> int32_t {
      auto it = std::lower_bound(rooms.begin(), rooms.end(), room);
      return it != rooms.end() && *it == room ? int32_t(it - rooms.begin()) : -1;
    };
    std::vector<int32_t> rowEng(std::max<uint32_t>(rows, 1), -1);
    for (uint32_t r = 0; r < e->nRooms; r++) {
      const int32_t row = rowOf(e->spkRoomIds[r]);
      if (row < 0) {
        e->err = "room_summaries: a room with microphones is not among room_ids";
        return LKF_EINVAL;
      }
      rowEng[row] = int32_t(r);
    }
    // active DownTracks by (row, subscriber, handle); a room's first s subscribers get slots
    std::vector<std::tuple<int32_t, uint32_t, uint32_t>> by;
    for (uint32_t d = 0; d < nd; d++) {
      if (!e->active[d]) continue;
      const int32_t row = rowOf(e->tracks[e->dtp[d].track].room);
      if (row < 0) {
        e->err = "room_summaries: a DownTrack's room is not among room_ids";
        return LKF_EINVAL;
      }
      by.emplace_back(row, e->dtp[d].subscriber, d);
    }
    std::sort(by.begin(), by.end());
    const size_t nslots = size_t(std::max<uint32_t>(rows, 1)) * s;
    std::vector<uint32_t> off(nslots + 1, 0), dts;
    std::vector<int64_t> sub(nslots, -1);
    std::vector<uint32_t> cnt(nslots, 0);
    for (size_t i = 0; i < by.size();) {
      const int32_t row = std::get<0>(by[i]);
      uint32_t pos = 0;
      while (i < by.size() && std::get<0>(by[i]) == row) {
        const uint32_t su = std::get<1>(by[i]);
        size_t j = i;
        while (j < by.size() && std::get<0>(by[j]) == row && std::get<1>(by[j]) == su) j++;
        if (pos < s) {
          const size_t slot = size_t(row) * s + pos;
          sub[slot] = su;
          cnt[slot] = uint32_t(j - i);
        }
        pos++;
        i = j;
      }
    }
    for (size_t q = 0; q < nslots; q++) off[q + 1] = off[q] + cnt[q];
    dts.resize(std::max<uint32_t>(off[nslots], 1));
    {
      std::vector<uint32_t> fillp(off.begin(), off.end() - 1);
      size_t i = 0;
      while (i < by.size()) {
        const int32_t row = std::get<0>(by[i]);
        uint32_t pos = 0;
        while (i < by.size() && std::get<0>(by[i]) == row) {
          const uint32_t su = std::get<1>(by[i]);
          while (i < by.size() && std::get<0>(by[i]) == row && std::get<1>(by[i]) == su) {
            if (pos < s) dts[fillp[size_t(row) * s + pos]++] = std::get<2>(by[i]);
            i++;
          }
          pos++;
        }
      }
    }
    HIPCHK(hipStreamSynchronize(e->ingS), "sync ingest stream");  // (a queued pack may read the old layout)
    HIPCHK(hipStreamSynchronize(e->decS), "sync decide stream");
    for (void *p : {static_cast<void *>(e->dRsRowEng), static_cast<void *>(e->dRsSlotOff),
                    static_cast<void *>(e->dRsSlotDts), static_cast<void *>(e->dRsSlotSub)})
      if (p) HIPCHK(dfree(p), "free");
    HIPCHK(dalloc(&e->dRsRowEng, rowEng.size()), "alloc");
    HIPCHK(dalloc(&e->dRsSlotOff, off.size()), "alloc");
    HIPCHK(dalloc(&e->dRsSlotDts, dts.size()), "alloc");
    HIPCHK(dalloc(&e->dRsSlotSub, sub.size()), "alloc");
    HIPCHK(hipMemcpy(e->dRsRowEng, rowEng.data(), rowEng.size() * 4, hipMemcpyHostToDevice), "copy");
    HIPCHK(hipMemcpy(e->dRsSlotOff, off.data(), off.size() * 4, hipMemcpyHostToDevice), "copy");
    HIPCHK(hipMemcpy(e->dRsSlotDts, dts.data(), dts.size() * 4, hipMemcpyHostToDevice), "copy");
    HIPCHK(hipMemcpy(e->dRsSlotSub, sub.data(), sub.size() * 8, hipMemcpyHostToDevice), "copy");
    e->rsRooms = rooms;
    e->rsK = k;
    e->rsS = s;
    e->rsGen = e->topoGen;
  }
  hipStream_t cs = reinterpret_cast<hipStream_t>(stream);
  if (e->nRooms) {
    SpeakersLaunch a;
    a.nrooms = e->nRooms;
    a.roomPartOff = e->dRoomPartOff;
    a.partId = e->dPartId;
    a.partMicOff = e->dPartMicOff;
    a.mics = e->dMics;
    a.roomId = e->dRoomId;
    a.streams = e->dStreams;
    a.hot = e->dStreamHot;
    a.nowNs = now_ns;
    a.slots = e->dSpkSlots;
    a.counts = e->dSpkCounts;
    HIPCHK(launch_speakers(e->ingS, a), "speakers");
  }
  RoomPackLaunch p;
  p.rows = rows;
  p.k = k;
  p.s = s;
  p.rowEng = e->dRsRowEng;
  p.slots = e->dSpkSlots;
  p.counts = e->dSpkCounts;
  p.slotOff = e->dRsSlotOff;
  p.slotDts = e->dRsSlotDts;
  p.slotSub = e->dRsSlotSub;
  p.cum = e->dDTCum;
  p.spk = spk;
  p.bwe = bwe;
  // the ranking's pack right behind the ranking (ingest stream), the totals'
  // right behind the last enqueued decide: each reads its source before the
  // next ingest / decide on its stream can change it, and nothing of the
  // engine waits for the caller
  HIPCHK(launch_room_pack(e->ingS, e->decS, p), "room pack");
  HIPCHK(hipEventRecord(e->rsSpk, e->ingS), "event");
  HIPCHK(hipEventRecord(e->rsDec, e->decS), "event");
  HIPCHK(hipStreamWaitEvent(cs, e->rsSpk, 0), "wait");
  HIPCHK(hipStreamWaitEvent(cs, e->rsDec, 0), "wait");
  return LKF_OK;
}

// Not part of include/lkfwd.h: the bounds-check record of a checked build
// (-DLKF_CHECKED=1, liblkfwd_checked.so): {violations, first site, index,
// capacity}; LKF_ENODEV from a product build.
// Not part of include/lkfwd.h: the SVC-run stop counters of a diagnostic
// build (-DLKF_SVC_STATS=1; forward_kernels.hip g_svc), after a drain.
int lkf_debug_svc_stats(lkf_engine *e, uint64_t out[48], int reset) {
  if (!e || !out) return LKF_EINVAL;
  int rc = drain_streams(e);
  if (rc) return rc;
  unsigned long long v[48];
  const hipError_t r = read_svc_stats(v, reset);
  for (int i = 0; i < 48; i++) out[i] = v[i];
  return r == hipSuccess ? LKF_OK : LKF_ENODEV;
}

int lkf_debug_check(lkf_engine *e, uint64_t out[4], int reset) {
  if (!out) return LKF_EINVAL;
  if (e) {
    int rc = drain_streams(e);
    if (rc) return rc;
  } else if (hipDeviceSynchronize() != hipSuccess) {  // no engine: the whole device
    return LKF_EHIP;
  }
  unsigned long long v[4];
  hipError_t r = read_check(v, reset);
  for (int i = 0; i < 4; i++) out[i] = v[i];
  // host-side device -> host range violations (CHKRANGE) count as well, in
  // every build; site 0xD2H marks one when the device recorded none
  // an engine's own refusals; with no engine, every engine's
  std::atomic<uint64_t> &ctr = e ? e->rangeViolations : gRangeViolationsAll;
  const uint64_t rv = reset ? ctr.exchange(0) : ctr.load();
  if (rv) {
    if (!out[0]) out[1] = 0xD2, out[2] = 0, out[3] = 0;
    out[0] += rv;
    return LKF_OK;
  }
  return r == hipSuccess ? LKF_OK : LKF_ENODEV;
}

// Not part of include/lkfwd.h: every batch context's DD arena and spill bump
// cursors (out[2c], out[2c+1]) after a drain, and the arena's capacity
// (out[6]); LKF_EINVAL before the DD tables exist.  tests/test_dd_recapture_gpu.py
// checks them after graph re-captures forced under queued runs.
int lkf_debug_dd_cursors(lkf_engine *e, uint64_t out[7]) {
  if (!e || !out || !e->ddAlloc) return LKF_EINVAL;
  int rc = drain_streams(e);
  if (rc) return rc;
  for (int c = 0; c < lkf_engine::kCtx; c++) {
    uint64_t u[2] = {0, 0};
    D2H(u, e->ctx[c].dDDUsed, sizeof(u), "dd cursor copy");
    out[2 * c] = u[0];
    out[2 * c + 1] = u[1] & 0xffffffffu;
  }
  out[6] = e->ddArenaCap;
  return LKF_OK;
}

// Not part of include/lkfwd.h: a DD DownTrack's selector state for debugging
// (out[16]: cache init, base, last, masks[8], chain broken bits, chain active
// bits, frames the unbroken chains wait on, frame-number wrapper last, current layers
// spatial | temporal << 8 (+128 each)).
int lkf_debug_dd_state(lkf_engine *e, int32_t dt, uint64_t out[16]) {
  if (!e || !out || dt < 0 || size_t(dt) >= e->dtp.size() || !e->dDDState) return LKF_EINVAL;
  int rc = drain_streams(e);
  if (rc) return rc;
  DDState d;
  DTHot h;
  D2H(&d, e->dDDState + dt, sizeof(d), "dd state");
  D2H(&h, e->dHot + dt, sizeof(h), "hot state");
  out[0] = (d.flags & DS_CACHE_INIT) ? 1 : 0;
  out[1] = d.cBase;
  out[2] = d.cLast;
  for (int i = 0; i < 8; i++) out[3 + i] = d.masks[i];
  const uint32_t cm = d.numChains >= 32 ? ~0u : (1u << d.numChains) - 1;
  out[11] = d.chBroken & cm;
  out[12] = d.chActive & cm;
  uint64_t ex = 0;
  for (int c = 0; c < d.numChains; c++) {  // (the set's size: the ring's bits and the frame beyond it)
    if ((d.chBroken >> c) & 1) continue;    // (a broken chain's set is inert until it is cleared)
    ex += d.expFar[c] ? 1 : 0;
    for (int w = 0; w < kDDExpWords; w++) ex += uint64_t(__builtin_popcountll(d.exp[c][w]));
  }
  out[13] = ex;
  out[14] = (d.flags & DS_FN_INIT) ? d.fnLast : ~0ull;
  out[15] = uint64_t(uint8_t(h.curS + 128)) | (uint64_t(uint8_t(h.curT + 128)) << 8);
  return LKF_OK;
}

int lkf_downtrack_summaries(lkf_engine *e, lkf_dt_summary *out, uint32_t cap, uint32_t *n_out) {
  if (!e || !n_out) return LKF_EINVAL;
  const uint32_t nd = uint32_t(e->dtp.size());
  *n_out = nd;
  if (cap < nd) return LKF_ENOSPC;
  if (!nd) return LKF_OK;
  if (!out) return LKF_EINVAL;
  int rc = flush_topology(e);
  if (rc) return rc;
  rc = drain_streams(e);
  if (rc) return rc;
  std::vector<DTCum> c(nd);
  D2H(c.data(), e->dDTCum, nd * sizeof(DTCum), "dt totals copy");
  for (uint32_t d = 0; d < nd; d++) {
    lkf_dt_summary &s = out[d];
    s.dt = int32_t(d);
    s.subscriber = e->dtp[d].subscriber;
    s.room = e->tracks[e->dtp[d].track].room;
    s.flags = (e->active[d] ? LKF_DTS_ACTIVE : 0u) | ((c[d].flags & F_DEFICIENT) ? LKF_DTS_DEFICIENT : 0u);
    s.packets_sent = c[d].packets;
    s.bytes_sent = c[d].bytes;
  }
  return LKF_OK;
}

int lkf_get_cumulative(lkf_engine *e, lkf_stats *out, int reset) {
  if (!e || !out) return LKF_EINVAL;
  int rc = drain_streams(e);
  if (rc) return rc;
  uint64_t st[kStatsWords];
  D2H(st, e->dCum, sizeof(st), "cum copy");
  out->tuples = st[0];
  out->forwarded = st[1];
  out->out_bytes = st[2];
  out->arena_bytes = st[3];
  for (int i = 0; i < LKF_DROP_NREASONS; i++) out->drops[i] = st[4 + i];
  if (reset) {
    HIPCHK(hipMemset(e->dCum, 0, sizeof(st)), "cum reset");
    HIPCHK(hipDeviceSynchronize(), "cum reset sync");  // before the next run's k_accumulate (emit stream)
  }
  return LKF_OK;
}

}  // extern "C"
