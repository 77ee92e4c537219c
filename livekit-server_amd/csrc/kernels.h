// kernels.h — launch interface between the host engine (engine.cpp) and the
// gfx950 kernels (forward_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/lkfwd.h"
#include "fwd_state.h"

namespace lkf {

struct DecideLaunch {
  const uint32_t *sched;    // wave -> DownTrack (per-XCD interleaved schedule)
  const uint32_t *waveTrack;
  uint32_t nlanes;          // waves
  uint32_t ddLanes;         // the last ddLanes waves: DownTracks of the DD selector (k_decide_dt<true>)
  uint32_t perWave;         // DownTracks per wave (1..64; 0 = 1)
  DTHot *hot;
  const DevDT *dts;
  const DevTrack *tracks;
  RangeEntry *rm;
  VP8Cold *vc;
  SeqMeta *seq;
  uint32_t seqSize;
  uint8_t *srm;  // SeqRM regions (the sequencer RangeMaps of padding exclusions)
  uint64_t srmStride;
  uint32_t srmCap;
  const lkf_pkt *pkts;
  const uint32_t *tBegin, *tEnd;
  const uint64_t *slotBase;
  FwdRec *recs;     // forwarded records at slotBase[dt] + j
  FwdBase *fbase;   // per DownTrack: the base of its records' 32-bit SN / TS
  FwdBase *wide;    // per tuple slot: the full SN / TS of a T_WIDE record
  uint64_t tupleCap;
  uint32_t *err;
  SenderStats *ss;  // RTPStatsSender per DownTrack, updated by decide (snInfo ring, gap histogram)
  uint32_t *ssRing, *ssGap;
  uint32_t *dtOffs;  // per DownTrack kDTOffsWords: the reference-layer offsets its Forwarder reads
  const DevEvent *events;
  const uint32_t *evOff;
  uint32_t *fwdCnt;
  uint64_t *fwdBytes;
  DTCum *dtCum;
  uint64_t *stats;
  const uint32_t *layerList, *layerBefore, *layerCnt;  // launch_layer_index outputs
  uint32_t pktStride;                                  // max_batch_pkts
  // dependency descriptor (nullptr when no track uses the DD selector)
  const DDPkt *ddPkts;
  const DDStruct *ddStructs;
  DDState *ddState;
  uint8_t *ddArena;
  uint64_t *ddUsed;
  uint64_t ddCap;
  const uint16_t *ddSpill;  // k_dd_decode's spilled frame-diff lists
  // capacities (tested in -DLKF_CHECKED=1 builds)
  uint32_t maxDts, maxTracks, npkts, nev;
};

struct EmitLaunch {
  const uint32_t *perm;  // output position -> DownTrack
  const uint64_t *recBase, *byteBase, *slotBase, *totals;  // recBase/byteBase by position
  const uint32_t *gFirst;  // [group] position owning record 64*group (k_scan_down mode 1)
  const FwdRec *recs;
  const FwdBase *fbase;
  const FwdBase *wide;
  const lkf_pkt *pkts;
  const uint8_t *arena;
  const DevDT *dts;
  uint32_t ndts;
  lkf_out *out;
  uint8_t *outArena;
  uint64_t outCap, outByteCap;
  uint32_t *err;
  uint32_t grid;
  const uint8_t *ddArena;  // non-null: batches with DD tracks (k_emit<PRE_MAX_DD>)
  const uint32_t *twccBase = nullptr;  // per DownTrack transport-cc base of the batch (DownTracks with extTcc)
  uint32_t ldsPad = 0;  // dynamic LDS reserved per workgroup (caps residency; the plain instantiation)
  // capacities (tested in -DLKF_CHECKED=1 builds)
  uint32_t maxDts, npkts;
  uint64_t tupleCap, arenaLen, ddCap, gCap;
};
// transport-wide sequence numbers (pion TWCC header-extension interceptor):
// the batch's base per DownTrack after decide, and the stamping of control-rate
// packets (padding / blank: recs + recOff + cnt; RTX: rtx + off + len)
hipError_t launch_twcc_base(hipStream_t s, const DevDT *dts, uint32_t ndts, const uint32_t *fwdCnt, uint32_t *ctrD,
                            uint32_t *ctrT, const uint32_t *tOff, const uint32_t *tList, uint32_t ntr,
                            uint32_t *base);
hipError_t launch_twcc_stamp(hipStream_t s, const DevDT *dts, uint32_t *ctrD, uint32_t *ctrT, uint32_t n,
                             const lkf_out *recs, const uint64_t *recOff, const uint32_t *cnt, const lkf_rtx *rtx,
                             const uint64_t *off, const uint32_t *len, uint8_t *arena);
// -DLKF_CHECKED=1 builds: {violations, first site, its index, its capacity}
hipError_t read_check(unsigned long long out[4], int reset);
hipError_t read_svc_stats(unsigned long long out[48], int reset);  // LKF_SVC_STATS builds

hipError_t launch_batch_init(hipStream_t s, uint32_t ntracks, uint32_t ndts, uint32_t nstats, uint32_t *tBegin,
                             uint32_t *tEnd, uint32_t *tRuns, uint32_t *err, uint64_t *stats, uint32_t *fwdCnt,
                             uint64_t *fwdBytes);
hipError_t launch_track_ranges(hipStream_t s, const RunDesc *desc, uint32_t maxPkts, uint32_t ntracks,
                               uint32_t *tBegin, uint32_t *tEnd, uint32_t *tRuns, uint32_t *err);
// the scan's state (partA): scan_state_words(maxN) u64 words, zeroed at allocation
// (each launch leaves it zeroed); partB is unused
size_t scan_state_words(uint32_t maxN);
hipError_t launch_scan(hipStream_t s, int mode, const DevDT *dts, const uint32_t *tBegin, const uint32_t *tEnd,
                       const uint32_t *cnt, const uint64_t *bytes, uint32_t n, uint64_t *partA, uint64_t *partB,
                       uint64_t *outA, uint64_t *outB, uint64_t *totA, uint64_t *totB,
                       const uint32_t *perm, uint32_t *gFirst = nullptr, uint64_t gCap = 0);
struct BucketLaunch;
// What a NACK queue reads of one datagram of its stream's list, written by the
// stream kernel in list order ([layer slot * listStride + tBegin + j], like the
// list): the NACK kernel's loads are then contiguous instead of one scattered
// line per datagram in each of the raw, parsed and flow arrays.
struct NackIn {
  int64_t arrival;  // lkf_raw_pkt.arrival_ns
  uint32_t stream;  // lkf_raw_pkt.stream (a list may hold another stream's datagrams)
  uint32_t snFl;    // RTP SN | (2: parsed (updateStreamState ran), 4: a loss range) << 16
  uint32_t s0, len; // the loss range's first SN and length (flow loss_start, loss_end - loss_start)
};
static_assert(sizeof(NackIn) == 24, "24 B per datagram");
// The NACK kernel's lane-parallel form: at most this many nack events per
// stream and ingest, so at most this many RTCP NACK pairs; each stream writes
// them to its own block past the shared pair buffer (nackPairCap + stream *
// kNackFastPairs), the serial form bump-allocates in the shared part.
constexpr uint32_t kNackFastPairs = 256;
struct IngestLaunch {
  const lkf_raw_pkt *raws;
  uint32_t n;
  const uint8_t *raw;
  const DevStream *streams;
  uint32_t nstreams, ntracks;
  StreamHot *hot;
  uint64_t *hist;
  uint32_t *rxGap;  // per stream RTPStatsReceiver gap histogram (kGapWords)
  RangeEntry *rings;
  IngParsed *parsed;
  uint32_t *tBegin, *tEnd, *tRuns, *err;
  lkf_flow *flows;
  uint32_t *fwd;
  uint32_t *twcc;  // per datagram: TWCC responder push word (LKF_TWCC_*)
  uint64_t *pos, *partA, *partB, *total;
  lkf_pkt *out;
  // dependency descriptor (nullptr: no stream negotiated the DD extension)
  DDIngState *ddStates;
  DDStruct *ddStructs;  // two per DD stream
  IngDD *ingDD;         // per datagram
  lkf_pkt_dd *outDD;    // the batch's side array
  // per-stream datagram lists (k_ing_lists): [layer slot * listStride + tBegin + j], counts [track * 3 + slot]
  uint32_t *list, *listCnt;
  uint32_t listStride;
  // NACK queues (nullptr: no stream has one): per stream state, per datagram
  // result (n_pairs | num_nacked << 16, 0: no RTCP NACK) and pair offset in
  // the bump-allocated pair buffer
  NackState *nack;
  uint32_t *nackInfo, *nackPairOff, *nackPairCnt;
  lkf_nack_pair *nackPairs;
  uint32_t nackPairCap;
  NackIn *nackIn;  // 3 * listStride records (nullptr: the NACK kernel reads the raw arrays)
  const BucketLaunch *bucket = nullptr;  // the RTX buckets (nullptr: none)
  // the forwarding batch context's preparation, done by k_ing_out (tBegin
  // nullptr: not done): per-track ExtPacket ranges from the ingest's datagram
  // ranges and positions, and the zeroing k_batch_init would do (lkf_run then
  // skips k_batch_init and k_track_ranges)
  struct {
    uint32_t *tBegin = nullptr, *tEnd = nullptr, *err = nullptr, *fwdCnt = nullptr;
    uint64_t *stats = nullptr, *fwdBytes = nullptr;
    uint32_t nstats = 0, ndts = 0;
  } fwdPrep;
};
// The receivers' RTX buckets (mediatransportutil bucket, buffer.go:471; oracle
// bucket_oracle.h): per stream a ring of maxSteps slots of kBktSlot bytes (the
// packet at +16), its logical state (size << 16 | stored SN; size 0xFFFF =
// invalid) in tag, the last writer of a slot in owner (ingest epoch << 32 |
// datagram), and per datagram of the batch what to store (valid << 63 |
// adjusted SN << 32 | slot; 0: nothing — not stored, or a later datagram of
// the batch took the slot).  k_bkt_store reads only that and the datagrams, so
// it runs off the forwarding path (the sender stream) while the next batches
// are ingested and decided.
constexpr uint32_t kBktSlot = 1536;
struct BucketState {  // 16 B
  uint32_t base;      // first slot of the stream's ring
  uint32_t maxSteps;  // 200 (audio) / PacketBufferSize (video)
  uint32_t step;
  uint16_t head;
  uint8_t init, pad;
};
struct BucketLaunch {
  const lkf_raw_pkt *raws;
  const uint8_t *raw;
  uint32_t n;
  const DevStream *streams;
  uint32_t nstreams;
  const uint32_t *tBegin, *tEnd, *list, *listCnt;
  uint32_t listStride;
  lkf_flow *flows;
  uint32_t *fwd;
  BucketState *state;
  uint32_t *tag;
  uint64_t *owner;
  uint64_t *store;  // per datagram of this batch (its context's array)
  uint8_t *ring;
  uint32_t epoch;   // this ingest's number (from 1)
};
// the bucket arrays k_ing_stream_wave decides AddPacketWithSequenceNumber on
// (state nullptr: no buckets)
struct BktArgs {
  BucketState *state;
  uint32_t *tag;
  uint64_t *owner;
  uint64_t *store;
  uint32_t epoch;
};
hipError_t launch_bucket_store(hipStream_t s, const BucketLaunch &a);
// Bucket.GetPacket for RTX records: stream[i] (-1: no buffer / closed) and the
// source SN; the packet is gathered to out + i * kBktSlot and src[i] = (that
// offset, its length, its header size in reserved) or len 0
hipError_t launch_bucket_read(hipStream_t s, uint32_t n, const int32_t *stream, const uint16_t *sn,
                              const BucketState *state, const uint32_t *tag, const uint8_t *ring, uint8_t *out,
                              lkf_raw_pkt *src);

// lkf_ingest_nacks: the last ingest's RTCP NACKs compacted in datagram order
hipError_t launch_nack_compact(hipStream_t s, uint32_t n, const lkf_raw_pkt *raws, const DevStream *streams,
                               const uint32_t *info, const uint32_t *pairOff, const lkf_nack_pair *pairs,
                               uint64_t *partA, uint64_t *partB, uint64_t *recPos, uint64_t *pairPos, uint64_t *totals,
                               lkf_rtcp_nack *outRecs, lkf_nack_pair *outPairs);

struct SpeakersLaunch {
  uint32_t nrooms;
  const uint32_t *roomPartOff, *partId, *partMicOff, *mics, *roomId;
  const DevStream *streams;
  StreamHot *hot;
  int64_t nowNs;
  lkf_speaker *slots;
  uint32_t *counts;
};

// the ingest chain on s; with NACK queues k_ing_nack forks onto `side` after the
// stream kernel (*sideUsed: sideDone was recorded there)
hipError_t launch_ingest(hipStream_t s, const IngestLaunch &a, hipStream_t side, hipEvent_t sideFork,
                         hipEvent_t sideDone, bool *sideUsed);
hipError_t launch_speakers(hipStream_t s, const SpeakersLaunch &a);
// The room manager's fixed-shape summary records (lkf_room_summaries_enqueue):
// row r of spk [rows, k, 3] = the ranking slots of engine room rowEng[r];
// slot i of bwe [rows, s, 5] = the DownTracks slotDts[slotOff[i] .. slotOff[i+1]).
struct RoomPackLaunch {
  uint32_t rows, k, s;
  const int32_t *rowEng;  // row -> engine speaker room (-1: no microphones)
  const lkf_speaker *slots;
  const uint32_t *counts;
  const uint32_t *slotOff, *slotDts;
  const int64_t *slotSub;  // subscriber of a slot (-1 padding)
  const DTCum *cum;
  int32_t *spk;
  int64_t *bwe;
};
// (the ranking's pack on spkStream, the totals' pack on bweStream)
hipError_t launch_room_pack(hipStream_t spkStream, hipStream_t bweStream, const RoomPackLaunch &a);
hipError_t launch_decide(hipStream_t s, const DecideLaunch &a);
hipError_t launch_layer_index(hipStream_t s, const RunDesc *desc, const uint32_t *tBegin, const uint32_t *tEnd,
                              uint32_t ntracks, uint32_t stride, uint32_t *list, uint32_t *before, uint32_t *cnt,
                              uint64_t *zero2 = nullptr);
hipError_t launch_emit(hipStream_t s, const EmitLaunch &a);
hipError_t launch_dd_decode(hipStream_t s, const RunDesc *desc, const uint32_t *tBegin, const uint32_t *tEnd,
                            const DevTrack *tracks, uint32_t ntracks, DDStruct *structs, DDTrack *ddTracks, DDPkt *out,
                            uint32_t *err, const uint32_t *trackDDTrk, DDTrkState *ddTrk, uint16_t *spill,
                            uint32_t *spillUsed, uint32_t spillCap);
// the DD stream trackers' bitrate report (tracker_kernels.hip)
hipError_t launch_dd_tracker_tick(hipStream_t s, DDTrkState *st, const int32_t *ids, uint32_t n, int64_t elapsedNs,
                                  lkf_dd_tracker_status *out);
hipError_t launch_h2d(hipStream_t s, const uint8_t *stage, RunDesc *dDesc, DevEvent *dEv, uint32_t *dLane);
hipError_t launch_stats_reduce(hipStream_t s, uint64_t *stats);
// dense per-lane op offsets from the lane-sorted op list: off[l] = first op with lane >= l
hipError_t launch_ev_offsets(hipStream_t s, const uint32_t *laneOf, const RunDesc *desc, uint32_t nl, uint32_t *off);
hipError_t launch_accumulate(hipStream_t s, const uint64_t *stats, const uint64_t *tot, uint64_t *cum,
                             const uint32_t *err, uint32_t *sticky);
hipError_t launch_err_fold(hipStream_t s, const uint32_t *err, uint32_t *sticky, uint32_t shift);
hipError_t launch_rtx_lookup(hipStream_t s, const DTHot *hot, SeqMeta *seq, uint32_t seqSize, uint8_t *srm,
                             uint64_t srmStride, uint32_t srmCap, const lkf_nack *nacks,
                             const uint32_t *gStart, uint32_t ngroups, int64_t nowMs, lkf_rtx *out, uint32_t *valid);
hipError_t launch_rtx_emit(hipStream_t s, bool write, uint32_t n, const lkf_rtx *rtx, const lkf_raw_pkt *src,
                           const uint8_t *arena, const DevDT *dts, const DevTrack *tracks, uint32_t *lens,
                           const uint64_t *offs, uint8_t *out, const uint8_t *dd);
// ---- SRTP protect (srtp_kernels.hip) ----
struct SrtpKeys {  // one transport's session (RFC 3711 AES_CM_128_HMAC_SHA1_80)
  uint32_t rk[44];   // AES-128 schedule of the session key (big-endian words)
  uint32_t ih[5];    // SHA-1 state after the HMAC ipad block
  uint32_t oh[5];    // ... after the opad block
  uint32_t salt[4];  // 14-byte session salt, big-endian words, low 16 bits zero
  uint32_t profile;
  uint32_t pad[5];
};
static_assert(sizeof(SrtpKeys) == 256, "SrtpKeys is 256 B");
struct SrtpDT {       // per DownTrack (SSRC)
  uint32_t tp1;       // transport + 1 (0: none)
  uint32_t init;      // rollover base fixed
  uint64_t rocBase;   // (ext SN of the first protected packet) >> 16
};
struct SrtpProtectArgs {
  const uint32_t *tab;  // AES te[256] + S-box
  const uint64_t *totals;  // [0] = records of the batch
  const lkf_out *out;
  const uint8_t *arena;
  uint8_t *prot;
  const DevDT *dts;
  SrtpDT *sd;  // (k_srtp_roc fixes rollover bases; k_srtp_protect reads)
  const SrtpKeys *keys;
  uint64_t cap;      // record capacity (grid bound)
  uint32_t absVal;   // abs-send-time, 24 bits
};
hipError_t launch_aes_tables(hipStream_t s, uint32_t *tab);
hipError_t launch_srtp_keys(hipStream_t s, const lkf_transport_params *in, uint32_t first, uint32_t n,
                            const uint32_t *tab, SrtpKeys *keys);
hipError_t launch_srtp_protect(hipStream_t s, const SrtpProtectArgs &a, uint32_t ndts, const uint32_t *perm,
                               const uint64_t *recBase, const uint32_t *fwdCnt);

hipError_t launch_seq_lookup(hipStream_t s, DTHot *hot, SeqMeta *seq, uint32_t seqSize, uint8_t *srm,
                             uint64_t srmStride, uint32_t srmCap, uint32_t d,
                             const uint16_t *sns, uint32_t n, int64_t nowMs, lkf_seq_meta *out, uint32_t *nOut);

// ---- padding / blank frames (WritePaddingRTP, writeBlankFrameRTP) ----
struct PadLaunch {
  int blank;  // 0: WritePaddingRTP requests, 1: one writeBlankFrameRTP tick per request
  uint32_t n;
  const lkf_pad_req *reqs;
  int64_t nowNs;
  DTHot *hot;
  const DevDT *dts;
  const DevTrack *tracks;
  RangeEntry *rm;
  SeqMeta *seq;
  uint32_t seqSize;
  uint8_t *srm;
  uint64_t srmStride;
  uint32_t srmCap;
  DTCum *dtCum;
  const uint64_t *recOff, *byteOff;  // per request: first reserved record / arena byte
  lkf_out *out;
  uint8_t *arena;
  uint32_t *cnt;    // per request: packets written
  uint32_t *bytes;  // per request: WritePaddingRTP's return value (blank: bytes counted by sendingPacket)
};
hipError_t launch_pad(hipStream_t s, const PadLaunch &a);
// allocation control kernels (alloc_kernels.hip); `last` is the stored
// lastAllocation per DownTrack; `out` is lkf_allocation[n] or, for
// ALLOC_TRANSITION, lkf_video_transition[n]; `capacity` only for NEXT_HIGHER
enum AllocMode { ALLOC_OPTIMAL = 0, ALLOC_NEXT_HIGHER = 1, ALLOC_TRANSITION = 2, ALLOC_PAUSE = 3 };
// the cooperative pass (alloc_kernels.hip k_prov / k_allocate_all)
enum ProvMode { PROV_PREPARE = 0, PROV_RESET, PROV_ALLOCATE, PROV_COOPERATIVE, PROV_BEST_WEIGHTED, PROV_COMMIT };
struct ProvLaunch {
  int mode;
  uint32_t n;
  const lkf_prov_req *reqs;   // (PROV_PREPARE: alloc)
  const lkf_alloc_req *alloc;
  DTHot *hot;
  const DevDT *dts;
  const DevTrack *tracks;
  lkf_allocation *last;
  ProvState *prov;
  void *out;  // lkf_prov_result / lkf_video_transition / lkf_allocation per request
};
hipError_t launch_prov(hipStream_t s, const ProvLaunch &a);
hipError_t launch_allocate_all(hipStream_t s, const lkf_alloc_group *groups, uint32_t ngroups, const lkf_alloc_req *reqs,
                               DTHot *hot, const DevDT *dts, const DevTrack *tracks, lkf_allocation *last,
                               ProvState *prov, lkf_allocation *out);
hipError_t launch_allocate(hipStream_t s, int mode, const lkf_alloc_req *reqs, const int64_t *capacity, uint32_t n,
                           DTHot *hot, const DevDT *dts, const DevTrack *tracks, lkf_allocation *last, void *out);

// ---- RED for Opus (red_kernels.hip) ----
struct RedEncState {  // RedReceiver.pktBuff (redreceiver.go:45): the last two primaries of a track
  uint8_t has[2];
  uint16_t sn[2];
  uint32_t ts[2];
  uint16_t len[2];
  uint8_t pay[2][1500];
};
struct RedDecState {  // RedPrimaryReceiver (redprimaryreceiver.go:37-48)
  uint8_t first, hist;
  uint16_t lastSeq;
};
struct RedLaunch {
  const lkf_pkt *in;
  const uint8_t *inArena;
  const uint32_t *gBegin, *gEnd;  // per mapped track of the batch: its packet range
  uint32_t ngroups;
  const int32_t *map;             // source track -> destination track
  RedEncState *enc;
  RedDecState *dec;
  const uint64_t *recOff, *byteOff;  // per input packet: reserved output records / arena bytes
  lkf_pkt *out;
  uint8_t *outArena;
  uint32_t *cnt;  // per input packet: packets written
};
hipError_t launch_red(hipStream_t s, bool decode, const RedLaunch &a);

// ---- stream trackers (tracker_kernels.hip) ----
struct TrackerState {  // StreamTracker + StreamTrackerPacket of one (track, spatial layer)
  uint32_t track;
  int32_t layer;
  uint32_t samples, cycles;  // SamplesRequired, CyclesRequired
  uint32_t countSinceLast, cycleCount, notifications;
  uint8_t initialized, paused, stopped, workerLive, status, lastNotified, bitrateChanged, pad;
  int64_t bytes[4];    // bytesForBitrate
  int64_t bitrate[4];
  // StreamTrackerFrame (streamtracker_frame.go:39-211) when `frame`
  uint8_t frame, tsInit, lastCheckSet, pad2;
  uint32_t clockRate, oldestTS, newestTS;
  int32_t numFrames, pad3;
  double minFPS, estFps;
  int64_t evalIntervalNs, lastCheckNs;  // virtual clock
};
// StreamTrackerFrame.resetFPSCalculator + updateEvalInterval (host and device)
__host__ __device__ inline void tracker_frame_eval_interval(TrackerState &t) {
  t.evalIntervalNs = 500000000;  // checkInterval
  if (t.estFps > 0.0) {
    const int64_t iv = int64_t(1e9 / t.estFps);
    if (iv > t.evalIntervalNs) t.evalIntervalNs = iv;
  }
  if (t.minFPS > 0.0) {
    const int64_t iv = int64_t(1e9 / t.minFPS);
    if (iv > t.evalIntervalNs) t.evalIntervalNs = iv;
  }
}
__host__ __device__ inline void tracker_frame_reset_fps(TrackerState &t) {
  t.tsInit = 0;
  t.oldestTS = t.newestTS = 0;
  t.numFrames = 0;
  t.estFps = 0.0;
  tracker_frame_eval_interval(t);
}
hipError_t launch_tracker_observe(hipStream_t s, TrackerState *st, uint32_t n, const RunDesc *desc,
                                  const uint32_t *tBegin, const uint32_t *tEnd);
hipError_t launch_tracker_tick(hipStream_t s, TrackerState *st, const int32_t *ids, uint32_t n, int check,
                               int64_t elapsedNs, int64_t nowNs, lkf_tracker_status *out);

// ---- sequencer ddBytes (forward_kernels.hip k_seq_dd, ingress_kernels.hip k_rtx_dd)
struct SeqDDLaunch {
  const uint32_t *list;  // DownTracks with a DD entry ring
  uint32_t n;
  const DTHot *hot;
  const SeqMeta *seq;
  uint32_t seqSize;
  uint8_t *srm;
  uint64_t srmStride;
  uint32_t srmCap;
  const uint32_t *ddIdx;  // DownTrack -> ring index
  uint8_t *seqDD;         // [ring index][slot] kSeqDDBytes
  const FwdRec *recs;
  const FwdBase *fbase;
  const FwdBase *wide;
  const uint64_t *slotBase;
  const uint32_t *fwdCnt;
  const lkf_pkt *pkts;
  const uint8_t *ddArena;
};
hipError_t launch_seq_dd(hipStream_t s, const SeqDDLaunch &a);
// per lkf_rtx record: the DD bytes of its sequencer slot (still holding its
// target SN) staged at dd + 256 * i (length byte first); 0 length otherwise
hipError_t launch_rtx_dd(hipStream_t s, uint32_t n, const lkf_rtx *rtx, const DevDT *dts, const SeqMeta *seq,
                         uint32_t seqSize, const uint32_t *ddIdx, const uint8_t *seqDD, uint8_t *dd);

// ---- DownTrack sender statistics (sender_kernels.hip) ------------------------
struct SenderUpd {  // one host-listed sendingPacket (padding, blank frame, RTX)
  uint64_t esn, ets;
  int64_t t;
  uint32_t dt;
  uint16_t hdr, pay, pad;
  uint8_t marker, rsv;
};
struct SenderListLaunch {
  const SenderUpd *list;   // grouped by DownTrack, call order within a group
  const uint32_t *gBegin;  // ngroups + 1
  uint32_t ngroups;
  SenderStats *ss;
  uint32_t *ring;
  uint32_t *gap;
};
hipError_t launch_sender_updates(hipStream_t s, const SenderListLaunch &a);

}  // namespace lkf
