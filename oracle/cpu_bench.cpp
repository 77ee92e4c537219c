// cpu_bench.cpp — the CPU baseline driver of bench.py (TEST INFRASTRUCTURE:
// only bench.py's cpu_baseline leg calls it; the product path never does).
//
// the reference Go path cannot run here or on the GPU box,
// so the CPU baseline is the oracle (this directory's scalar C++ restatement
// of the Go forwarding path) timed on the host cores: one oracle engine per
// thread, each forwarding its own shard of rooms (no shared state), every
// thread started by one barrier; the timed region is the batches' control ops
// (orc_ctl_batch), Buffer.calc (orc_ingest, with `ingress`) and the forwarding
// (orc_run) — the same step bench.py times on the GPU.  Driving the shards
// from C++ threads keeps Python (the GIL, ctypes marshalling) out of the
// measurement.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <map>
#include <vector>

#include "../include/lkfwd.h"

extern "C" {
struct orc_engine;
orc_engine *orc_create(uint32_t seq_size);
void orc_destroy(orc_engine *e);
int32_t orc_add_track(orc_engine *e, const lkf_track_params *p);
int32_t orc_add_downtrack(orc_engine *e, const lkf_downtrack_params *p);
int32_t orc_add_stream(orc_engine *e, const lkf_stream_params *p);
int orc_ctl_batch(orc_engine *e, const lkf_ctl_event *evs, uint32_t n);
int orc_submit_dd(orc_engine *e, const lkf_pkt_dd *dd, uint32_t n);
int orc_run(orc_engine *e, const lkf_pkt *pkts, uint32_t n, const uint8_t *arena, uint64_t arena_len);
int orc_get_stats(orc_engine *e, lkf_stats *out);
int orc_ingest(orc_engine *e, const lkf_raw_pkt *pkts, uint32_t n, const uint8_t *raw, uint64_t raw_len);
int orc_ingested_ptr(orc_engine *e, const lkf_pkt **pkts, uint32_t *n);
int orc_get_state(orc_engine *e, int32_t dt, lkf_fwd_state *o);
int orc_sender_stats_get(orc_engine *e, int32_t dt, lkf_sender_stats *o);
int orc_stream_stats_get(orc_engine *e, int32_t s, lkf_stream_stats *o);

// one batch of a shard (pointers into the synthetic trace)
typedef struct orc_bench_batch {
  const lkf_pkt *pkts;
  uint32_t n;
  uint32_t nraw;
  const uint8_t *arena;
  uint64_t alen;
  const lkf_pkt_dd *dd;     // nullptr: no DD side array
  const lkf_raw_pkt *raws;  // the same batch as datagrams (ingress)
  const lkf_ctl_event *ev;
  uint32_t nev;
  uint32_t pad;
} orc_bench_batch;

typedef struct orc_bench_shard {
  const lkf_track_params *tracks;
  const lkf_downtrack_params *dts;
  const lkf_stream_params *streams;
  const orc_bench_batch *batches;
  uint32_t ntracks, ndts, nstreams, nbatches;
} orc_bench_shard;

// per shard, after its last batch (the engine still alive): nullptr, or a
// callback that reads its state out
struct ShardDone {
  virtual void done(uint32_t shard, orc_engine *e, const lkf_stats &cum) = 0;
};
static int drive(const orc_bench_shard *shards, uint32_t nshards, uint32_t nthreads, int ingress, uint32_t seq_size,
                 uint64_t *forwarded, double *busy_s, double *wall_s, ShardDone *after);

int orc_cpu_bench(const orc_bench_shard *shards, uint32_t nshards, uint32_t nthreads, int ingress,
                  uint32_t seq_size, uint64_t *forwarded, double *busy_s, double *wall_s) {
  return drive(shards, nshards, nthreads, ingress, seq_size, forwarded, busy_s, wall_s, nullptr);
}

// bench.py's parity gate (outside its timed region): the same shards run to
// the end, then per shard its cumulative counters (cum[shard]) and, per
// DownTrack, {ssrc, subscriber, lkf_fwd_state, lkf_sender_stats} (dtRecs, shards' DownTracks
// in order, stride dtStride bytes) and per stream {ssrc, lkf_stream_stats}
// (stRecs, stride stStride; ingress only).  SSRCs key the records to the GPU
// engine's DownTracks and streams (a room shard keeps its rooms' SSRCs).
int orc_parity_run(const orc_bench_shard *shards, uint32_t nshards, uint32_t nthreads, int ingress,
                   uint32_t seq_size, lkf_stats *cum, uint8_t *dtRecs, uint64_t dtStride, uint8_t *stRecs,
                   uint64_t stStride) {
  struct Reader : ShardDone {
    const orc_bench_shard *sh;
    uint32_t n;
    lkf_stats *cum;
    uint8_t *dt, *st;
    uint64_t dtStride, stStride;
    int rc = 0;
    void done(uint32_t i, orc_engine *e, const lkf_stats &c) override {
      uint64_t d0 = 0, s0 = 0;
      for (uint32_t k = 0; k < i; k++) {
        d0 += sh[k].ndts;
        s0 += sh[k].nstreams;
      }
      cum[i] = c;
      // key: (room, the DownTrack's ordinal among its room's DownTracks) — one
      // per DownTrack (random SSRCs of different rooms can collide), the same
      // ordinal a single trace of those rooms gives it (rooms generate alike)
      std::map<uint32_t, uint32_t> ordOf;
      for (uint32_t d = 0; d < sh[i].ndts; d++) {
        uint8_t *r = dt + (d0 + d) * dtStride;
        const uint32_t room = sh[i].tracks[sh[i].dts[d].track].room;
        const uint32_t ord = ordOf[room]++;
        std::memcpy(r, &room, 4);
        std::memcpy(r + 4, &ord, 4);
        lkf_fwd_state fs{};
        lkf_sender_stats ss{};
        if (orc_get_state(e, int32_t(d), &fs) || orc_sender_stats_get(e, int32_t(d), &ss)) rc = -1;
        std::memcpy(r + 8, &fs, sizeof(fs));
        std::memcpy(r + 8 + sizeof(fs), &ss, sizeof(ss));
      }
      if (st)
        for (uint32_t k = 0; k < sh[i].nstreams; k++) {
          uint8_t *r = st + (s0 + k) * stStride;
          std::memcpy(r, &sh[i].streams[k].ssrc, 4);
          std::memcpy(r + 4, &sh[i].tracks[sh[i].streams[k].track].room, 4);  // (keyed by room and SSRC)
          lkf_stream_stats ts{};
          if (orc_stream_stats_get(e, int32_t(k), &ts)) rc = -1;
          std::memcpy(r + 8, &ts, sizeof(ts));
        }
    }
  } rd;
  rd.sh = shards;
  rd.n = nshards;
  rd.cum = cum;
  rd.dt = dtRecs;
  rd.st = ingress ? stRecs : nullptr;
  rd.dtStride = dtStride;
  rd.stStride = stStride;
  if (dtStride < 8 + sizeof(lkf_fwd_state) + sizeof(lkf_sender_stats) ||
      (rd.st && stStride < 8 + sizeof(lkf_stream_stats)))
    return -22;
  std::vector<uint64_t> fwd(nshards);
  double wall = 0;
  const int r = drive(shards, nshards, nthreads, ingress, seq_size, fwd.data(), nullptr, &wall, &rd);
  return r ? r : rd.rc;
}

// Runs the shards on `nthreads` threads: every shard's engine is built
// first (tracks, DownTracks, streams: untimed), then all threads start at one
// barrier and pull shards from a shared counter, each shard's batches in
// order on the thread that took it (dynamic balancing: rooms differ in work —
// mutes, layer switches, loss — so a static split leaves threads idle while
// the slowest finishes).  forwarded[i] = shard i's forwarded tuples, *wall_s =
// seconds from the common start to the last thread's end, busy_s[t] = thread
// t's own timed seconds (nullptr: not wanted).  0, or the first non-zero
// return code of an oracle call.
static int drive(const orc_bench_shard *shards, uint32_t nshards, uint32_t nthreads, int ingress, uint32_t seq_size,
                 uint64_t *forwarded, double *busy_s, double *wall_s, ShardDone *after) {
  if (nthreads == 0) nthreads = 1;
  std::vector<orc_engine *> eng(nshards, nullptr);
  std::atomic<int> rc{0};
  std::atomic<uint32_t> built{0}, next{0}, ready{0};
  std::atomic<bool> go{false};
  using clk = std::chrono::steady_clock;
  std::vector<std::thread> th;
  clk::time_point t0;
  auto build = [&](uint32_t i) {
    const orc_bench_shard &s = shards[i];
    orc_engine *e = orc_create(seq_size);
    eng[i] = e;
    int r = 0;
    for (uint32_t t = 0; t < s.ntracks && !r; t++) r = orc_add_track(e, &s.tracks[t]) == int32_t(t) ? 0 : -1;
    for (uint32_t d = 0; d < s.ndts && !r; d++) r = orc_add_downtrack(e, &s.dts[d]) == int32_t(d) ? 0 : -1;
    if (ingress && s.streams)
      for (uint32_t k = 0; k < s.nstreams && !r; k++) r = orc_add_stream(e, &s.streams[k]) == int32_t(k) ? 0 : -1;
    if (r) rc = r;
  };
  auto forward = [&](uint32_t i) {
    const orc_bench_shard &s = shards[i];
    orc_engine *e = eng[i];
    uint64_t fwd = 0;
    lkf_stats cum{};
    int r = 0;
    for (uint32_t b = 0; b < s.nbatches && !r; b++) {
      const orc_bench_batch &x = s.batches[b];
      if (x.nev) r = orc_ctl_batch(e, x.ev, x.nev);
      if (r) break;
      if (ingress && x.raws) {
        r = orc_ingest(e, x.raws, x.nraw, x.arena, x.alen);
        const lkf_pkt *p = nullptr;
        uint32_t n = 0;
        if (!r) r = orc_ingested_ptr(e, &p, &n);
        if (!r) r = orc_run(e, p, n, x.arena, x.alen);
      } else {
        if (x.dd) r = orc_submit_dd(e, x.dd, x.n);
        if (!r) r = orc_run(e, x.pkts, x.n, x.arena, x.alen);
      }
      lkf_stats st{};
      if (!r) r = orc_get_stats(e, &st);
      fwd += st.forwarded;
      if (after) {
        cum.tuples += st.tuples;
        cum.forwarded += st.forwarded;
        cum.out_bytes += st.out_bytes;
        cum.arena_bytes += st.arena_bytes;
        for (int k = 0; k < LKF_DROP_NREASONS; k++) cum.drops[k] += st.drops[k];
      }
    }
    forwarded[i] = fwd;
    if (after && !r) after->done(i, e, cum);
    if (r) rc = r;
  };
  for (uint32_t t = 0; t < nthreads; t++)
    th.emplace_back([&, t]() {
      for (uint32_t i; (i = built.fetch_add(1)) < nshards;) build(i);  // (untimed)
      ready++;
      while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
      const clk::time_point a = clk::now();
      for (uint32_t i; (i = next.fetch_add(1)) < nshards;) forward(i);
      if (busy_s) busy_s[t] = std::chrono::duration<double>(clk::now() - a).count();
    });
  while (ready.load() < nthreads) std::this_thread::yield();
  t0 = clk::now();
  go.store(true, std::memory_order_release);
  for (auto &t : th) t.join();
  *wall_s = std::chrono::duration<double>(clk::now() - t0).count();
  for (orc_engine *e : eng)
    if (e) orc_destroy(e);
  return rc.load();
}
}
