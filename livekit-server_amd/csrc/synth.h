/*
 * synth.h — deterministic synthetic RTP workloads for the BASELINE.json
 * configs.  Seeded splitmix64 (seed = 0x4C4B + config).
 *
 * Produces the topology (lkf_track_params / lkf_downtrack_params), the
 * ExtPacket batches (lkf_pkt + raw RTP arena, grouped by track, arrival order
 * within a track) and the scripted control events — the same inputs for the
 * MI355X engine and for the CPU oracle.  Data only: no forwarding logic.
 */
#ifndef LKF_SYNTH_H_
#define LKF_SYNTH_H_

#include <stdint.h>

#include "../../include/lkfwd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lkfs_cfg {
  int32_t config;        /* 1..4 (BASELINE.json configs[config-1]) */
  uint64_t seed;         /* 0 -> 0x4C4B + config */
  double duration_s;     /* media time (default 10 s) */
  double batch_s;        /* batch window of media time (default 1 s) */
  uint32_t rooms;        /* 0 -> config default */
  uint32_t participants; /* per room (publishers for cfg 4: subscribers) 0 -> default */
  uint32_t room_base;    /* first room index (room sharding across ranks) */
  double loss;           /* -1 -> config default */
  double reorder;        /* -1 -> config default */
  int32_t with_events;   /* -1 -> default (1) */
  int32_t has_callbacks; /* -1 -> default (1): has_ref_ts / has_expected_ts */
  int32_t svc_dd;        /* config 5: -1 -> default (1): AV1 + VP9 publishers with the dependency
                            descriptor beside VP9-descriptor ones; 0: VP9 descriptor only; 2: as 1
                            with the wide descriptor (9 chains, 17-18 frame diffs); 3: as 1 with
                            chain 0 over every frame and bursts of every other frame lost (chains
                            waiting on dozens of frames) */
  int32_t h264;          /* configs 1-3: 1 -> H.264 simulcast publishers (config 1: the publisher;
                            else every third) with SPS key frames as single NALU / STAP-A / STAP-B /
                            FU-A; <= 0 -> VP8 only */
  int32_t twcc;          /* send-side BWE: 1 -> every second subscriber's video DownTracks negotiate
                            transport-cc (id 5) instead of abs-send-time; 2 -> all of them; 0 -> none */
  const uint32_t *room_ids; /* non-null: generate rooms room_ids[0..rooms) (a bin-packed shard)
                               instead of room_base + [0, rooms) */
} lkfs_cfg;

typedef struct lkfs_event {
  int32_t dt;
  int32_t op;
  int64_t a[4];
  uint32_t at_pkt; /* batch-relative packet index */
  uint32_t pad;
} lkfs_event;

typedef struct lkfs_trace lkfs_trace;

lkfs_trace *lkfs_generate(const lkfs_cfg *cfg);
void lkfs_free(lkfs_trace *t);

uint32_t lkfs_num_tracks(const lkfs_trace *t);
uint32_t lkfs_num_downtracks(const lkfs_trace *t);
const lkf_track_params *lkfs_tracks(const lkfs_trace *t);
const lkf_downtrack_params *lkfs_downtracks(const lkfs_trace *t);

uint32_t lkfs_num_batches(const lkfs_trace *t);
/* Batch b: descriptors (track handles = index into lkfs_tracks) and arena. */
int lkfs_batch(const lkfs_trace *t, uint32_t b, const lkf_pkt **pkts, uint32_t *n, const uint8_t **arena,
               uint64_t *arena_len);
int lkfs_batch_events(const lkfs_trace *t, uint32_t b, const lkfs_event **ev, uint32_t *n);
/* Batch b's lkf_pkt_dd side array (parallel to lkfs_batch; meaningful for
 * LKF_PKT_DD packets): what the ingress DependencyDescriptorParser reports for
 * the generated stream (extended frame numbers, the structure's frame, updates,
 * frame integrity in arrival order). */
int lkfs_batch_dd(const lkfs_trace *t, uint32_t b, const lkf_pkt_dd **dd, uint32_t *n);
/* Totals over the whole trace. */
uint64_t lkfs_total_pkts(const lkfs_trace *t);
uint64_t lkfs_total_arena(const lkfs_trace *t);
uint32_t lkfs_max_batch_pkts(const lkfs_trace *t);
uint64_t lkfs_max_batch_arena(const lkfs_trace *t);
/* max over batches of sum over DownTracks of their track's packets */
uint64_t lkfs_max_batch_tuples(const lkfs_trace *t);
/* max over batches of the output arena if every tuple were forwarded */
uint64_t lkfs_max_batch_out_bytes(const lkfs_trace *t);
/* Ingress view: one stream per received SSRC, and batch b as raw datagrams
 * (the same packets as lkfs_batch, offsets into the same arena). */
uint32_t lkfs_num_streams(const lkfs_trace *t);
const lkf_stream_params *lkfs_streams(const lkfs_trace *t);
int lkfs_batch_raw(const lkfs_trace *t, uint32_t b, const lkf_raw_pkt **raws, uint32_t *n);

#ifdef __cplusplus
}
#endif
#endif
