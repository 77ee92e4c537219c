"""bench.py — forwarded RTP packets/s of the MI355X forwarding engine.

Default workload (the headline): BASELINE.json configs[1] = 100 rooms x 10
participants, VP8 3-layer simulcast + Opus per participant, each subscribing
to the other 9 (18,000 DownTracks), 2% loss, 1% reorder, target-layer switches
every 2 s per DownTrack, subscriber mutes.  Synthetic (seeded splitmix64).
One step = one batch = 1 s of media time of all 100 rooms through the full
per-packet path (Forwarder/RTPMunger/VP8 munger/sequencer + wire-packet
emission), inputs resident in HBM.  Multi-GPU: one process per GPU, each rank
forwards its own 100 rooms (room sharding, no data-path collective) -> weak
scaling.

--config N times BASELINE.json configs[N-1] instead (per GPU):
  1  1 room x 10 participants (the reference's CPU-runnable case)
  3  125 rooms x 50 participants, audio-heavy (1,000 rooms over 8 GPUs):
     raw datagrams -> Buffer.calc (audio levels, NACK queues) -> forward,
     plus the speaker ranking tick every step (lkf_speakers_enqueue)
  4  10 rooms x 1 publisher x 5,000 subscribers (payload-copy bound)
  5  2,000 rooms x 5 participants, VP9/AV1 SVC with dependency descriptors
     + Opus DTX, congestion-driven layer drops (the serial SVC decide path)

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes as C
import importlib
import glob
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def algorithmic_bytes(trace, batches, fwd, out_bytes, active_dts, ingress=False):
    """sum_in (64 + in_payload) + sum_fwd (out_len + 32) + sum_active_DT 256 per batch.
    With the ingress stage (Buffer.calc in the step), per raw datagram its
    24-B descriptor and bytes read once and a 40-B flow record written, plus
    each stored packet's bytes written into its RTX bucket (counted as the
    ExtPackets' header + payload: every ExtPacket was stored, padding not
    counted — a lower bound).  -> (B, forward-stage input bytes, ingress bytes)"""
    import numpy as np
    b_in = b_ing = 0
    for b in batches:
        pk, n, _, _ = trace.batch(b)
        arr = np.ctypeslib.as_array(C.cast(pk, C.POINTER(C.c_uint8)), shape=(n * 64,)).view(
            np.dtype([("x", "V36"), ("payload_off", "<u2"), ("payload_len", "<u2"), ("y", "V24")]))
        pl = int(arr["payload_len"].astype(np.int64).sum())
        b_in += 64 * n + pl
        if ingress:
            rp, nraw, _, _ = trace.batch_raw(b)
            raw = np.ctypeslib.as_array(C.cast(rp, C.POINTER(C.c_uint8)), shape=(nraw * 24,)).view(
                np.dtype([("t", "<i8"), ("s", "<u4"), ("off", "<u4"), ("len", "<u4"), ("r", "<u4")]))
            b_ing += (24 + 40) * nraw + int(raw["len"].astype(np.int64).sum())
            b_ing += pl + int(arr["payload_off"].astype(np.int64).sum())
    return b_in + b_ing + out_bytes + 32 * fwd + 256 * active_dts * len(batches), b_in, b_ing


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# per config: default rooms per GPU, CPU-baseline sample rooms (about 10-30 s
# of oracle work on 16 host threads), one-thread sample rooms
CONFIGS = {
    1: dict(rooms=1, sample=1, sample1=1),
    2: dict(rooms=100, sample=256, sample1=32),
    3: dict(rooms=125, sample=64, sample1=8),
    4: dict(rooms=10, sample=2, sample1=1),
    5: dict(rooms=2000, sample=2048, sample1=256),
}


def workload_name(config, rooms, ndts):
    return {
        1: "configs[0]: 1 room x 10 participants, VP8 3-layer simulcast + Opus, %d DownTracks, no loss" % ndts,
        2: "configs[1]: %d rooms x 10 participants per GPU, VP8 3-layer simulcast + Opus, %d DownTracks, 2%% loss, "
           "1%% reorder, layer switching" % (rooms, ndts),
        3: "configs[2]: %d rooms x 50 participants per GPU (1,000 rooms over 8 GPUs), Opus + 5 VP8 publishers per "
           "room, %d DownTracks, speaker ranking every step" % (rooms, ndts),
        4: "configs[3]: %d rooms x 1 publisher x 5,000 subscribers per GPU (webinar), %d DownTracks" % (rooms, ndts),
        5: "configs[4]: %d rooms x 5 participants per GPU, VP9/AV1 L3T3 SVC with dependency descriptors + Opus "
           "DTX, %d DownTracks, congestion-driven layer drops" % (rooms, ndts),
    }[config]


class _BenchBatch(C.Structure):  # oracle/cpu_bench.cpp orc_bench_batch
    _fields_ = [("pkts", C.c_void_p), ("n", C.c_uint32), ("nraw", C.c_uint32), ("arena", C.c_void_p),
                ("alen", C.c_uint64), ("dd", C.c_void_p), ("raws", C.c_void_p), ("ev", C.c_void_p),
                ("nev", C.c_uint32), ("pad", C.c_uint32)]


class _BenchShard(C.Structure):  # oracle/cpu_bench.cpp orc_bench_shard
    _fields_ = [("tracks", C.c_void_p), ("dts", C.c_void_p), ("streams", C.c_void_p), ("batches", C.c_void_p),
                ("ntracks", C.c_uint32), ("ndts", C.c_uint32), ("nstreams", C.c_uint32), ("nbatches", C.c_uint32)]


def _dt_subset_shard(tr, b_events, keep):
    """A shard of one trace holding only DownTracks `keep` (all its tracks and
    streams): the DownTrack parameters and each batch's control ops (dt
    re-indexed, ops of other DownTracks dropped)."""
    abi = importlib.import_module("livekit-server_amd.abi")
    dts = (type(tr.downtracks[0]) * len(keep))(*[tr.downtracks[d] for d in keep])
    where = {d: i for i, d in enumerate(keep)}
    evs = []
    for ev, nev in b_events:
        sel = [ev[i] for i in range(nev) if ev[i].dt in where]
        arr = (abi.lkfs_event * max(1, len(sel)))()
        for i, x in enumerate(sel):
            arr[i] = x
            arr[i].dt = where[x.dt]
        evs.append((arr, len(sel)))
    return dts, evs


def cpu_baseline(threads, sample_rooms=256, sample_batches=4, config=2, ingress=False):
    """CPU oracle (C++ restatement of the Go path, -O3) on a bounded sample of
    the same workload: `sample_rooms` rooms of the config's shape,
    `sample_batches` one-second batches, in shards of a few rooms (one oracle
    engine each) that `threads` C++ threads pull from a shared counter
    (oracle/cpu_bench.cpp; no Python in the timed region).  With `ingress`
    each batch goes through Buffer.calc (orc_ingest) first, as the GPU step
    does.  When the rooms are too few to keep the threads busy and their
    tracks fan out to 20 or more DownTracks, each room's DownTracks are split
    over several engines as well: the reference writes such a track's
    DownTracks in parallel (DownTrackSpreader.Broadcast -> utils.ParallelExec
    with the receiver's load-balance threshold 20, downtrackspreader.go:89-102,
    rtc/mediatrack.go:257); the room's Buffer.calc runs once, on the first of
    them, and the others forward the ExtPackets it produces (as the reference
    calculates once per packet and then fans out).  Returns
    (forwarded/s, wall s, rooms, batches, per-thread busy s, engines)."""
    from tests.oracle_lib import load as load_oracle
    wl = importlib.import_module("livekit-server_amd.workload")
    o = load_oracle()
    threads = max(1, threads)
    per = max(1, sample_rooms // (threads * 8))  # about 8 shards per thread
    nrs = max(1, sample_rooms // per)
    traces = []
    for t in range(nrs):
        traces.append(wl.Trace(config, duration_s=float(sample_batches), batch_s=1.0, rooms=per, room_base=t * per))
        if ingress:
            wl.events_at_batch_start(traces[-1])
    fan = max(int(np.bincount([traces[0].downtracks[d].track for d in range(traces[0].ndts)]).max()), 0)
    split = 1
    if nrs < threads * 4 and fan >= 20:  # DownTrackSpreader's parallel fan-out
        split = -(-threads * 4 // nrs)
    units = [(tr, k) for tr in traces for k in range(split)]
    # Buffer.calc runs once per room: the first engine of a split room ingests
    # (timed), the others forward the ExtPackets that ingest produces (made
    # here, untimed, by one more oracle engine per room)
    pre = {}
    if ingress and split > 1:
        fptr = o.lib.orc_ingested_ptr
        fptr.restype, fptr.argtypes = C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint32)]
        for tr in traces:
            h = o.create(500)
            wl.load_topology(o.api, h, tr)
            wl.load_streams(o.api, h, tr)
            lst = []
            for b in range(tr.nbatches):
                rp, nraw, ar, alen = tr.batch_raw(b)
                assert o.api["ingest"](h, rp, nraw, ar, alen) == 0
                p_, m_ = C.c_void_p(), C.c_uint32()
                assert fptr(h, C.byref(p_), C.byref(m_)) == 0
                lst.append((np.frombuffer(C.string_at(p_, max(1, m_.value) * 64), dtype=np.uint8).copy(), m_.value))
            o.destroy(h)
            pre[id(tr)] = lst
    shards, keep = (_BenchShard * len(units))(), []
    for i, (tr, k) in enumerate(units):
        bevs = [wl.events_ptr(tr, b) for b in range(tr.nbatches)]
        if split > 1:
            sel = [d for d in range(tr.ndts) if d % split == k]
            dts, bevs = _dt_subset_shard(tr, bevs, sel)
            keep.append((dts, bevs))
            ndts = len(sel)
        else:
            dts, ndts = tr.downtracks, tr.ndts
        bb = (_BenchBatch * tr.nbatches)()
        dd = tr.has_dd() and not ingress
        for b in range(tr.nbatches):
            pk, n, ar, alen = tr.batch(b)
            ev, nev = bevs[b]
            x = bb[b]
            x.pkts, x.n, x.arena, x.alen = C.cast(pk, C.c_void_p), n, C.cast(ar, C.c_void_p), alen
            x.ev, x.nev = C.cast(ev, C.c_void_p), nev
            x.dd = C.cast(tr.batch_dd(b)[0], C.c_void_p) if dd else None
            if ingress and k == 0:
                rp, nraw, _, _ = tr.batch_raw(b)
                x.raws, x.nraw = C.cast(rp, C.c_void_p), nraw
            elif ingress:  # a split room's other engines: the room's ExtPackets, no Buffer.calc of their own
                arr, m_ = pre[id(tr)][b]
                x.pkts, x.n, x.raws, x.nraw = C.c_void_p(arr.ctypes.data), m_, None, 0
        keep.append(bb)
        sh = shards[i]
        sh.tracks, sh.dts = C.cast(tr.tracks, C.c_void_p), C.cast(dts, C.c_void_p)
        sh.streams = C.cast(tr.streams, C.c_void_p) if ingress and k == 0 else None
        sh.batches = C.cast(bb, C.c_void_p)
        sh.ntracks, sh.ndts, sh.nstreams, sh.nbatches = tr.ntracks, ndts, (tr.nstreams if ingress else 0), tr.nbatches
    nsh = len(units)
    threads = min(threads, nsh)
    fwd = (C.c_uint64 * nsh)()
    busy = (C.c_double * threads)()
    wall = C.c_double()
    o.lib.orc_cpu_bench.restype = C.c_int
    o.lib.orc_cpu_bench.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_void_p, C.c_void_p,
                                    C.c_void_p]
    rc = o.lib.orc_cpu_bench(C.cast(shards, C.c_void_p), nsh, threads, 1 if ingress else 0, 500,
                             C.cast(fwd, C.c_void_p), C.cast(busy, C.c_void_p), C.byref(wall))
    assert rc == 0, rc
    nb = traces[0].nbatches
    for tr in traces:
        tr.close()
    return sum(fwd) / wall.value, wall.value, per * nrs, nb, list(busy), nsh


def parity_gate(eng, pkg, config, room_ids, nb, batch_s, ingress, trace, threads, warm_cum, timed_cum):
    """The parity gate (timing is reported only for bit-exact
    output), outside the timed region: the CPU oracle runs the same rooms and
    the same `nb` batches as the GPU did (shards of rooms on `threads` C++
    threads, oracle/cpu_bench.cpp orc_parity_run), then
      - the cumulative counters over all nb batches (tuples, forwarded, bytes,
        arena bytes, every drop reason),
      - every DownTrack's exported Forwarder state and RTPStatsSender,
      - every stream's RTPStatsReceiver (with the ingress step)
    must be identical, DownTracks keyed by (room, ordinal among the room's
    DownTracks) and streams by (SSRC, room), matched one to one (a room shard
    generates its rooms exactly as the full trace does).  -> dict (parity:
    bool + what was compared)."""
    from tests.oracle_lib import load as load_oracle
    wl = importlib.import_module("livekit-server_amd.workload")
    abi = pkg.abi
    o = load_oracle()
    t0 = time.perf_counter()
    per = max(1, len(room_ids) // (threads * 4))
    chunks = [room_ids[i:i + per] for i in range(0, len(room_ids), per)]
    traces, keep, shards = [], [], (_BenchShard * len(chunks))()
    for t, rids in enumerate(chunks):
        tr = wl.Trace(config, duration_s=nb * batch_s, batch_s=batch_s, room_ids=rids)
        if ingress:
            wl.events_at_batch_start(tr)  # (as the GPU's trace)
        traces.append(tr)
        bb = (_BenchBatch * nb)()
        dd = tr.has_dd() and not ingress
        for b in range(nb):
            pk, n, ar, alen = tr.batch(b)
            ev, nev = wl.events_ptr(tr, b)
            x = bb[b]
            x.pkts, x.n, x.arena, x.alen = C.cast(pk, C.c_void_p), n, C.cast(ar, C.c_void_p), alen
            x.ev, x.nev = C.cast(ev, C.c_void_p), nev
            x.dd = C.cast(tr.batch_dd(b)[0], C.c_void_p) if dd else None
            if ingress:
                rp, nraw, _, _ = tr.batch_raw(b)
                x.raws, x.nraw = C.cast(rp, C.c_void_p), nraw
        keep.append(bb)
        sh = shards[t]
        sh.tracks, sh.dts = C.cast(tr.tracks, C.c_void_p), C.cast(tr.downtracks, C.c_void_p)
        sh.streams = C.cast(tr.streams, C.c_void_p) if ingress else None
        sh.batches = C.cast(bb, C.c_void_p)
        sh.ntracks, sh.ndts, sh.nstreams, sh.nbatches = tr.ntracks, tr.ndts, (tr.nstreams if ingress else 0), nb
    ndts = sum(tr.ndts for tr in traces)
    nst = sum(tr.nstreams for tr in traces) if ingress else 0
    fs_sz, ss_sz, st_sz = C.sizeof(abi.lkf_fwd_state), abi.SENDER_STATS_DTYPE.itemsize, C.sizeof(abi.lkf_stream_stats)
    dstride = (8 + fs_sz + ss_sz + 7) & ~7
    sstride = (8 + st_sz + 7) & ~7
    drec = np.zeros(max(1, ndts) * dstride, dtype=np.uint8)
    srec = np.zeros(max(1, nst) * sstride, dtype=np.uint8)
    cum = (abi.lkf_stats * len(chunks))()
    f = o.lib.orc_parity_run
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64,
                  C.c_void_p, C.c_uint64]
    rc = f(C.cast(shards, C.c_void_p), len(chunks), threads, 1 if ingress else 0, 500, C.cast(cum, C.c_void_p),
           drec.ctypes.data, dstride, srec.ctypes.data, sstride)
    for tr in traces:
        tr.close()
    res = {"parity": False, "oracle_rc": rc}
    if rc != 0:
        return res
    # cumulative counters
    ocum = {"tuples": 0, "forwarded": 0, "out_bytes": 0, "arena_bytes": 0, "drops": [0] * abi.LKF_DROP_NREASONS}
    for c in cum:
        d = c.as_dict()
        for k in ("tuples", "forwarded", "out_bytes", "arena_bytes"):
            ocum[k] += d[k]
        ocum["drops"] = [a + b for a, b in zip(ocum["drops"], d["drops"])]
    gcum = {k: warm_cum[k] + timed_cum[k] for k in ("tuples", "forwarded", "out_bytes", "arena_bytes")}
    gcum["drops"] = [a + b for a, b in zip(warm_cum["drops"], timed_cum["drops"])]
    ok_cum = gcum == ocum
    # per DownTrack, keyed by (room, ordinal among its room's DownTracks): one
    # oracle record per GPU DownTrack, matched 1:1 (a key seen twice fails)
    orc = {}
    dup_keys = 0
    for i in range(ndts):
        r = drec[i * dstride:(i + 1) * dstride]
        k = tuple(int(x) for x in r[:8].view(np.uint32))
        if k in orc:
            dup_keys += 1
        orc[k] = r
    bad_dt = 0
    examples = []
    st = abi.lkf_fwd_state()
    ss = np.zeros(1, dtype=abi.SENDER_STATS_DTYPE)
    ord_of = {}
    for d in range(trace.ndts):
        room = int(trace.tracks[trace.downtracks[d].track].room)
        key = (room, ord_of.get(room, 0))
        ord_of[room] = key[1] + 1
        r = orc.pop(key, None)
        if r is None or eng.api["get_state"](eng.h, d, C.byref(st)) != 0 or \
                eng.api["sender_stats_get"](eng.h, d, ss.ctypes.data) != 0:
            bad_dt += 1
            continue
        ost = abi.lkf_fwd_state.from_buffer_copy(bytes(r[8:8 + fs_sz]))
        oss = np.frombuffer(bytes(r[8 + fs_sz:8 + fs_sz + ss_sz]), dtype=abi.SENDER_STATS_DTYPE)
        if not (st.as_tuple() == ost.as_tuple() and all(np.array_equal(ss[k], oss[k]) for k in ss.dtype.names)):
            bad_dt += 1
            if len(examples) < 4:  # what differs (GPU, oracle), for the record
                fd = {n: (getattr(st, n), getattr(ost, n)) for n, *_ in abi.lkf_fwd_state._fields_
                      if not isinstance(getattr(st, n), C.Array) and getattr(st, n) != getattr(ost, n)}
                sd = {k: (ss[k].tolist(), oss[k].tolist()) for k in ss.dtype.names if not np.array_equal(ss[k], oss[k])}
                examples.append({"dt": d, "track": int(trace.downtracks[d].track), "fwd_state": fd,
                                 "sender_stats": {k: v for k, v in list(sd.items())[:6]}})
    bad_dt += len(orc)  # oracle DownTracks no GPU DownTrack matched
    # per stream (by SSRC): RTPStatsReceiver
    bad_st = 0
    if ingress:
        ors = {}
        for i in range(nst):  # keyed by (SSRC, room)
            r = srec[i * sstride:(i + 1) * sstride]
            k = tuple(int(x) for x in r[:8].view(np.uint32))
            if k in ors:
                dup_keys += 1
            ors[k] = r
        for s_ in range(trace.nstreams):
            r = ors.get((int(trace.streams[s_].ssrc), int(trace.tracks[trace.streams[s_].track].room)))
            if r is None or pkg.stream_stats(eng.api, eng.h, s_) != \
                    abi.lkf_stream_stats.from_buffer_copy(bytes(r[8:8 + st_sz])).as_tuple():
                bad_st += 1
    res.update({"parity": bool(ok_cum and bad_dt == 0 and bad_st == 0 and ndts == trace.ndts and dup_keys == 0),
                "counters_equal": ok_cum, "downtracks_checked": trace.ndts, "downtracks_differing": bad_dt,
                "streams_checked": trace.nstreams if ingress else 0, "streams_differing": bad_st,
                "batches": nb, "forwarded_total": gcum["forwarded"], "oracle_threads": threads,
                "keys_not_unique": dup_keys, "key": "(room, ordinal in room) per DownTrack, (SSRC, room) per stream",
                "gate_s": round(time.perf_counter() - t0, 1)})
    if not ok_cum:
        res["counters_gpu_oracle"] = {k: (gcum[k], ocum[k]) for k in gcum if gcum[k] != ocum[k]}
    if examples:
        res["differing_examples"] = examples
    return res


def launch_ranks(n):
    """`bench.py --gpus N` without a torch.distributed launcher: start N fresh
    child processes of this script, one per GPU, with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (the same environment
    `torch.distributed.run --nproc-per-node N` gives them).  The parent never
    touches the GPU: it only waits.  Rank 0 prints the JSON line.  A failing
    rank ends the others (they would block in a collective).  -> exit code."""
    import signal
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:  # the exact process groups this launcher started
                    try:
                        os.killpg(q.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def tick_times(b, batch_s, update_ms):
    """Room.audioUpdateWorker ticks (every UpdateInterval of media time,
    room.go:1278-1316, config.go:380-384) that fall in batch b's media window
    (b * batch_s, (b + 1) * batch_s], in seconds.  A tick runs after the batch
    that contains it has been enqueued (levels and totals as of that batch)."""
    if update_ms <= 0:
        return []
    u = update_ms / 1e3
    k0 = int(np.floor(b * batch_s / u + 1e-9)) + 1
    out = []
    k = k0
    while k * u <= (b + 1) * batch_s + 1e-9:
        out.append(k * u)
        k += 1
    return out


def kernel_sources_sha():
    """Digest of the engine sources: a PMC traffic summary is only quoted for
    the build it was measured on."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "livekit-server_amd", "csrc")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp")) or f == "Makefile")
    for f in files + ["../../include/lkfwd.h"]:  # every file compiled into liblkfwd.so / the workload
        p = os.path.join(csrc, f)
        if os.path.exists(p):
            h.update(f.encode())
            h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[N-1] (2 = configs[1], the headline)")
    ap.add_argument("--rooms", type=int, default=0, help="rooms per GPU (0: the config's)")
    ap.add_argument("--batch-s", type=float, default=1.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    # HBM traffic per launch from the committed rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE
    # summary of this same workload (scripts/gpu_pmc.sh -> profiles/)
    ap.add_argument("--pmc-csv", default=os.environ.get("LKF_PMC_CSV", ""),
                    help="PMC summary to quote (default: the profiles/r*_pmc_*.json measured on this build and shape)")
    ap.add_argument("--sync-each", action="store_true",
                    help="diagnostic: wait for each step (no decide/emit overlap; standalone kernel times)")
    ap.add_argument("--extpackets", action="store_true",
                    help="step = forwarding of pre-built ExtPacket batches (lkf_submit_device + lkf_run) instead of "
                         "the default raw datagrams -> Buffer.calc (lkf_ingest_device: RTPStatsReceiver, NACK "
                         "queues, RTX buckets) -> forwarding")
    ap.add_argument("--ingress", action="store_true", help="(the default step; kept for older command lines)")
    ap.add_argument("--host-io", action="store_true",
                    help="host-fed deployment shape: lkf_submit from pinned host memory and lkf_drain_run of "
                         "the previous batch into pinned host memory inside the timed region (PCIe both ways)")
    ap.add_argument("--srtp", action="store_true",
                    help="step = forward + SRTP protect (lkf_protect: abs-send-time + AES_CM_128_HMAC_SHA1_80 "
                         "per subscriber transport, every DownTrack bound)")
    ap.add_argument("--alloc-per-step", type=int, default=0,
                    help="deployment shape: the stream allocator's AllocateOptimal for this many video DownTracks "
                         "after every step's run (a control-rate call: it waits for the queued runs)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the parity gate (the CPU oracle over the same rooms and batches, compared after "
                         "the timed region: counters, every Forwarder state, RTPStatsSender, RTPStatsReceiver)")
    ap.add_argument("--srtp-profile", choices=["aes_cm", "gcm"], default="aes_cm",
                    help="with --srtp: SRTP_AES128_CM_HMAC_SHA1_80 or SRTP_AEAD_AES_128_GCM transports")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI)")
    ap.add_argument("--update-ms", type=float, default=400.0,
                    help="N > 1: the room manager's summary all-gather every this many ms of media "
                         "(Room.audioUpdateWorker, UpdateInterval 400 ms); 0 = only once after the run")
    ap.add_argument("--ticks-n1", action="store_true",
                    help="run the --update-ms summary ticks at N = 1 too (packing only: no peer to gather from)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher rehearsal without a GPU: the CPU oracle (tests/dryrun_engine.py) stands in for "
                         "the engine and the backend is gloo; the line is marked dry_run and is not a measurement")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))  # (before anything touches the GPU)
    if not args.rooms:
        args.rooms = CONFIGS[args.config]["rooms"]
    speakers = args.config == 3
    # the whole north-star path by default: raw datagrams through Buffer.calc
    # (pkg/sfu/buffer sequence and NACK tracking) then the forwarding path;
    # configs[2]'s audio levels come from the ingress path in any case
    args.ingress = not args.extpackets or args.config == 3
    if args.host_io and args.config != 3:  # the host-fed shape submits ExtPacket batches from pinned host memory
        args.ingress = False

    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dry = args.dry_run
    backend = "gloo" if dry else args.dist_backend
    if dry:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)

    def csync():
        if not dry:
            torch.cuda.synchronize(dev)

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # where collective tensors live

    pkg = importlib.import_module("livekit-server_amd")
    wl = importlib.import_module("livekit-server_amd.workload")

    nb = args.warmup + args.steps
    # rooms -> ranks: LPT bin packing by expected tuples per batch (SURVEY.md
    # §8(e)); configs[1]'s rooms are all the same shape, so every rank gets
    # args.rooms of them
    rooms_mod = importlib.import_module("livekit-server_amd.rooms")
    plan = rooms_mod.plan_room_shards([1.0] * (world * args.rooms), world)
    trace = wl.Trace(args.config, duration_s=nb * args.batch_s, batch_s=args.batch_s, room_ids=plan[rank])
    if args.ingress:
        wl.events_at_batch_start(trace)
    has_dd = trace.has_dd() and not args.ingress  # (ingest produces the DD side array on the GPU)
    lib = os.environ.get("LKF_LIB") or None
    if lib and os.sep not in lib:  # a name: one of the in-tree builds
        lib = os.path.join(ROOT, "livekit-server_amd", "lib", lib)
    if dry:  # (test infrastructure: the oracle behind Engine's bench-facing methods)
        eng = importlib.import_module("tests.dryrun_engine").DryRunEngine.for_trace(trace)
    else:
        eng = pkg.Engine.for_trace(trace, device=local, lib_path=lib)
    wl.load_topology(eng.api, eng.h, trace)

    if args.ingress:
        wl.load_streams(eng.api, eng.h, trace)
    if args.srtp:  # one transport per (room, subscriber), seeded master keys
        rng = np.random.default_rng(1234)
        tps = {}
        for d in range(trace.ndts):
            k = (int(trace.tracks[trace.downtracks[d].track].room), int(trace.downtracks[d].subscriber))
            if k not in tps:
                gcm = args.srtp_profile == "gcm"
                tps[k] = eng.api["add_transport"](eng.h, C.byref(pkg.transport_params(
                    rng.integers(0, 256, 16, dtype=np.uint8).tobytes(),
                    rng.integers(0, 256, 12 if gcm else 14, dtype=np.uint8).tobytes(),
                    pkg.abi.LKF_SRTP_AEAD_AES_128_GCM if gcm else pkg.abi.LKF_SRTP_AES128_CM_HMAC_SHA1_80)))
                assert tps[k] >= 0
            assert eng.api["set_downtrack_transport"](eng.h, d, tps[k]) == 0

    # inputs resident in HBM before the timed region (--host-io: in pinned host memory)
    dpk, dar, meta, ddd = [], [], [], []
    hdev = torch.device("cpu") if args.host_io or dry else dev
    for b in range(nb):
        if args.ingress:
            pk, n, ar, alen = trace.batch_raw(b)  # raw datagrams: Buffer.calc runs inside the step
            rsz = C.sizeof(pkg.abi.lkf_raw_pkt)
        else:
            pk, n, ar, alen = trace.batch(b)
            rsz = 64
        tp = torch.frombuffer(bytearray(C.string_at(pk, max(1, n) * rsz)), dtype=torch.uint8).to(hdev)
        if args.host_io:
            tp = tp.pin_memory()
        ta = torch.zeros(alen + 64, dtype=torch.uint8, device=hdev, pin_memory=args.host_io)
        if alen:
            ta[:alen].copy_(torch.frombuffer(bytearray(C.string_at(ar, alen)), dtype=torch.uint8))
        dpk.append(tp)
        dar.append(ta)
        meta.append((n, alen))
        if has_dd:  # the batch's lkf_pkt_dd side array, resident like the packets
            dptr, dn = trace.batch_dd(b)
            dsz = C.sizeof(pkg.abi.lkf_pkt_dd)
            ddd.append(torch.frombuffer(bytearray(C.string_at(dptr, max(1, dn) * dsz)), dtype=torch.uint8).to(hdev))
    sp = None if dry else C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    # N > 1: the room manager's summaries (speaker ranking + per-subscriber
    # bandwidth records) all-gathered every --update-ms of media inside the
    # loop.  On the GPU path the engine packs them in HBM on a stream of their
    # own (lkf_room_summaries_enqueue: no host wait, the forwarding pipeline
    # keeps running) and RCCL gathers them there; the gather's own time is
    # measured with events on that stream and reported apart from the metric.
    # Without a GPU (--dry-run) or over gloo they go through host memory.
    width = max(len(p) for p in plan)
    my_rooms = np.asarray(plan[rank], dtype=np.int64)
    tick_on = args.update_ms > 0 and (world > 1 or args.ticks_n1)
    dev_ticks = tick_on and not dry and backend == "nccl"
    tick_log = []  # per tick: (media s, gather events or host ms)
    if dev_ticks:
        K, S = rooms_mod.K_MAX, rooms_mod.S_MAX
        mgr = torch.cuda.Stream(dev)
        ring = []
        for _ in range(8):
            spk = torch.full((width, K, 3), -1, dtype=torch.int32, device=dev)
            spk[:, :, 1:] = 0
            bwe = torch.zeros((width, S, 5), dtype=torch.int64, device=dev)
            bwe[:, :, 0] = -1
            spk_all, bwe_all = (torch.empty((world,) + tuple(spk.shape), dtype=spk.dtype, device=dev),
                                torch.empty((world,) + tuple(bwe.shape), dtype=bwe.dtype, device=dev)) \
                if world > 1 else (spk[None], bwe[None])  # (N = 1: the records are the table)
            ring.append((spk, bwe, spk_all, bwe_all, torch.cuda.Event(enable_timing=True),
                         torch.cuda.Event(enable_timing=True)))
        torch.cuda.synchronize(dev)
        rs_call = eng.api["room_summaries_enqueue"]
        rs_ids = np.ascontiguousarray(my_rooms.astype(np.uint32))
        mgr_p = mgr.cuda_stream

    def gather_tables(spk_np, bwe_np):
        """host path: one all-gather of each record table -> numpy [world, ...]"""
        if not dist:
            return spk_np[None], bwe_np[None]
        return (rooms_mod.all_gather_records(dist, cdev, spk_np), rooms_mod.all_gather_records(dist, cdev, bwe_np))

    def host_records(now):
        spk = rooms_mod.pack_speakers(pkg.speakers_array(eng.api, eng.h, now), my_rooms)
        if width > len(spk):  # a short bin-packed shard: padding rows
            pad = np.full((width - len(spk),) + spk.shape[1:], -1, dtype=np.int32)
            pad[:, :, 1:] = 0
            spk = np.concatenate([spk, pad])
        return spk, rooms_mod.fold_summaries(pkg.downtrack_summaries(eng.api, eng.h), my_rooms, rows=width)

    def summary_tick(t_s):
        now = 1700000000 * 10**9 + int(round(t_s * 1e9))
        if dev_ticks:
            i = len(tick_log) % len(ring)
            spk, bwe, spk_all, bwe_all, e0, e1 = ring[i]
            if len(tick_log) >= len(ring):  # the engine writes these buffers: their last gather must be done
                e1.synchronize()
                j = len(tick_log) - len(ring)
                tick_log[j] = (tick_log[j][0], e0.elapsed_time(e1), None)
            rc = rs_call(eng.h, now, rs_ids.ctypes.data, len(rs_ids), spk.data_ptr(), K, bwe.data_ptr(), S, mgr_p)
            assert rc == 0, rc
            e0.record(mgr)
            if dist:
                with torch.cuda.stream(mgr):
                    dist.all_gather_into_tensor(spk_all, spk)
                    dist.all_gather_into_tensor(bwe_all, bwe)
            e1.record(mgr)
            tick_log.append((t_s, (e0, e1), i))
        else:
            spk, bwe = host_records(now)
            t0_ = time.perf_counter()
            tabs = gather_tables(spk, bwe)
            tick_log.append((t_s, (time.perf_counter() - t0_) * 1e3, tabs))

    hprof = [0.0, 0.0, 0.0] if os.environ.get("LKF_HOST_PROF") else None
    if args.host_io:  # pinned host output buffers for lkf_drain_run
        out_cap = int(trace.max_batch_tuples)
        h_out = torch.empty(out_cap * 40, dtype=torch.uint8, pin_memory=True)
        ar_cap = int(trace.max_batch_out_bytes) + 16 * out_cap
        h_ar = torch.empty(ar_cap, dtype=torch.uint8, pin_memory=True)
    drained = [0, 0]

    def drain_prev(age):
        # the previous drain's copies are done before the buffers are reused;
        # this one's run on the engine's copy stream while the next lkf_submit
        # moves its batch the other way (PCIe both directions at once)
        eng.drain_wait()
        nrec, nbytes = eng.drain_run_async(age, C.c_void_p(h_out.data_ptr()), out_cap,
                                           C.c_void_p(h_ar.data_ptr()), ar_cap)
        drained[0] += nrec
        drained[1] += nbytes

    if args.alloc_per_step:
        vdts = np.array([d for d in range(trace.ndts)
                         if trace.tracks[trace.downtracks[d].track].kind == pkg.abi.LKF_KIND_VIDEO], dtype=np.int32)
        areq = np.zeros(args.alloc_per_step, dtype=pkg.abi.ALLOC_REQ_DTYPE)
        areq["available_layers"] = 7
        areq["bitrates"] = np.sort(np.random.default_rng(7).integers(100_000, 3_000_000, (args.alloc_per_step, 12)),
                                   axis=1).reshape(-1, 3, 4)
        aout = np.zeros(args.alloc_per_step, dtype=pkg.abi.ALLOCATION_DTYPE)

    def step(b):
        ta = time.perf_counter()
        wl.queue_events(eng.api, eng.h, trace, b)
        tb = time.perf_counter()
        n, alen = meta[b]
        if args.ingress:
            eng.ingest_device(C.c_void_p(dpk[b].data_ptr()), n, C.c_void_p(dar[b].data_ptr()), alen)
        elif args.host_io:
            eng.submit(C.c_void_p(dpk[b].data_ptr()), n, C.c_void_p(dar[b].data_ptr()), alen)
        else:
            eng.submit_device(C.c_void_p(dpk[b].data_ptr()), n, C.c_void_p(dar[b].data_ptr()), alen)
            if has_dd:
                assert eng.api["submit_dd_device"](eng.h, C.c_void_p(ddd[b].data_ptr()), n) == 0
        tc = time.perf_counter()
        eng.run(sp)
        if speakers and not tick_on and not dry:  # Room.audioUpdateWorker's tick (ranking stays in HBM; N > 1: summary_tick)
            assert eng.api["speakers_enqueue"](eng.h, 1700000000 * 10**9 + int((b + 1) * args.batch_s * 1e9)) == 0
        if args.srtp:
            assert eng.api["protect"](eng.h, 1700000000 * 10**9 + int(b * args.batch_s * 1e9)) == 0
        if args.alloc_per_step:  # StreamAllocator tick: AllocateOptimal on a rotating set of video DownTracks
            k = args.alloc_per_step
            sel = vdts[(b * k + np.arange(k)) % len(vdts)]
            areq["dt"] = sel
            assert eng.api["allocate_optimal"](eng.h, areq.ctypes.data, k, aout.ctypes.data) == 0
        if args.host_io and b > args.warmup:  # batch b-1's output over PCIe while batch b computes
            drain_prev(1)
        if args.sync_each:
            eng.sync()
        if tick_on:
            for t_s in tick_times(b, args.batch_s, args.update_ms):
                summary_tick(t_s)
        if hprof is not None:
            td = time.perf_counter()
            hprof[0] += tb - ta
            hprof[1] += tc - tb
            hprof[2] += td - tc

    for b in range(args.warmup):
        step(b)
    csync()
    eng.sync()
    warm_cum = eng.cumulative(reset=True)
    if dist:
        dist.barrier()
    csync()
    t0 = time.perf_counter()
    for b in range(args.warmup, nb):
        step(b)
    if args.host_io:
        drain_prev(0)  # the last batch's output reaches host memory inside the timed region
        eng.drain_wait()
    t_host = time.perf_counter() - t0  # host time to enqueue the K steps (control ops, submit, lkf_run)
    if hprof is not None:
        print("host ms/step (incl. warmup): queue_events %.4f submit %.4f run %.4f" %
              tuple(1e3 * x / nb for x in hprof), file=sys.stderr)
    csync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    eng.sync()
    elapsed = t1 - t0
    cum = eng.cumulative()
    # HIP-event window: the engine keeps the last 256 runs' events; longer runs
    # time the last `win` steps and scale the sums to all K steps (steady state)
    win = min(args.steps, 250)
    dec_ms, emit_ms, tot_ms = (v * args.steps / win for v in eng.timing_window(win))
    prot_ms = 0.0
    if args.srtp:
        pm = C.c_float()
        assert eng.lib.lkf_protect_timing_window(C.c_void_p(eng.h), win, C.byref(pm)) == 0
        prot_ms = pm.value * args.steps / win
    coll = None
    if dist or tick_on:
        # the per-room speaker and per-subscriber bandwidth
        # records, gathered every --update-ms of media inside the loop (above)
        if not tick_log:  # (--update-ms 0: once, after the run)
            summary_tick(nb * args.batch_s)
        csync()
        t_last, _, last = tick_log[-1]
        timed = [x for x in tick_log if x[0] > args.warmup * args.batch_s + 1e-9]
        match = None
        if dev_ticks:
            def ms_of(x):
                return x[1] if x[2] is None else x[1][0].elapsed_time(x[1][1])
            gms = [ms_of(x) for x in tick_log]
            gms_timed = [ms_of(x) for x in timed]
            table, btab = ring[last][2].cpu().numpy(), ring[last][3].cpu().numpy()
            if t_last > (nb - 1) * args.batch_s:  # the last tick saw the final state: pack it on the host too
                hs, hb = host_records(1700000000 * 10**9 + int(round(t_last * 1e9)))
                match = bool(np.array_equal(table[rank], hs) and np.array_equal(btab[rank], hb))
        else:
            gms = [x[1] for x in tick_log]
            gms_timed = [x[1] for x in timed]
            table, btab = last
        coll = {"op": "all_gather of per-room speaker records + per-subscriber bandwidth records (%s)" % (
                    "RCCL" if backend == "nccl" else backend),
                "path": ("device: lkf_room_summaries_enqueue packs the records in HBM on a side stream, RCCL "
                         "all_gather_into_tensor there (no host wait in the loop)" if dev_ticks else
                         "host: lkf_speakers + lkf_downtrack_summaries, packed and gathered from host memory"),
                "update_ms": args.update_ms, "ticks": len(tick_log), "ticks_in_timed_region": len(timed),
                "gather_ms_mean": round(float(np.mean(gms)), 4) if gms else None,
                "gather_ms_per_step": round(float(np.sum(gms_timed)) / args.steps, 4),
                "bytes_per_rank": int(table[0].nbytes + btab[0].nbytes),
                "rooms_gathered": int(table.shape[0] * table.shape[1]),
                "rooms_with_speakers": int((table[:, :, 0, 0] >= 0).sum()),
                "subscribers_gathered": int((btab[:, :, :, 0] >= 0).sum()),
                "subscribers_deficient": int((btab[:, :, :, 3] > 0).sum()),
                "device_records_match_host": match,
                "room_plan": "LPT bin packing by expected tuples (rooms.plan_room_shards)",
                "note": "the gathers' time is reported here, apart from the metric; the timed loop includes "
                        "their enqueue"}

    cpu = None
    if not args.no_cpu_baseline:
        # the GPU box gives one GPU a 16-CPU share (os.cpu_count() is the whole
        # host); at N > 1 every rank runs its share at once (N x 16 threads on
        # the node, the memory system shared as the GPUs' hosts would share it)
        # and the rates add up; the single-thread sample runs on rank 0 alone
        thr = args.cpu_threads or min(16, os.cpu_count() or 1)
        cc = CONFIGS[args.config]
        if dist:
            dist.barrier()
        v, secs, rooms, nbat, busy, neng = cpu_baseline(thr, sample_rooms=cc["sample"], config=args.config,
                                                        ingress=args.ingress)
        v_all, busy_min, busy_max = v, min(busy), max(busy)
        if dist:
            t = torch.tensor([v, -min(busy), max(busy)], dtype=torch.float64, device=cdev)
            tsum = t.clone()
            dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            v_all, busy_min, busy_max = float(tsum[0]), -float(t[1]), float(t[2])
        v1 = secs1 = rooms1 = 0
        if rank == 0:
            v1, secs1, rooms1, _, _, _ = cpu_baseline(1, sample_rooms=cc["sample1"], config=args.config,
                                                      ingress=args.ingress)
        if dist:
            dist.barrier()
        used = max(1, min(thr, neng))
        cpu = {"value": round(v_all, 1), "unit": "forwarded RTP pkts/s", "cores": used * world, "kind": "port",
               "sample": "configs[%d] shape%s: %d rooms, 4 s of media (%d batches incl. the arrival tail), %d "
                         "oracle engines (rooms%s) pulled by %d C++ threads (oracle/cpu_bench.cpp; %.1f s "
                         "wall)%s; single thread: %d rooms, %.1f s wall" % (
                             args.config - 1, " through Buffer.calc (orc_ingest)" if args.ingress else "", rooms,
                             nbat, neng, " and, as DownTrackSpreader's parallel fan-out, their DownTracks"
                             if neng > rooms else "", used, secs,
                             (" on each of %d ranks at once (one 16-CPU share per GPU), rates summed" % world)
                             if world > 1 else "", rooms1, secs1),
               "single_thread_value": round(v1, 1), "host_nproc": os.cpu_count(), "cpu_model": cpu_model(),
               "thread_busy_s": {"min": round(busy_min, 3), "max": round(busy_max, 3)}}
        if world > 1:
            cpu["per_rank_value"] = round(v, 1)
        # thread_scaling_eff = the threads' rate over (threads x the single-thread rate), both measured
        cpu["thread_scaling_eff"] = round(v_all / (v1 * used * world), 3) if v1 else None

    parity = None
    if not args.no_parity and not args.srtp and not args.alloc_per_step:
        # (outside the timed region; every rank checks its own rooms)
        thr = args.cpu_threads or min(16, os.cpu_count() or 1)
        parity = parity_gate(eng, pkg, args.config, plan[rank], nb, args.batch_s, args.ingress, trace, thr,
                             warm_cum, cum)
        if dist:
            ok = torch.tensor([1.0 if parity["parity"] else 0.0], dtype=torch.float64, device=cdev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            parity["parity_all_ranks"] = bool(ok.item() > 0)
    fwd = cum["forwarded"]
    steps_pkts = sum(meta[b][0] for b in range(args.warmup, nb))
    algo, b_in, b_ing = algorithmic_bytes(trace, range(args.warmup, nb), fwd, cum["out_bytes"], trace.ndts,
                                          ingress=args.ingress)
    payload_in = b_in - 64 * steps_pkts
    # per-kernel algorithmic bytes (the two halves of SURVEY.md §8(d)'s B):
    #   decide: packet descriptors once + sequencer record per forwarded tuple + DT hot state
    #   emit:   input payload once + wire bytes + one 40-B output record per forwarded tuple
    decide_bytes = 64 * steps_pkts + 32 * fwd + 256 * trace.ndts * args.steps
    emit_bytes = payload_in + cum["out_bytes"] + 40 * fwd
    if dist:
        t = torch.tensor([elapsed, float(fwd), float(algo), tot_ms, emit_ms], dtype=torch.float64, device=cdev)
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        fwd_all = float(t[1])
    else:
        fwd_all = float(fwd)

    if rank == 0:
        def kern(name, nbytes, ms_sum):
            avg_s = ms_sum / 1e3 / args.steps
            ach = nbytes / args.steps / avg_s / 1e9 if avg_s > 0 else 0.0
            return {"kernel": name, "avg_ms": round(ms_sum / args.steps, 4),
                    "algorithmic_bytes_per_launch": int(nbytes // args.steps),
                    "achieved": round(ach, 1), "frac": round(ach / PEAK_HBM_GBPS, 4)}

        ms_step = elapsed * 1e3 / args.steps
        b_step = algo / args.steps
        # the whole step's algorithmic bytes B over the step time
        # (decide and emit overlap across batches on two streams, so the step —
        # not one kernel — is what B is spent in); per-kernel figures below are
        # a breakdown (each kernel's own bytes over its own HIP-event time).
        ach = b_step / (ms_step / 1e3) / 1e9
        kd = kern("k_decide_dt", decide_bytes, dec_ms)
        ke = kern("k_emit", emit_bytes, emit_ms)
        traffic, traffic_src = None, None
        cands = [args.pmc_csv] if args.pmc_csv else sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_*.json")))
        sha = kernel_sources_sha()
        for path in cands:  # a summary of this build and this exact shape (scripts/gpu_pmc.sh)
            try:
                pmc = json.load(open(path))
            except Exception:
                continue
            if (pmc.get("kernel_sources_sha") == sha and pmc.get("bench_args_rooms") == args.rooms
                    and pmc.get("bench_args_config", 2) == args.config
                    and bool(pmc.get("bench_args_ingress", False)) == bool(args.ingress)
                    and abs(float(pmc.get("bench_args_batch_s", 1.0)) - args.batch_s) < 1e-9
                    and bool(pmc.get("bench_args_srtp", False)) == bool(args.srtp)):
                traffic = pmc.get("hbm_bytes_per_step")
                traffic_src = os.path.relpath(path, ROOT)
                break
        pipe_ach = algo / (tot_ms / 1e3) / 1e9 if tot_ms else 0.0
        line = {
            "metric": "forwarded RTP pkts/sec per GPU & node (bit-exact) + % HBM roofline",
            "value": round(fwd_all / elapsed, 1),
            "unit": "forwarded RTP pkts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": workload_name(args.config, args.rooms, trace.ndts),
                       "batch": "%.3g s of media per step" % args.batch_s,
                       "step": ("raw datagrams -> Buffer.calc -> forward (lkf_ingest_device + lkf_run)"
                                if args.ingress else
                                "host-fed: pinned host ExtPacket batch -> lkf_submit (H2D) + lkf_run + "
                                "lkf_drain_run of the previous batch (D2H)" if args.host_io else
                                "ExtPacket batch -> forward (lkf_submit_device + lkf_run) + SRTP protect (lkf_protect)"
                                if args.srtp else
                                "ExtPacket batch -> forward (lkf_submit_device + lkf_run)"),
                       "parallelism": "room-sharded x%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": round(ach / PEAK_HBM_GBPS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "whole step (k_decide_dt || k_emit + prep kernels)",
                         "algorithmic_bytes_per_step": int(b_step),
                         "kernels": [kd, ke],
                         "pipeline": {"gpu_ms_per_step": round(tot_ms / args.steps, 4),
                                      "achieved": round(pipe_ach, 1),
                                      "frac": round(pipe_ach / PEAK_HBM_GBPS, 4)}},
            "cpu_baseline": cpu,
            "parity": (parity["parity_all_ranks"] if parity and "parity_all_ranks" in parity
                       else parity["parity"] if parity else None),
            "parity_gate": parity,
            "host_enqueue_ms_per_step": round(t_host * 1e3 / args.steps, 4),
            "collective": coll,
            "tuples_per_step": cum["tuples"] // args.steps,
            "forwarded_per_step": fwd // args.steps,
            "forwarded_total": int(fwd_all),
        }
        if dry:
            line["dry_run"] = True
            line["note"] = ("launcher rehearsal: the CPU oracle stood in for the engine (tests/dryrun_engine.py); "
                            "not a measurement")
        if args.host_io:  # PCIe-inclusive deployment shape (never the headline value)
            h2d = sum(meta[b][0] * 64 + meta[b][1] for b in range(args.warmup, nb))
            line["host_io"] = {"h2d_bytes_per_step": h2d // args.steps,
                               "d2h_bytes_per_step": (drained[0] * 40 + drained[1]) // args.steps,
                               "drained_records": drained[0], "records_forwarded": fwd,
                               "pcie_GBps_both_ways": round((h2d + drained[0] * 40 + drained[1]) / elapsed / 1e9, 2)}
        if args.srtp:  # the protect stage: VALU/LDS-bound crypto, reported against HBM for the record
            tag = 16 if args.srtp_profile == "gcm" else 10
            prot_bytes = cum["out_bytes"] * 2 + tag * fwd + 40 * fwd
            pa = prot_bytes / args.steps / (prot_ms / 1e3 / args.steps) / 1e9 if prot_ms else 0.0
            line["srtp"] = {"profile": "SRTP_AEAD_AES_128_GCM" if tag == 16 else "SRTP_AES128_CM_HMAC_SHA1_80", "protected_per_step": fwd // args.steps,
                            "protect_ms_per_step": round(prot_ms / args.steps, 4),
                            "protected_pkts_per_s_kernel": round(fwd / (prot_ms / 1e3), 1) if prot_ms else None,
                            "algorithmic_bytes_per_launch": int(prot_bytes // args.steps),
                            "achieved": round(pa, 1), "frac_hbm": round(pa / PEAK_HBM_GBPS, 4)}
        if args.alloc_per_step:  # control-rate calls inside the timed loop (each drains the queued runs)
            line["control"] = {"alloc_optimal_per_step": args.alloc_per_step,
                               "note": "lkf_allocate_optimal after every run: waits for the queued runs (no overlap "
                                       "across that step boundary)"}
        print(json.dumps(line))
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
