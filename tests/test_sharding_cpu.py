"""Room sharding across ranks on CPU with torch.distributed/gloo.

Each rank generates only its own rooms (room_base = rank * rooms, as bench.py
does per GPU) and forwards them through the CPU oracle; the per-rank totals,
all-reduced over gloo, must equal one process forwarding all rooms.  This is
the property that lets the GPU bench shard rooms with no data-path collective.
"""
import ctypes as C
import importlib
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOMS_PER_RANK = 2
WORLD = 2


def _forward(rooms, room_base):
    from tests.oracle_lib import load as load_oracle
    wl = importlib.import_module("livekit-server_amd.workload")
    abi = importlib.import_module("livekit-server_amd.abi")
    o = load_oracle()
    tr = wl.Trace(2, duration_s=2.0, batch_s=1.0, rooms=rooms, room_base=room_base)
    h = o.create(500)
    tot = [0] * (4 + 11)
    try:
        wl.load_topology(o.api, h, tr)
        for b in range(tr.nbatches):
            wl.queue_events(o.api, h, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(h, pk, n, ar, alen)
            st = abi.lkf_stats()
            o.api["get_stats"](h, C.byref(st))
            d = st.as_dict()
            tot[0] += d["tuples"]
            tot[1] += d["forwarded"]
            tot[2] += d["out_bytes"]
            for i, v in enumerate(d["drops"]):
                tot[4 + i] += v
    finally:
        o.destroy(h)
        tr.close()
    return tot


def _worker(rank, port, q):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        tot = _forward(ROOMS_PER_RANK, rank * ROOMS_PER_RANK)
        t = torch.tensor(tot, dtype=torch.int64)
        dist.all_reduce(t)
        if rank == 0:
            q.put(t.tolist())
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_room_sharding_gloo_matches_single_process(pkg):
    from tests import oracle_lib
    oracle_lib.load()  # build before forking
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    got = q.get(timeout=10)
    want = _forward(ROOMS_PER_RANK * WORLD, 0)
    assert got == want
    assert got[1] > 0


# ---- §8(e): the one collective — per-room speaker summaries, all-gathered ----
SPK_ROOMS_PER_RANK = 1


def _speakers(rooms, room_base, now):
    from tests.oracle_lib import load as load_oracle
    wl = importlib.import_module("livekit-server_amd.workload")
    pkg = importlib.import_module("livekit-server_amd")
    o = load_oracle()
    tr = wl.Trace(3, duration_s=2.0, batch_s=0.4, rooms=rooms, room_base=room_base)
    h = o.create(500)
    try:
        wl.load_topology(o.api, h, tr)
        wl.load_streams(o.api, h, tr)
        for b in range(tr.nbatches):
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](h, rp, n, ar, alen) == 0
        return pkg.speakers_array(o.api, h, now)
    finally:
        o.destroy(h)
        tr.close()


def _spk_worker(rank, port, q):
    import torch
    rooms_mod = importlib.import_module("livekit-server_amd.rooms")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        now = 1700000000 * 10**9 + int(2.0e9)
        base = rank * SPK_ROOMS_PER_RANK
        sp = _speakers(SPK_ROOMS_PER_RANK, base, now)
        table = rooms_mod.all_gather_speakers(dist, torch.device("cpu"), sp,
                                              rooms_mod.rank_rooms(base, SPK_ROOMS_PER_RANK))
        if rank == 0:
            q.put(table)
    finally:
        dist.destroy_process_group()


def test_speaker_summaries_all_gathered():
    """Every rank's per-room speaker records, all-gathered, equal one process ranking all rooms."""
    rooms_mod = importlib.import_module("livekit-server_amd.rooms")
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_spk_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    table = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert table.shape == (WORLD, SPK_ROOMS_PER_RANK, rooms_mod.K_MAX, 3)
    now = 1700000000 * 10**9 + int(2.0e9)
    full = _speakers(WORLD * SPK_ROOMS_PER_RANK, 0, now)
    want = rooms_mod.pack_speakers(full, rooms_mod.rank_rooms(0, WORLD * SPK_ROOMS_PER_RANK)).reshape(table.shape)
    assert (table == want).all()
    assert (table[:, :, 0, 0] >= 0).any()  # at least one room has a ranked speaker


# ---- §8(e): per-subscriber bandwidth records over a bin-packed room plan ----
BWE_ROOMS = 5


def _bwe(room_ids, rows=None):
    """Forward the rooms through the oracle; fold lkf_downtrack_summaries per (room, subscriber)."""
    from tests.oracle_lib import load as load_oracle
    wl = importlib.import_module("livekit-server_amd.workload")
    pkg = importlib.import_module("livekit-server_amd")
    rooms_mod = importlib.import_module("livekit-server_amd.rooms")
    o = load_oracle()
    tr = wl.Trace(2, duration_s=2.0, batch_s=1.0, room_ids=list(room_ids))
    h = o.create(500)
    try:
        wl.load_topology(o.api, h, tr)
        for b in range(tr.nbatches):
            wl.queue_events(o.api, h, tr, b)
            pk, n, ar, alen = tr.batch(b)
            o.run(h, pk, n, ar, alen)
        summ = pkg.downtrack_summaries(o.api, h)
        # the summaries are the per-DownTrack sums of the drained output
        return rooms_mod.fold_summaries(summ, sorted(room_ids), rows=rows), summ
    finally:
        o.destroy(h)
        tr.close()


def _bwe_worker(rank, port, plan, q):
    width = max(len(p) for p in plan)
    import torch
    rooms_mod = importlib.import_module("livekit-server_amd.rooms")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        rec, _ = _bwe(plan[rank], rows=width)
        table = rooms_mod.all_gather_records(dist, torch.device("cpu"), rec)
        if rank == 0:
            q.put(table)
    finally:
        dist.destroy_process_group()


def test_bwe_records_bin_packed_match_single_process():
    """Rooms bin-packed onto 2 ranks (unequal room counts); each rank forwards
    only its rooms and folds its DownTrack summaries; the all-gathered
    per-(room, subscriber) records equal one process forwarding every room."""
    rooms_mod = importlib.import_module("livekit-server_amd.rooms")
    costs = [3.0, 1.0, 1.0, 1.0, 2.0]  # expected tuples per room (heterogeneous on purpose)
    plan = rooms_mod.plan_room_shards(costs, WORLD)
    assert sorted(r for p in plan for r in p) == list(range(BWE_ROOMS))
    assert len(plan[0]) != len(plan[1])
    # fixed-shape gather: pad the shorter shard's room list to the longest
    width = max(len(p) for p in plan)
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bwe_worker, args=(r, port, plan, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    table = q.get(timeout=10)
    assert table.shape[0] == WORLD and table.shape[1] == width
    got = rooms_mod.unpack_bwe(table, plan)
    full, summ = _bwe(range(BWE_ROOMS))
    want = rooms_mod.unpack_bwe(full[None], [list(range(BWE_ROOMS))])
    assert got == want
    assert sum(v[1] for v in got.values()) == int(summ["bytes_sent"].sum()) > 0
    assert any(v[2] for v in got.values())  # some subscriber was left deficient by an allocation


def test_plan_room_shards_lpt():
    rooms_mod = importlib.import_module("livekit-server_amd.rooms")
    import itertools
    costs = [7, 5, 4, 4, 3, 3, 2, 1]
    plan = rooms_mod.plan_room_shards(costs, 3)
    loads = [sum(costs[r] for r in p) for p in plan]
    best = min(max(sum(costs[r] for r in range(8) if a[r] == w) for w in range(3))
               for a in itertools.product(range(3), repeat=8))
    assert max(loads) <= best * 4 / 3 + 1e-9  # Graham's LPT bound
    assert sorted(r for p in plan for r in p) == list(range(8))
