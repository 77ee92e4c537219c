"""Per-room speaker summaries gathered to every rank.

Rooms shard across GPUs with no data-path exchange; the one collective is an
all-gather of fixed-size per-room records every 400 ms of virtual time, which
the room manager consumes (Room.GetActiveSpeakers room.go:254-279 results;
pkg/service/roommanager.go is the consumer in the reference).

A rank packs its rooms' ranked speakers (lkf_speakers output, grouped by room,
sorted within a room) into a dense int32 tensor

    [rooms_per_rank, K, 3] = (participant, float32 bits of the quantised level, active)

padded with participant = -1, then `torch.distributed.all_gather_into_tensor`
(RCCL over xGMI with the nccl backend, gloo on CPU) gives every rank the
[world, rooms_per_rank, K, 3] table.  Records are fixed-size so the gather is
one collective of a known shape; slot i of a rank's records is the i-th room
of that rank's (ascending) room list — a contiguous range or a bin-packed
shard (plan_room_shards).
"""
import numpy as np

K_MAX = 64  # participants per room the record holds (lkf_speakers ranks <= 64 per room)


def _slots(room_of_record, room_ids):
    """Index of each record's room in this rank's (ascending) room list."""
    ids = np.asarray(room_ids, dtype=np.int64)
    rr = np.asarray(room_of_record, dtype=np.int64)
    rel = np.searchsorted(ids, rr)
    if len(rr) and (rel.max() >= len(ids) or np.any(ids[np.minimum(rel, len(ids) - 1)] != rr)):
        raise ValueError("record outside this rank's rooms")
    return rel


def rank_rooms(room_base, rooms):
    """The contiguous shard [room_base, room_base + rooms) as a room list."""
    return np.arange(room_base, room_base + rooms, dtype=np.int64)


def pack_speakers(speakers, room_ids, k=K_MAX):
    """speakers: SPEAKER_DTYPE array (room, participant, level, active), grouped by
    room in ascending order, ranked within a room; room_ids: this rank's rooms
    (ascending).  -> int32 [len(room_ids), k, 3]."""
    out = np.full((len(room_ids), k, 3), -1, dtype=np.int32)
    out[:, :, 1:] = 0
    if len(speakers):
        rel = _slots(speakers["room"], room_ids)
        # position within its room = index - first index of that room
        first = np.searchsorted(rel, rel, side="left")
        pos = np.arange(len(rel)) - first
        keep = pos < k
        r, p = rel[keep], pos[keep]
        out[r, p, 0] = speakers["participant"][keep].astype(np.int32)
        out[r, p, 1] = speakers["level"][keep].astype(np.float32).view(np.int32)
        out[r, p, 2] = speakers["active"][keep].astype(np.int32)
    return out


def unpack(table, rank_room_ids):
    """[world, rooms, k, 3] int32 + each rank's room list -> {room: [(participant, level, active), ...]}."""
    res = {}
    for w in range(table.shape[0]):
        for s, room in enumerate(rank_room_ids[w]):
            rec = table[w, s]
            live = rec[:, 0] >= 0
            if not live.any():
                continue
            lv = rec[live, 1].astype(np.int32).view(np.float32)
            res[int(room)] = [(int(a), float(b), int(c)) for a, b, c in zip(rec[live, 0], lv, rec[live, 2])]
    return res


def all_gather_speakers(dist, device, speakers, room_ids, k=K_MAX):
    """One all-gather of this rank's packed room records -> numpy [world, rooms, k, 3]."""
    return all_gather_records(dist, device, pack_speakers(speakers, room_ids, k))


# ---- per-subscriber bandwidth summaries -------------------
# A rank folds lkf_downtrack_summaries (per DownTrack: sendingPacket's bytesSent
# and packet count, lastAllocation.IsDeficient) into one record per
# (room, subscriber) — what the room manager needs to see a subscriber's
# downstream rate and whether the allocator left it deficient — packed as
#
#     [rooms_per_rank, S, 5] int64 = (subscriber, packets, bytes, deficient DownTracks, DownTracks)
#
# with subscriber = -1 padding; one all-gather gives every rank the table.
S_MAX = 64  # subscribers per room the record holds


def fold_summaries(summ, room_ids, s=S_MAX, active_only=True, rows=None):
    """summ: DT_SUMMARY_DTYPE rows; room_ids: this rank's rooms (ascending)
    -> int64 [rows or len(room_ids), s, 5], subscribers ascending within a
    room (rows > len(room_ids) pads a short bin-packed shard to the gather's
    common shape)."""
    out = np.zeros((max(rows or 0, len(room_ids)), s, 5), dtype=np.int64)
    out[:, :, 0] = -1
    rows = summ[(summ["flags"] & 1) != 0] if active_only else summ
    if not len(rows):
        return out
    rel = _slots(rows["room"], room_ids)
    key = rel * (1 << 32) + rows["subscriber"].astype(np.int64)
    uk, inv = np.unique(key, return_inverse=True)
    pk = np.bincount(inv, weights=None, minlength=len(uk))  # DownTracks
    agg = np.zeros((len(uk), 3), dtype=np.int64)
    np.add.at(agg[:, 0], inv, rows["packets_sent"].astype(np.int64))
    np.add.at(agg[:, 1], inv, rows["bytes_sent"].astype(np.int64))
    np.add.at(agg[:, 2], inv, ((rows["flags"] & 2) != 0).astype(np.int64))
    ur, us = uk >> 32, uk & 0xFFFFFFFF
    first = np.searchsorted(ur, ur, side="left")
    pos = np.arange(len(uk)) - first
    keep = pos < s
    r, p = ur[keep], pos[keep]
    out[r, p, 0] = us[keep]
    out[r, p, 1] = agg[keep, 0]
    out[r, p, 2] = agg[keep, 1]
    out[r, p, 3] = agg[keep, 2]
    out[r, p, 4] = pk[keep]
    return out


def all_gather_records(dist, device, local_np):
    """One all-gather of a rank's fixed-shape record table -> numpy [world, ...]."""
    import torch
    local = torch.from_numpy(np.ascontiguousarray(local_np)).to(device)
    world = dist.get_world_size()
    out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=device)
    try:
        dist.all_gather_into_tensor(out, local)
    except (RuntimeError, NotImplementedError):
        parts = list(out.unbind(0))
        dist.all_gather(parts, local)
        out = torch.stack(parts)
    return out.cpu().numpy()


def unpack_bwe(table, rank_room_ids):
    """[world, rooms, s, 5] + each rank's room list -> {(room, subscriber): (packets, bytes, deficient_dts, dts)}."""
    res = {}
    for w in range(table.shape[0]):
        for r, room in enumerate(rank_room_ids[w]):
            for rec in table[w, r]:
                if rec[0] < 0:
                    continue
                res[(int(room), int(rec[0]))] = tuple(int(v) for v in rec[1:])
    return res


# ---- room -> rank assignment ---------------------------------------------
def plan_room_shards(costs, world):
    """Longest-processing-time bin packing of rooms onto ranks by expected
    per-batch work (tuples = packets x subscribing DownTracks): rooms in
    descending cost, each to the least-loaded rank (ties: lowest rank, then
    lowest room).  Returns per-rank sorted room lists.  A room never splits:
    its DownTracks share the track's packets and the speaker ranking."""
    order = sorted(range(len(costs)), key=lambda r: (-costs[r], r))
    load = [0.0] * world
    out = [[] for _ in range(world)]
    for r in order:
        w = min(range(world), key=lambda k: (load[k], k))
        out[w].append(r)
        load[w] += costs[r]
    return [sorted(x) for x in out]


def room_cost(trace_room_tuples):
    """Expected tuples of a room per batch from a topology: sum over its tracks
    of (packets per batch) x (subscribing DownTracks)."""
    return float(sum(trace_room_tuples))
