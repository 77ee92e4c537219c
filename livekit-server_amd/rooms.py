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
one collective of a known shape; the room index of a record is
room_base(rank) + slot.
"""
import numpy as np

K_MAX = 64  # participants per room the record holds (lkf_speakers ranks <= 64 per room)


def pack_speakers(speakers, room_base, rooms, k=K_MAX):
    """speakers: SPEAKER_DTYPE array (room, participant, level, active), grouped by
    room in ascending order, ranked within a room.  -> int32 [rooms, k, 3]."""
    out = np.full((rooms, k, 3), -1, dtype=np.int32)
    out[:, :, 1:] = 0
    if len(speakers):
        rel = speakers["room"].astype(np.int64) - room_base
        if rel.min() < 0 or rel.max() >= rooms:
            raise ValueError("speaker record outside this rank's rooms")
        # position within its room = index - first index of that room
        first = np.searchsorted(rel, rel, side="left")
        pos = np.arange(len(rel)) - first
        keep = pos < k
        r, p = rel[keep], pos[keep]
        out[r, p, 0] = speakers["participant"][keep].astype(np.int32)
        out[r, p, 1] = speakers["level"][keep].astype(np.float32).view(np.int32)
        out[r, p, 2] = speakers["active"][keep].astype(np.int32)
    return out


def unpack(table, rooms_per_rank):
    """[world, rooms, k, 3] int32 -> {room: [(participant, level, active), ...]} (ranked)."""
    res = {}
    world = table.shape[0]
    for w in range(world):
        for s in range(rooms_per_rank):
            rec = table[w, s]
            live = rec[:, 0] >= 0
            if not live.any():
                continue
            lv = rec[live, 1].astype(np.int32).view(np.float32)
            res[w * rooms_per_rank + s] = [(int(a), float(b), int(c)) for a, b, c in zip(rec[live, 0], lv, rec[live, 2])]
    return res


def all_gather_speakers(dist, device, speakers, room_base, rooms_per_rank, k=K_MAX):
    """One all-gather of this rank's packed room records -> numpy [world, rooms, k, 3]."""
    import torch
    local = torch.from_numpy(pack_speakers(speakers, room_base, rooms_per_rank, k)).to(device)
    world = dist.get_world_size()
    out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=device)
    try:
        dist.all_gather_into_tensor(out, local)
    except (RuntimeError, NotImplementedError):  # backends without the fused form
        parts = list(out.unbind(0))
        dist.all_gather(parts, local)
        out = torch.stack(parts)
    return out.cpu().numpy()
