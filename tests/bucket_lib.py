"""Raw batches that push the receivers' buckets to their edges (test
infrastructure): one batch long enough that a stream wraps its bucket inside
the batch (audio: 200 slots, a 5-s batch holds ~250 packets per Opus
stream), and a datagram of a video and of an audio stream each delivered late
— moved to the end of its track's group, ~250 / ~300 sequence numbers behind
the head — so AddPacketWithSequenceNumber rejects it as too old."""
import ctypes as C
import importlib

abi = importlib.import_module("livekit-server_amd.abi")


def late_batch(trace, b=0, seq_size=500):
    """Batch b of `trace` as raw datagrams with two late arrivals (one audio,
    one video datagram moved behind the rest of its track, later than its
    bucket's window); returns (raws ctypes array, n, arena pointer, arena
    length, [(stream, sn16)] of the moved datagrams)."""
    rp, n, ar, alen = trace.batch_raw(b)
    copies = [abi.lkf_raw_pkt() for _ in range(n)]
    for i in range(n):
        C.memmove(C.byref(copies[i]), C.byref(rp[i]), C.sizeof(abi.lkf_raw_pkt))
    arena = C.string_at(ar, alen)
    track_of = [int(trace.streams[int(c.stream)].track) for c in copies]
    moved = []
    for kind in (abi.LKF_KIND_AUDIO, abi.LKF_KIND_VIDEO):
        window = 200 if kind == abi.LKF_KIND_AUDIO else seq_size
        for t in sorted(set(track_of)):
            if trace.tracks[t].kind != kind:
                continue
            idx = [i for i in range(n) if track_of[i] == t]
            by_stream = {}
            for i in idx:
                by_stream.setdefault(int(copies[i].stream), []).append(i)
            s, lst = max(by_stream.items(), key=lambda kv: len(kv[1]))
            if len(lst) < window + 20:
                continue
            src, end = lst[5], idx[-1]
            row = copies.pop(src)
            copies.insert(end, row)
            track_of.insert(end, track_of.pop(src))
            pkt = arena[row.off:row.off + row.len]
            moved.append((s, (pkt[2] << 8) | pkt[3]))
            break
    arr = (abi.lkf_raw_pkt * n)(*copies)
    return arr, n, ar, alen, moved
