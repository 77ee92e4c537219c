"""Parity of the exact step bench.py times.

bench.py's headline step is lkf_ingest_device + lkf_run on configs[1] at 100
rooms (18,000 DownTracks), 1-s batches, with the raw datagrams resident in
HBM and every batch queued without a sync: three batch contexts and two
alternating ingest scratch sets in flight, the NACK queues on the side
stream, the bucket copies on the sender stream, RTPStatsSender folded into
decide.  Here the same shape runs next to the CPU oracle (which ingests and
forwards each batch serially) and, once everything has drained:

  - the last three batches' records and wire bytes (lkf_drain_run, ages 0-2),
  - the cumulative counters over every batch,
  - every DownTrack's exported Forwarder state and RTPStatsSender,
  - every stream's RTPStatsReceiver (Buffer.calc) and the per-DownTrack
    sendingPacket summaries

must be identical.  bench.py's own parity gate (--parity) checks a digest of
the same quantities at the benched step count."""
import ctypes as C
import importlib

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle
from tests.test_parity_gpu import _state_tuple, check_sender_stats

pytestmark = pytest.mark.gpu


def _drain_age(eng, age, cap, acap):
    out = np.zeros(cap, dtype=importlib.import_module("livekit-server_amd.abi").OUT_DTYPE)
    ar = np.zeros(acap, dtype=np.uint8)
    n, nb = eng.drain_run_into(age, C.c_void_p(out.ctypes.data), cap, C.c_void_p(ar.ctypes.data), acap)
    return out[:n], ar[:nb]


def test_pipelined_ingest_device_bench_shape(pkg, workload, abi):
    import torch

    rooms = importlib.import_module("livekit-server_amd.rooms")
    plan = rooms.plan_room_shards([1.0] * 100, 1)
    tr = workload.Trace(2, duration_s=6.0, batch_s=1.0, room_ids=plan[0])
    assert tr.ndts == 18000 and tr.nbatches >= 6
    nb = tr.nbatches
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    eng = pkg.Engine.for_trace(tr)
    o = load_oracle()
    oh = o.create(500)
    try:
        for api, h in ((eng.api, eng.h), (o.api, oh)):
            workload.load_topology(api, h, tr)
            workload.load_streams(api, h, tr)
        dpk, dar, meta = [], [], []
        rsz = C.sizeof(abi.lkf_raw_pkt)
        for b in range(nb):  # HBM-resident inputs, as bench.py holds them
            rp, n, ar, alen = tr.batch_raw(b)
            dpk.append(torch.frombuffer(bytearray(C.string_at(rp, max(1, n) * rsz)), dtype=torch.uint8).to(dev))
            ta = torch.zeros(alen + 64, dtype=torch.uint8, device=dev)
            if alen:
                ta[:alen].copy_(torch.frombuffer(bytearray(C.string_at(ar, alen)), dtype=torch.uint8))
            dar.append(ta)
            meta.append((n, alen))
        torch.cuda.synchronize(dev)
        sp = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        for b in range(nb):  # the engine: every batch queued, no sync
            workload.queue_events(eng.api, eng.h, tr, b)
            n, alen = meta[b]
            eng.ingest_device(C.c_void_p(dpk[b].data_ptr()), n, C.c_void_p(dar[b].data_ptr()), alen)
            eng.run(sp)
        # the oracle, batch by batch
        cum = {}
        last = {}
        for b in range(nb):
            workload.queue_events(o.api, oh, tr, b)
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](oh, rp, n, ar, alen) == 0
            k = C.c_uint32()
            assert o.api["ingested"](oh, None, 0, C.byref(k)) in (0, -28)
            arr = (abi.lkf_pkt * max(1, k.value))()
            assert o.api["ingested"](oh, arr, k.value, C.byref(k)) == 0
            o.run(oh, arr if k.value else None, k.value, ar, alen)
            st = abi.lkf_stats()
            assert o.api["get_stats"](oh, C.byref(st)) == 0
            for key, v in st.as_dict().items():
                if isinstance(v, list):
                    cum[key] = [a + c for a, c in zip(cum.get(key, [0] * len(v)), v)]
                else:
                    cum[key] = cum.get(key, 0) + v
            if b >= nb - 3:
                last[b] = pkg.drain_arrays(o.api, oh)
        torch.cuda.synchronize(dev)
        eng.sync()
        cap = int(tr.max_batch_tuples * 1.25) + 1024
        acap = int(tr.max_batch_out_bytes * 1.25) + (1 << 20)
        for age in range(3):
            b = nb - 1 - age
            grec, gar = _drain_age(eng, age, cap, acap)
            orec, oar = last[b]
            assert len(grec) == len(orec), (b, len(grec), len(orec))
            for f in abi.OUT_DTYPE.names:
                assert np.array_equal(grec[f], orec[f]), (b, f)
            assert np.array_equal(gar, oar), b
        gc = eng.cumulative()
        assert gc == cum, (gc, cum)
        assert gc["forwarded"] > 5_000_000
        for d in range(tr.ndts):
            assert _state_tuple(eng.api, eng.h, d, abi) == _state_tuple(o.api, oh, d, abi), d
        check_sender_stats(pkg, eng.api, eng.h, o.api, oh, range(tr.ndts))
        for s in range(tr.nstreams):
            assert eng.stream_stats(s) == pkg.stream_stats(o.api, oh, s), s
        gs, os_ = pkg.downtrack_summaries(eng.api, eng.h), pkg.downtrack_summaries(o.api, oh)
        assert np.array_equal(gs, os_)
    finally:
        eng.close()
        o.destroy(oh)
