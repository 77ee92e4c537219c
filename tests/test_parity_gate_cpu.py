"""bench.py's parity gate on CPU: the oracle run over a whole shard of rooms
plays the engine, the gate's sharded oracle run (orc_parity_run, several room
shards on C++ threads) must agree with it on every counter, Forwarder state,
RTPStatsSender and RTPStatsReceiver — which checks the SSRC keying and the
shard/whole-trace equivalence the gate relies on — and a perturbed state must
make it fail."""
import ctypes as C
import importlib

import pytest

from tests.oracle_lib import load as load_oracle


class _OracleAsEngine:
    def __init__(self, o, h):
        self.api, self.h = o.api, h


def _run_whole(o, wl, abi, tr, nb, ingress):
    h = o.create(500)
    wl.load_topology(o.api, h, tr)
    if ingress:
        wl.load_streams(o.api, h, tr)
    warm = {"tuples": 0, "forwarded": 0, "out_bytes": 0, "arena_bytes": 0, "drops": [0] * abi.LKF_DROP_NREASONS}
    for b in range(nb):
        wl.queue_events(o.api, h, tr, b)
        if ingress:
            rp, n, ar, alen = tr.batch_raw(b)
            assert o.api["ingest"](h, rp, n, ar, alen) == 0
            k = C.c_uint32()
            assert o.api["ingested"](h, None, 0, C.byref(k)) in (0, -28)
            arr = (abi.lkf_pkt * max(1, k.value))()
            assert o.api["ingested"](h, arr, k.value, C.byref(k)) == 0
            o.run(h, arr if k.value else None, k.value, ar, alen)
        else:
            pk, n, ar, alen = tr.batch(b)
            o.run(h, pk, n, ar, alen, tr.batch_dd(b)[0] if tr.has_dd() else None)
        st = abi.lkf_stats()
        assert o.api["get_stats"](h, C.byref(st)) == 0
        d = st.as_dict()
        for k in ("tuples", "forwarded", "out_bytes", "arena_bytes"):
            warm[k] += d[k]
        warm["drops"] = [a + c for a, c in zip(warm["drops"], d["drops"])]
    return h, warm


@pytest.mark.parametrize("config,ingress", [(2, True), (2, False), (5, False)])
def test_parity_gate_oracle_vs_oracle(config, ingress):
    bench = importlib.import_module("bench")
    pkg = importlib.import_module("livekit-server_amd")
    wl = importlib.import_module("livekit-server_amd.workload")
    abi = pkg.abi
    rooms = importlib.import_module("livekit-server_amd.rooms")
    room_ids = rooms.plan_room_shards([1.0] * 12, 2)[1]  # rank 1's rooms of a 2-rank plan
    nb = 3
    tr = wl.Trace(config, duration_s=float(nb), batch_s=1.0, room_ids=room_ids)
    if ingress:  # (bench.py's ingress step: control ops at the batch start)
        wl.events_at_batch_start(tr)
    o = load_oracle()
    h, tot = _run_whole(o, wl, abi, tr, nb, ingress)
    zero = {"tuples": 0, "forwarded": 0, "out_bytes": 0, "arena_bytes": 0, "drops": [0] * abi.LKF_DROP_NREASONS}
    try:
        res = bench.parity_gate(_OracleAsEngine(o, h), pkg, config, room_ids, nb, 1.0, ingress, tr, 3, zero, tot)
        assert res["parity"], res
        assert res["downtracks_checked"] == tr.ndts and res["forwarded_total"] > 1000
        # a perturbed counter and a perturbed DownTrack state are both caught
        bad = dict(tot)
        bad["forwarded"] += 1
        res = bench.parity_gate(_OracleAsEngine(o, h), pkg, config, room_ids, nb, 1.0, ingress, tr, 3, zero, bad)
        assert not res["parity"] and not res["counters_equal"]
        # one more batch on the engine side only: its DownTracks move on
        pk, n, ar, alen = tr.batch(nb)
        o.run(h, pk, n, ar, alen, tr.batch_dd(nb)[0] if tr.has_dd() else None)
        res = bench.parity_gate(_OracleAsEngine(o, h), pkg, config, room_ids, nb, 1.0, ingress, tr, 3, zero, tot)
        assert not res["parity"] and res["downtracks_differing"] >= 1
    finally:
        o.destroy(h)
        tr.close()
