"""The stream allocator's cooperative pass on the CPU oracle (the checker of
the GPU path): allocateAllTracks' greedy pass never hands a subscriber more
than its channel capacity when pausing is allowed, and every call of an
allocator tick (tests/prov_lib.py) runs on forwarded state; the restatement
itself is pinned by the four Provisional* tests of forwarder_test.go
(oracle/kat_sfu.inc, run by test_oracle_kat.py)."""
import numpy as np

from tests import prov_lib
from tests.oracle_lib import load as load_oracle


def _forward(o, h, tr, workload, b):
    workload.queue_events(o.api, h, tr, b)
    pk, n, ar, alen = tr.batch(b)
    o.run(h, pk, n, ar, alen, tr.batch_dd(b)[0] if tr.has_dd() else None)


def test_allocate_all_respects_capacity(pkg, workload):
    abi = pkg.abi
    o = load_oracle()
    tr = workload.Trace(2, duration_s=2.0, batch_s=1.0, rooms=3, seed=31)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        _forward(o, h, tr, workload, 0)
        rng = np.random.default_rng(5)
        kind, (g, reqs) = prov_lib.steps(tr, seed=9)[-1]
        assert kind == "allocate_all"
        g["allow_pause"] = 1
        g["allow_overshoot"] = 0
        g["capacity"] = rng.integers(0, 4_000_000, len(g))
        out = prov_lib.run(o.api, h, (kind, (g, reqs)))
        paused = 0
        for gr in g:
            a = out[gr["first"]:gr["first"] + gr["count"]]
            assert int(a["bandwidth_requested"].sum()) <= int(gr["capacity"])
            paused += int((a["target_spatial"] < 0).sum())
        assert paused > 0 and (out["target_spatial"] >= 0).sum() > 0
        _forward(o, h, tr, workload, 1)  # the next batch forwards on the committed targets
    finally:
        o.destroy(h)
        tr.close()


def test_allocator_tick_runs_on_oracle(pkg, workload):
    o = load_oracle()
    tr = workload.Trace(5, duration_s=2.0, batch_s=1.0, rooms=4, svc_dd=1, seed=32)
    h = o.create(500)
    try:
        workload.load_topology(o.api, h, tr)
        _forward(o, h, tr, workload, 0)
        res = [prov_lib.run(o.api, h, s) for s in prov_lib.steps(tr, seed=10)]
        coop = res[1]
        assert len(coop) and (coop["available"] == 1).all()
        assert any(r is not None and "is_candidate" in r.dtype.names and r["is_candidate"].any() for r in res)
        _forward(o, h, tr, workload, 1)
    finally:
        o.destroy(h)
        tr.close()
