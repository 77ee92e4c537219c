"""Golden-vector digests shared by tests/golden/make_golden.py and the tests.

A golden case = one synthetic trace (BASELINE.json config shape at a size the
CPU oracle finishes in seconds).  Its fixture holds, per batch, the drop/forward
counters, the number of output records and SHA-256 digests of the record fields
and of the wire bytes; plus a digest of every DownTrack's exported Forwarder
state at the end.  Fixtures were produced by the CPU oracle (oracle/, pinned by
oracle/kat.cpp) and let the engine be checked against committed data without
running the oracle.
"""
import ctypes as C
import hashlib
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# (name, Trace kwargs) — keep each case to a few seconds of oracle time
CASES = [
    ("config1_3s", dict(config=1, duration_s=3.0, batch_s=1.0)),
    ("config2_2rooms", dict(config=2, duration_s=3.0, batch_s=0.5, rooms=2)),
    ("config2_loss25", dict(config=2, duration_s=2.0, batch_s=0.25, rooms=1, loss=0.25, reorder=0.2, seed=91)),
    ("config2_nocb", dict(config=2, duration_s=2.0, batch_s=0.1, rooms=1, has_callbacks=0)),
    ("config3_1room", dict(config=3, duration_s=2.0, batch_s=1.0, rooms=1)),
    ("config4_64subs", dict(config=4, duration_s=1.0, batch_s=0.5, rooms=1, participants=64)),
    ("config5_4rooms", dict(config=5, duration_s=3.0, batch_s=0.5, rooms=4)),
    ("config5_vp9only", dict(config=5, duration_s=2.0, batch_s=0.5, rooms=3, svc_dd=0)),
    ("config5_dd_loss", dict(config=5, duration_s=3.0, batch_s=0.25, rooms=2, loss=0.15, reorder=0.1, seed=17)),
]

RECORD_FIELDS = ("ext_sn", "ext_ts", "out_off", "dt", "pkt", "out_len", "flags", "layer")


def records_digest(rec):
    h = hashlib.sha256()
    for f in RECORD_FIELDS:
        h.update(np.ascontiguousarray(rec[f]).tobytes())
    return h.hexdigest()


def state_digest(api, h, ndts, abi):
    d = hashlib.sha256()
    for dt in range(ndts):
        st = abi.lkf_fwd_state()
        rc = api["get_state"](h, dt, C.byref(st))
        assert rc == 0, rc
        d.update(repr(st.as_tuple()).encode())
    return d.hexdigest()


def batch_entry(stats, rec, ar):
    return {
        "stats": stats,
        "n_out": int(len(rec)),
        "arena_len": int(len(ar)),
        "records_sha256": records_digest(rec) if len(rec) else "",
        "wire_sha256": hashlib.sha256(np.ascontiguousarray(ar).tobytes()).hexdigest() if len(ar) else "",
    }


def path(name):
    return os.path.join(GOLDEN_DIR, name + ".json")


def load(name):
    with open(path(name)) as f:
        return json.load(f)


def run_case(api, h, trace, workload, stats_fn, drain_fn, run_fn, abi):
    """Drives one trace through an lkf_*-shaped engine; returns the fixture dict.
    run_fn(pk, n, ar, alen, dd): dd = the lkf_pkt_dd side array pointer of the
    batch (dependency-descriptor traces) or None."""
    workload.load_topology(api, h, trace)
    has_dd = trace.has_dd()
    out = {"batches": []}
    for b in range(trace.nbatches):
        workload.queue_events(api, h, trace, b)
        pk, n, ar, alen = trace.batch(b)
        run_fn(pk, n, ar, alen, trace.batch_dd(b)[0] if has_dd else None)
        rec, war = drain_fn()
        out["batches"].append(dict(batch_entry(stats_fn(), rec, war), n_pkts=int(n)))
    out["state_sha256"] = state_digest(api, h, trace.ndts, abi)
    out["ndts"] = int(trace.ndts)
    return out
