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


# ---- control paths between batches (padding, blank frames, AllocateOptimal,
# RED, stream trackers, NACK lookups) on one trace: one digest per step ----
CONTROL_CASES = [
    ("control_config2", dict(config=2, duration_s=3.0, batch_s=0.25, rooms=2, seed=23)),
    # + Pause / GetNextHigherTransition / AllocateNextHigher and frame trackers
    ("control_config2_alloc", dict(config=2, duration_s=3.0, batch_s=0.25, rooms=2, seed=29)),
]


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def run_control_case(api, h, trace, workload, drain_fn, run_fn, abi, name="control_config2"):
    """Drives `trace` with control calls between its batches; returns the fixture dict."""
    from tests import pad_lib, red_lib, rtx_lib, tracker_lib
    from tests.test_alloc_gpu import make_alloc_reqs, run_step, stream_allocator_steps, video_mask
    ext = name.endswith("_alloc")
    workload.load_topology(api, h, trace)
    ids = tracker_lib.add_trackers(api, h, trace, seed=11)
    fids = tracker_lib.add_frame_trackers(api, h, trace, seed=12) if ext else None
    m = red_lib.opus_map(trace)
    out = {"steps": []}
    epoch = 1700000000 * 10**9
    for b in range(trace.nbatches):
        now = epoch + int(b * 0.25e9)
        if b % 4 == 1:  # padding probe
            reqs = pad_lib.make_reqs(trace.ndts, seed=b, frac=0.5)
            rec, war, sent = pad_lib.pad(api, h, reqs, now)
            out["steps"].append(["padding", b, int(len(rec)), _sha(rec, war, sent)])
        if b % 4 == 2:  # allocation
            reqs = make_alloc_reqs(abi, trace.ndts, seed=b)
            a = np.zeros(len(reqs), dtype=abi.ALLOCATION_DTYPE)
            assert api["allocate_optimal"](h, reqs.ctypes.data, len(reqs), a.ctypes.data) == 0
            out["steps"].append(["allocate", b, int(len(a)), _sha(a)])
        if ext and b >= 1:  # the stream allocator's pause / probe calls
            for k, step in enumerate(stream_allocator_steps(abi, trace.ndts, min(b, 9), video_mask(abi, trace))):
                r = run_step(api, h, abi, step)
                out["steps"].append([step[0], b, int(len(r)), _sha(r)])
        if b % 4 == 3:  # blank frames
            reqs = pad_lib.make_reqs(trace.ndts, seed=100 + b, frac=0.3)
            rec, war, _ = pad_lib.pad(api, h, reqs, now, blank=True)
            out["steps"].append(["blank", b, int(len(rec)), _sha(rec, war)])
        workload.queue_events(api, h, trace, b)
        pk, n, ar, alen = trace.batch(b)
        run_fn(pk, n, ar, alen)
        rec, war = drain_fn()
        out["steps"].append(["batch", b, int(len(rec)), _sha(records_digest(rec) if len(rec) else "", war)])
        pkts, n2, arena, alen2 = red_lib.batch_arrays(trace, b)
        rp, k, rar = red_lib.red(api, h, "red_encode", pkts, n2, arena, alen2, m)
        keep = np.arange(k) % 4 != 2
        lp, lk = red_lib.drop(rp, k, keep)
        dp, dk, dar = red_lib.red(api, h, "red_decode", lp, lk, rar, len(rar), m)
        out["steps"].append(["red", b, int(k), int(dk), _sha(rp, rar, dp, dar)])
        if b % 2 == 1:
            t = tracker_lib.tick(api, h, ids, True, 500_000_000 if b % 4 == 3 else 0)
            t = t[["tracker", "status", "bitrate_changed", "notifications", "bitrate", "cumulative"]]
            out["steps"].append(["trackers", b, int(len(t)), _sha(t.tobytes())])
        if ext:
            t = tracker_lib.tick_at(api, h, fids, b % 2 == 0, 10**9 if b % 4 == 0 else 0, now + int(0.25e9))
            t = t[["tracker", "status", "bitrate_changed", "notifications", "bitrate", "cumulative"]]
            out["steps"].append(["frame_trackers", b, int(len(t)), _sha(t.tobytes())])
    nacks = rtx_lib.make_nacks(api, h, trace, seed=3)
    r = rtx_lib.rtx_lookup(api, h, nacks, epoch + int(trace.nbatches * 0.25e9) + 10**8)
    out["steps"].append(["rtx", trace.nbatches, int(len(r)), _sha(r)])
    out["state_sha256"] = state_digest(api, h, trace.ndts, abi)
    return out
