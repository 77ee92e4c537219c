"""Committed golden vectors (tests/golden/*.json, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture exactly (it is deterministic and its
behaviour is frozen by the fixtures as well as by the KATs).
GPU: the MI355X engine reproduces every fixture exactly, independently of the
oracle at run time.
"""
import ctypes as C
import importlib

import pytest

from tests import golden_lib
from tests.oracle_lib import load as load_oracle

CASE_NAMES = [c[0] for c in golden_lib.CASES]
CASE_KW = dict(golden_lib.CASES)


def _compare(got, want):
    assert len(got["batches"]) == len(want["batches"])
    for b, (g, w) in enumerate(zip(got["batches"], want["batches"])):
        for k in ("n_pkts", "stats", "n_out", "arena_len", "records_sha256", "wire_sha256"):
            assert g[k] == w[k], "batch %d %s: got %s want %s" % (b, k, g[k], w[k])
    assert got["state_sha256"] == want["state_sha256"]


@pytest.mark.parametrize("name", CASE_NAMES)
def test_oracle_matches_golden(name, workload, abi, pkg):
    want = golden_lib.load(name)
    assert want["trace"] == CASE_KW[name]
    o = load_oracle()
    tr = workload.Trace(**CASE_KW[name])
    h = o.create(500)
    try:
        def stats():
            st = abi.lkf_stats()
            o.api["get_stats"](h, C.byref(st))
            return st.as_dict()

        got = golden_lib.run_case(o.api, h, tr, workload, stats, lambda: pkg.drain_arrays(o.api, h),
                                  lambda pk, n, ar, alen, dd: o.run(h, pk, n, ar, alen, dd), abi)
    finally:
        o.destroy(h)
        tr.close()
    _compare(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASE_NAMES)
def test_engine_matches_golden(name, workload, abi, pkg):
    want = golden_lib.load(name)
    tr = workload.Trace(**CASE_KW[name])
    eng = pkg.Engine.for_trace(tr)
    try:
        def run(pk, n, ar, alen, dd):
            eng.submit(pk, n, ar, alen, dd)
            eng.run()
            eng.sync()

        got = golden_lib.run_case(eng.api, eng.h, tr, workload, eng.stats, eng.drain, run, abi)
    finally:
        eng.close()
        tr.close()
    _compare(got, want)


CONTROL_NAMES = [c[0] for c in golden_lib.CONTROL_CASES]
CONTROL_KW = dict(golden_lib.CONTROL_CASES)


def _compare_control(got, want):
    assert len(got["steps"]) == len(want["steps"])
    for g, w in zip(got["steps"], want["steps"]):
        assert g == w, "step %s: got %s want %s" % (w[:2], g, w)
    assert got["state_sha256"] == want["state_sha256"]


@pytest.mark.parametrize("name", CONTROL_NAMES)
def test_oracle_matches_control_golden(name, workload, abi, pkg):
    """padding, blank frames, AllocateOptimal, RED, stream trackers, NACK lookups between batches"""
    want = golden_lib.load(name)
    assert want["trace"] == CONTROL_KW[name]
    o = load_oracle()
    tr = workload.Trace(**CONTROL_KW[name])
    h = o.create(500)
    try:
        got = golden_lib.run_control_case(o.api, h, tr, workload, lambda: pkg.drain_arrays(o.api, h),
                                          lambda pk, n, ar, alen: o.run(h, pk, n, ar, alen), abi, name)
    finally:
        o.destroy(h)
        tr.close()
    _compare_control(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CONTROL_NAMES)
def test_engine_matches_control_golden(name, workload, abi, pkg):
    want = golden_lib.load(name)
    tr = workload.Trace(**CONTROL_KW[name])
    eng = pkg.Engine.for_trace(tr, headroom=3.5)
    try:
        def run(pk, n, ar, alen):
            eng.submit(pk, n, ar, alen)
            eng.run()
            eng.sync()

        got = golden_lib.run_control_case(eng.api, eng.h, tr, workload, eng.drain, run, abi, name)
    finally:
        eng.close()
        tr.close()
    _compare_control(got, want)
