"""Bit-exact parity at the sizes the bench and the configs are quoted on.

The engine and the CPU oracle take the same full-size traces: configs[1] at the
benched size (100 rooms x 10 participants, 18,000 DownTracks, 1-s batches),
configs[3] at its full fan-out (one publisher to 5,000 subscribers) and
configs[2] at one GPU's full shard (125 rooms x 50 participants, ~337 k
DownTracks) and configs[4] at 2,000 rooms (the SVC / dependency-descriptor
path).  Every record, every wire byte, every counter, every exported
Forwarder state and sequencer probes must be identical.
"""
import pytest

from tests.test_parity_gpu import run_parity

pytestmark = pytest.mark.gpu


def test_config2_bench_size(pkg, workload, abi):
    """configs[1] exactly as bench.py runs it: 100 rooms, 1-s batches, 3 s + tail."""
    tr = workload.Trace(2, duration_s=3.0, batch_s=1.0, rooms=100)
    assert tr.ndts == 18000 and tr.nbatches >= 4
    t = run_parity(pkg, workload, abi, tr)
    assert t["forwarded"] > 3_000_000


def test_config4_full_fanout(pkg, workload, abi):
    """configs[3]: 1 publisher x 5,000 subscribers (10,000 DownTracks), with the state check."""
    tr = workload.Trace(4, duration_s=2.0, batch_s=1.0, rooms=1, participants=5000)
    t = run_parity(pkg, workload, abi, tr)
    assert t["forwarded"] > 2_000_000


def test_config3_full_shard(pkg, workload, abi):
    """configs[2] on one GPU's shard: 125 rooms x 50 participants (audio-heavy)."""
    tr = workload.Trace(3, duration_s=2.0, batch_s=1.0, rooms=125)
    assert tr.ndts > 300000
    t = run_parity(pkg, workload, abi, tr)
    assert t["forwarded"] > 25_000_000


def test_config5_full_shard(pkg, workload, abi):
    """configs[4] at its specified size: 2,000 rooms x 5 participants, VP9 / AV1
    L3T3 SVC with dependency descriptors (the DD decide path), 1-s batches."""
    tr = workload.Trace(5, duration_s=1.0, batch_s=1.0, rooms=2000)
    assert tr.ndts >= 2000 * 5 * 4
    t = run_parity(pkg, workload, abi, tr, seq_probe=False)
    assert t["forwarded"] > 1_000_000
