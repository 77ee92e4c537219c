"""bench.py's multi-GPU launcher, rehearsed on the CPU.

`python bench.py --gpus 2` with no torch.distributed environment must start
two ranks itself (the parent touches no GPU), shard the rooms, run the room
manager's summary all-gathers every 400 ms of media inside the loop, reduce
the time over ranks and print one line with n_gpus = 2.  `--dry-run` puts the
CPU oracle (tests/dryrun_engine.py) behind the engine methods and uses gloo,
so the launcher, the room plan, the gathers and the parity reduction are
exercised here; the forwarded totals of the two ranks must equal one process
forwarding all their rooms.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("config,rooms", [(1, 1), (3, 1)])
def test_launcher_two_ranks_matches_one_process(config, rooms):
    common = ["--dry-run", "--config", str(config), "--steps", "2", "--warmup", "1", "--cpu-threads", "2"]
    two = _bench("--gpus", "2", "--rooms", str(rooms), *common)
    one = _bench("--gpus", "1", "--rooms", str(2 * rooms), "--no-cpu-baseline", *common)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["dry_run"] is True
    assert two["parity"] is True and two["parity_gate"]["parity_all_ranks"] is True
    assert two["forwarded_total"] == one["forwarded_total"] > 0
    c = two["collective"]
    assert c["update_ms"] == 400.0
    # 3 s of media: ticks at 0.4 .. 2.8 s, 5 of them after the 1-s warmup batch
    assert c["ticks"] == 7 and c["ticks_in_timed_region"] == 5
    assert c["rooms_gathered"] == 2 * rooms
    assert c["subscribers_gathered"] > 0
    if config == 3:  # the audio-heavy config ranks speakers
        assert c["rooms_with_speakers"] > 0
    cb = two["cpu_baseline"]
    assert cb["cores"] % 2 == 0 and cb["value"] > 0 and cb["per_rank_value"] > 0  # (threads used x 2 ranks)


def test_tick_times():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.tick_times(0, 1.0, 400) == pytest.approx([0.4, 0.8])
    assert bench.tick_times(1, 1.0, 400) == pytest.approx([1.2, 1.6, 2.0])
    assert bench.tick_times(2, 1.0, 400) == pytest.approx([2.4, 2.8])
    assert bench.tick_times(0, 0.01, 400) == []
    assert bench.tick_times(39, 0.01, 400) == pytest.approx([0.4])
    assert bench.tick_times(3, 1.0, 0) == []
