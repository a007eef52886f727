"""bench.py --gpus N (BASELINE.json: 1/2/4/8 MI355X): run directly with N > 1 it starts N ranks
itself under torch.distributed.run (one process per GPU, the reference's one pipeline per queue,
ipfixprobe.cpp:381-464), and under a launcher WORLD_SIZE must equal N.  Driven here without a
GPU (--cpu-selftest: gloo), which also checks the N > 1 export exchange (shard.StreamGather):
rank 0 receives every rank's stream byte for byte, and exactly the streams' bytes."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True, timeout=300, env=e, cwd="/tmp")


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_starts_n_ranks_and_gathers_exact_streams(n):
    r = _run(["--gpus", str(n), "--cpu-selftest", "--steps", "5"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_ranks"] == n
    assert line["mismatches"] == []
    assert line["received_bytes"] == line["expected_bytes"] > 0  # no padding: exactly the streams
    assert line["header_bytes"] == 16 * n * 5


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--cpu-selftest"], env={"WORLD_SIZE": "3", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
