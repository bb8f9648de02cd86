"""bench.py --gpus N launches its own N ranks (one child torch.distributed.run, no external torchrun) and
rank 0 reports n_gpus / parallelism / global_batch from the real world size -- checked with the gloo/CPU
stub step (the GPU path is the same launcher with the nccl backend)."""

import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("n", [1, 2])
def test_bench_launches_n_ranks(n):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--stub-cpu", "--steps", "3",
                        "--warmup", "1", "--batch", "4"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}"
    assert d["config"]["global_batch"] == 4 * n and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0
