"""bench.py's multi-rank launch path (CPU): `--gpus N` without a launcher starts N ranks through
torch.distributed.run and the JSON line reports n_gpus = N; with fewer visible GPUs than asked it
exits non-zero before touching any GPU."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_gpus2_spawns_two_ranks():
    r = _run("--gpus", "2", "--steps", "3", "--dry-run")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] is True and rec["steps"] == 3


@pytest.mark.skipif(torch.cuda.device_count() >= 2, reason="needs a host with fewer than 2 GPUs")
def test_gpus2_refused_without_gpus():
    r = _run("--gpus", "2", "--steps", "3")
    assert r.returncode == 2
    assert "needs 2 visible GPUs" in r.stderr
