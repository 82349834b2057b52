"""``bench.py --gpus N`` launches N ranks itself.

The driver runs ``python3 bench.py --gpus N`` as a plain command; without a WORLD_SIZE in the environment
the bench must start N rank processes (as ``mpirun -npernode`` does for the reference,
/root/reference/submit.sh:64) and must never report a 1-GPU number for an N-GPU request.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    return env


@pytest.mark.slow
@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launches_n_ranks(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry_run", "1"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n
    assert sorted(j["rank"] for j in rec["ranks_joined"]) == list(range(n))
    assert len({j["pid"] for j in rec["ranks_joined"]}) == n  # n distinct processes


def test_bench_refuses_more_gpus_than_present():
    import torch

    if torch.cuda.device_count() >= 64:
        pytest.skip("node has that many GPUs")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode != 0
    assert "refusing to measure fewer" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
