"""Race detection by deterministic replay: the concurrent run (compute stream +
high-priority comm stream, event-ordered) must be bitwise identical to a fully serialised run
(AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING=1) of the same training steps (gpu)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(out, extra_env):
    env = dict(os.environ)
    env.update(extra_env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):  # a world of one, own rendezvous
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "race_replay.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=55)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return torch.load(out, weights_only=True)


def test_concurrent_run_matches_serialised_replay(cuda, tmp_path):
    a = _run(tmp_path / "concurrent.pt", {})
    b = _run(tmp_path / "serial.pt", {"AMD_SERIALIZE_KERNEL": "3", "HIP_LAUNCH_BLOCKING": "1"})
    assert a.keys() == b.keys()
    assert torch.isfinite(a["__losses__"]).all()
    diff = [k for k in a if not torch.equal(a[k], b[k])]
    assert not diff, f"{len(diff)} tensors differ between concurrent and serialised runs: {diff[:8]}"
