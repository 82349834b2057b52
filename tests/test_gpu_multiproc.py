"""The real multi-process data-parallel path on one MI355X.

RCCL refuses two ranks on one GPU (profiles/multirank_probe_r2.md), so these runs use the engine's
IPC transport (csrc/comm/ipc.h): each rank exports a window, the peers map it, and the collective
Plans run as pulls between per-rank flag barriers. Everything else is the production N > 1 path in
separate processes: bench.py's self-launch (torch.distributed.run), the rank bootstrap, GradSync's
steal-mode gather on the comm stream, late 3x3 weight gradients, per-bucket algorithm selection
(parallel/autotune.py) and the N > 1 JSON aggregation.

Checks: one JSON line with n_gpus 2 / comm_world 2; parameters, fp32 masters and gradients
bitwise equal on both ranks after the steps; gradients and weight updates match a one-process
oracle that runs the two ranks' batches as micro-batches (gradient accumulation, averaged) within
the teacher-forced 2e-2 bound -- BatchNorm statistics are per rank in data parallelism, so a single
batch-64 pass would be a different computation; and a rank killed mid-step makes the job fail with
a non-zero status instead of hanging. Reference: /root/reference/src/main.py:208-213,329-331,
/root/reference/submit.sh:64.
"""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

BATCH, STEPS = 32, 3


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["DLA_COMM_TIMEOUT_S"] = "60"
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_ipc_engine_two_processes(cuda):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ipc_engine_check.py"), "--ranks", "2",
                        "--same_device", "1", "--timeout", "200"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    if r.returncode != 0:  # pytest truncates long assertion messages: print the child's output in full first
        print(r.stdout[-6000:])
        print(r.stderr[-6000:], file=sys.stderr)
    assert r.returncode == 0, r.returncode
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["ok"] and rec["world"] == 2 and rec["checked"] >= 100, rec
    # every regrow cycle mapped a new window generation whose nonce every peer read back (or re-allocated)
    assert rec["regrow_cycles"] >= 8 and rec["window_generation"] >= rec["regrow_cycles"], rec
    print("ipc check:", {k: rec[k] for k in ("checked", "window_generation", "stale_mappings_refused")})


@pytest.fixture(scope="module")
def two_rank_run(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = tmp_path_factory.mktemp("dp2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same_device", "1", "--batch", str(BATCH),
           "--steps", str(STEPS), "--warmup", "0", "--check_dir", str(d), "--launch_timeout", "220"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=260, env=_env(), cwd=ROOT)
    return r, d


def test_bench_two_ranks_json(two_rank_run):
    r, _ = two_rank_run
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["comm_world"] == 2
    assert rec["config"]["transport"] == "ipc" and rec["config"]["same_device"]
    assert rec["config"]["global_batch"] == 2 * BATCH
    assert rec["allreduce_table"]["verified"], rec["allreduce_table"]
    assert any(rec["allreduce_table"]["verified"].values())
    assert rec["allreduce_ms_per_step"] > 0.0
    assert rec["value"] > 0 and rec["steps"] == STEPS


def _load(d, r):
    return torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True)


def test_ranks_bitwise_equal(two_rank_run):
    r, d = two_rank_run
    assert r.returncode == 0, r.stderr[-3000:]
    a, b = _load(d, 0), _load(d, 1)
    for key in ("params", "masters", "grads"):
        assert a[key].keys() == b[key].keys() and a[key], key
        for n in a[key]:
            assert torch.equal(a[key][n], b[key][n]), f"{key} {n} differs between ranks"


def _rel(x, y):
    x, y = x.double(), y.double()
    return float((x - y).norm() / y.norm().clamp_min(1e-30))


def test_matches_one_process_microbatch_oracle(two_rank_run, cuda):
    """One process, the same init, each step the two ranks' batches as micro-batches, gradients
    summed and halved -- data parallelism with per-rank BatchNorm, computed without communication."""
    r, d = two_rank_run
    assert r.returncode == 0, r.stderr[-3000:]
    sys.path.insert(0, ROOT)
    from distributed_learning_amd.data import SyntheticBatches
    from distributed_learning_amd.models import get_spec
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.optim import FusedSGD

    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        _oracle_steps(got_dir=d, cuda=cuda)
    finally:
        dnn.set_native_conv(False)
        dnn.set_backend("torch")


def _oracle_steps(got_dir, cuda):
    from distributed_learning_amd.data import SyntheticBatches
    from distributed_learning_amd.models import get_spec
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.optim import FusedSGD

    d = got_dir
    spec = get_spec("resnet50")
    torch.manual_seed(1234)
    model = spec.build().to(cuda).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    init = {n: p.detach().float().clone() for n, p in model.named_parameters()}
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.5, master_weights=True)
    data = [SyntheticBatches(BATCH, spec.input_shape, spec.num_classes, cuda, dtype=torch.bfloat16, seed=1234,
                             rank=rr, channels_last=True) for rr in range(2)]
    for _ in range(STEPS):
        opt.zero_grad(set_to_none=True)
        for rr in range(2):
            x, y = data[rr].next()
            cross_entropy(model(x), y).backward()
        torch.cuda.synchronize()
        for p in model.parameters():
            if p.grad is not None:
                p.grad.mul_(0.5)
        opt.step()
    torch.cuda.synchronize()
    got = _load(d, 0)
    worst_g, worst_u = 0.0, 0.0
    for n, p in model.named_parameters():
        g_ref = p.grad.detach().float().cpu()
        worst_g = max(worst_g, _rel(got["grads"][n].float(), g_ref))
        # fp32 masters for the bf16 weights; BatchNorm affine parameters are fp32 themselves
        m_ref = opt.state[p].get("master", p).detach().float().cpu()
        upd_ref = m_ref - init[n].cpu()
        upd = got["masters"].get(n, got["params"][n]).float() - init[n].cpu()
        if float(upd_ref.norm()) > 0:
            worst_u = max(worst_u, _rel(upd, upd_ref))
    assert worst_g <= 2e-2, worst_g
    assert worst_u <= 2e-2, worst_u


def test_killed_rank_fails_the_job(cuda):
    t0 = time.time()
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same_device", "1", "--batch", "16",
           "--steps", "4", "--warmup", "1", "--fail_rank", "1", "--fail_step", "2", "--algorithm", "ipc_direct",
           "--bucket_mb", "8", "--launch_timeout", "150"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=200, env=_env(), cwd=ROOT)
    assert r.returncode != 0
    assert "injected failure" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert time.time() - t0 < 190


def test_graph_capture_refused_on_ipc_transport(cuda):
    """the IPC barrier tokens are host-side launch arguments, so a replayed HIP graph would
    pass every barrier at once. bench.py refuses --graph on with the IPC transport before any step runs (and
    CommEngine.allreduce_ipc refuses a capturing stream)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same_device", "1", "--batch", "8",
           "--steps", "1", "--warmup", "0", "--graph", "on", "--launch_timeout", "150"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=200, env=_env(), cwd=ROOT)
    assert r.returncode != 0
    assert "cannot capture the IPC transport" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
