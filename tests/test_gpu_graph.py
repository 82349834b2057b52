"""Whole-step HIP graph capture (parallel/graphs.py) reproduces eager training (gpu)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graphed: bool, steps: int, world1, arch: str = "resnet18", force: bool = False):
    from distributed_learning_amd.data import SyntheticBatches
    from distributed_learning_amd.models import googlenet, resnet18
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.optim import FusedSGD
    from distributed_learning_amd.parallel import PipelinedFusedDP, make_reducer
    from distributed_learning_amd.parallel.graphs import GraphedStep

    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    batch = 16
    if arch == "googlenet":  # aux heads computed but unused (zero-filled grads), ceil-mode pools, torch.cat
        m = googlenet(10).to(dev).to(memory_format=torch.channels_last)
        m.dropout.p = 0.0  # the main-path dropout would make eager and replayed RNG streams matter
        shape = (3, 64, 64)
    elif arch == "resnet50":  # batch 24 at 224: the stage-1 one-pass 1x1 kernels and the BN hand-off engage
        from distributed_learning_amd.models import resnet50

        m = resnet50(10).to(dev).to(memory_format=torch.channels_last)
        shape, batch = (3, 224, 224), 24
    else:
        m = resnet18(10).to(dev).to(memory_format=torch.channels_last)
        shape = (3, 32, 32)
    dnn.bf16_weights(m)
    red = make_reducer("immediate", "builtin", native=True)
    w = PipelinedFusedDP(m, red, 1 << 20, dev, broadcast=False)
    if force:  # the multi-rank data path (gather -> fp32 staging -> ncclAllReduce -> cast) as graph nodes
        from distributed_learning_amd.parallel.executor import NativeStreamExecutor

        red.engine.impl.set_force(True)
        red.engine.set_accum_fp32(True)
        w.sync.executor = NativeStreamExecutor(red.engine, "builtin", passthrough=False)
        w.sync.passthrough = False
        w.sync.executor.reserve(w.sync.buckets)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, master_weights=True)
    data = SyntheticBatches(batch, shape, 10, dev, dtype=torch.bfloat16, channels_last=True, device_step=True)

    def step():
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(w(x), y)
        loss.backward()
        w.sync_gradients()
        opt.step()
        return loss.detach()

    runner = GraphedStep(step, warmup=2, device=dev) if graphed else step
    losses = []
    n = steps if graphed else steps + 2  # the graph runner does 2 eager warmup steps first
    for _ in range(n):
        losses.append(float(runner()))
    if graphed:
        assert runner.captured
    w.cleanup()
    if force:
        red.engine.impl.set_force(False)
        red.engine.set_accum_fp32(False)
    return losses, [p.detach().float().clone() for p in m.parameters()]


@pytest.fixture(scope="module")
def world1(cuda):
    from distributed_learning_amd.parallel import context as ctx

    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    c = ctx.init(backend="nccl")
    yield c
    ctx.shutdown()


@pytest.mark.parametrize("arch", ["resnet18", "googlenet", "resnet50"])
def test_graphed_step_matches_eager(world1, arch):
    from distributed_learning_amd.ops import nn as dnn

    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        le, pe = _run(False, 5, world1, arch)
        lg, pg = _run(True, 5, world1, arch)
    finally:
        dnn.set_native_conv(False)
        dnn.set_backend("torch")
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det
    # eager: 7 steps; graphed: 2 eager warmups + 5 replays -> replays are steps 3..7
    assert lg == pytest.approx(le[2:], rel=1e-5, abs=1e-5)
    for a, b in zip(pe, pg):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_graphed_step_with_collectives_matches_eager(world1):
    """the captured step must contain real collective nodes. With --force_comm's
    data path every bucket is gathered into the fp32 staging buffer and all-reduced by a 1-rank
    ncclAllReduce on the comm stream; the graph (collectives, the engine's reserved scratch, the
    cross-stream joins) must replay to the eager result."""
    from distributed_learning_amd.ops import nn as dnn

    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        le, pe = _run(False, 5, world1, "resnet18", force=True)
        lg, pg = _run(True, 5, world1, "resnet18", force=True)
    finally:
        dnn.set_native_conv(False)
        dnn.set_backend("torch")
    assert lg == pytest.approx(le[2:], rel=1e-5, abs=1e-5)
    for a, b in zip(pe, pg):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
