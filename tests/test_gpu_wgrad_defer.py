"""Late-joined weight gradients (ops/conv.py WGRAD_DEFER): the side-stream schedule must give the same
gradients as the inline one, bit for bit (same kernels, same operands, fixed-order reductions), under
both join points, with gradient accumulation (inline fallback) and through the DP wrapper's hooks."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture
def native(cuda):
    from distributed_learning_amd.ops import conv
    from distributed_learning_amd.ops import nn as dnn

    dnn.set_backend("native")
    dnn.set_native_conv(True)
    # the one-pass 1x1 kernel (DUAL_1X1) computes a weight gradient only when it is not deferred, so with it
    # an inline schedule and an "all" schedule run different weight-gradient kernels: these tests compare the
    # deferral itself, on the separate kernels
    old = conv.DUAL_1X1
    conv.DUAL_1X1 = False
    yield
    conv.DUAL_1X1 = old
    dnn.set_backend("torch")
    dnn.set_native_conv(False)


def _model():
    from distributed_learning_amd import models
    from distributed_learning_amd.ops import nn as dnn

    torch.manual_seed(1234)
    m = models.resnet50().to(DEV).to(memory_format=torch.channels_last)
    dnn.bf16_weights(m)
    return m


def _grads(model, defer, join, steps=1, batch=16):
    from distributed_learning_amd.ops import conv
    from distributed_learning_amd.ops.loss import cross_entropy

    old = conv.WGRAD_DEFER, conv.WGRAD_JOIN
    conv.WGRAD_DEFER, conv.WGRAD_JOIN = defer, join
    try:
        g = torch.Generator().manual_seed(5)
        x = torch.rand(batch, 3, 224, 224, generator=g).to(DEV, torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (batch,), generator=g).to(DEV)
        for p in model.parameters():
            p.grad = None
        for _ in range(steps):  # steps > 1: the second backward accumulates into existing grads
            cross_entropy(model(x), y).backward()
        assert not conv.side_pending(DEV), "compute stream did not join the side stream by the end of backward"
        torch.cuda.synchronize()
        return [p.grad.detach().clone() for p in model.parameters()]
    finally:
        conv.WGRAD_DEFER, conv.WGRAD_JOIN = old


@pytest.mark.parametrize("defer,join", [("3x3", "end"), ("auto", "end"), ("all", "end"), ("all", "conv")])
def test_deferred_wgrad_bitwise(native, defer, join):
    m = _model()
    ref = _grads(m, "0", "end")
    got = _grads(m, defer, join)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), f"parameter {i}: deferred weight gradient differs"


def test_deferred_wgrad_accumulation(native):
    m = _model()
    ref = _grads(m, "0", "end", steps=2)
    got = _grads(m, "all", "end", steps=2)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), f"parameter {i}: accumulated gradient differs"


def test_deferred_wgrad_through_dp_hooks(native):
    """The DP wrapper's post-accumulate hooks fire while the weight gradients are still on the side
    stream; with the forced multi-rank data path the native executor must make the collective wait."""
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.parallel import PipelinedFusedDP, make_reducer
    from distributed_learning_amd.parallel import context as ctxmod
    from distributed_learning_amd.parallel.executor import NativeStreamExecutor
    from distributed_learning_amd.ops import conv

    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    ctxmod.init(backend="nccl")
    results = []
    for defer in ("0", "all"):
        base = _model()
        reducer = make_reducer("immediate", "builtin", native=True)
        model = PipelinedFusedDP(base, reducer, 8 << 20, broadcast=False)
        model.sync.executor = NativeStreamExecutor(reducer.engine, "builtin", passthrough=False)
        model.sync.passthrough = False
        reducer.engine.impl.set_force(True)
        model.sync.executor.reserve(model.sync.buckets)
        old = conv.WGRAD_DEFER
        conv.WGRAD_DEFER = defer
        try:
            g = torch.Generator().manual_seed(5)
            x = torch.rand(16, 3, 224, 224, generator=g).to(DEV, torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            y = torch.randint(0, 1000, (16,), generator=g).to(DEV)
            for p in base.parameters():
                p.grad = None
            cross_entropy(model(x), y).backward()
            model.sync_gradients()
            torch.cuda.synchronize()
            results.append([p.grad.detach().clone() for p in base.parameters()])
        finally:
            conv.WGRAD_DEFER = old
            model.cleanup()
    ctxmod.shutdown()
    for i, (a, b) in enumerate(zip(results[1], results[0])):
        assert torch.equal(a, b), f"parameter {i}: gradient after the collective differs"


def test_torch_ddp_blocks_deferral(native):
    """torch DDP copies gradients into its buckets inside backward without joining the side stream
    (ADVICE r3): while a TorchDDP wrapper lives no weight gradient is deferred, so its all-reduced
    gradients equal the inline ones bit for bit."""
    from distributed_learning_amd.ops import conv
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.parallel import context as ctxmod
    from distributed_learning_amd.parallel.wrappers import TorchDDP

    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    ctxmod.init(backend="nccl")
    ref = _grads(_model(), "0", "end")
    old = conv.WGRAD_DEFER
    conv.WGRAD_DEFER = "all"
    base = _model()
    ddp = TorchDDP(base, grouping_size=8 << 20, find_unused_parameters=False)
    try:
        assert conv._DEFER_BLOCKS[0] > 0
        g = torch.Generator().manual_seed(5)
        x = torch.rand(16, 3, 224, 224, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (16,), generator=g).to(DEV)
        cross_entropy(ddp(x), y).backward()
        torch.cuda.synchronize()
        got = [p.grad.detach().clone() for p in base.parameters()]
    finally:
        conv.WGRAD_DEFER = old
        ddp.cleanup()
        ctxmod.shutdown()
    assert conv._DEFER_BLOCKS[0] == 0
    for i, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), f"parameter {i}: DDP gradient differs from the inline one"


def test_shared_weight_deferred_once(native):
    """A conv weight used twice in one graph is deferred at most once: the second use
    joins the first and runs inline, so autograd's sum of the two is taken over finished tensors."""
    import torch.nn as nn

    from distributed_learning_amd.ops import conv
    from distributed_learning_amd.ops import nn as dnn

    torch.manual_seed(3)

    class Twice(nn.Module):
        def __init__(self):
            super().__init__()
            self.c = nn.Conv2d(64, 64, 3, padding=1, bias=False)

        def forward(self, x):
            y, _ = conv.conv3x3(x, self.c)
            y, _ = conv.conv3x3(torch.relu(y), self.c)
            return y

    def run(defer):
        torch.manual_seed(3)
        m = Twice().to(DEV).to(memory_format=torch.channels_last)
        dnn.bf16_weights(m)
        x = torch.randn(8, 64, 56, 56, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        old = conv.WGRAD_DEFER
        conv.WGRAD_DEFER = defer
        try:
            m(x).float().square().mean().backward()
            assert not conv.side_pending(DEV)
            torch.cuda.synchronize()
            return m.c.weight.grad.detach().clone()
        finally:
            conv.WGRAD_DEFER = old

    assert torch.equal(run("all"), run("0"))
