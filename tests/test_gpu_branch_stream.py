"""Downsample shortcut conv on the branch stream (ops/nn.py BRANCH_STREAM): outputs, BN running statistics
and every gradient must equal the single-stream schedule bit for bit (same kernels, same operands), with
autograd replaying the shortcut's backward on the branch stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture
def native(cuda):
    from distributed_learning_amd.ops import nn as dnn

    dnn.set_backend("native")
    dnn.set_native_conv(True)
    yield
    dnn.set_backend("torch")
    dnn.set_native_conv(False)


def _run(branch: bool, arch: str, steps: int = 2):
    from distributed_learning_amd import models
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy

    old = dnn.BRANCH_STREAM
    dnn.BRANCH_STREAM = branch
    try:
        torch.manual_seed(1234)
        m = getattr(models, arch)().to(DEV).to(memory_format=torch.channels_last)
        dnn.bf16_weights(m)
        g = torch.Generator().manual_seed(3)
        x = torch.rand(16, 3, 224, 224, generator=g).to(DEV, torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (16,), generator=g).to(DEV)
        outs = []
        for _ in range(steps):
            for p in m.parameters():
                p.grad = None
            out = m(x)
            cross_entropy(out, y).backward()
            outs.append(out.detach().clone())
        torch.cuda.synchronize()
        bufs = [b.detach().clone() for b in m.buffers()]
        return outs, [p.grad.detach().clone() for p in m.parameters()], bufs
    finally:
        dnn.BRANCH_STREAM = old


@pytest.mark.parametrize("arch", ["resnet50", "resnet18"])
def test_branch_stream_bitwise(native, arch):
    o0, g0, b0 = _run(False, arch)
    o1, g1, b1 = _run(True, arch)
    for a, b in zip(o1, o0):
        assert torch.equal(a, b)
    for i, (a, b) in enumerate(zip(g1, g0)):
        assert torch.equal(a, b), f"parameter {i}"
    for i, (a, b) in enumerate(zip(b1, b0)):
        assert torch.equal(a, b), f"buffer {i}"
