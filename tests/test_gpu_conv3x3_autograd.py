"""3x3 conv autograd wrapper (ops/conv.py::_Conv3x3) under every engine policy (gpu)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fwd", ["native", "miopen"])
@pytest.mark.parametrize("stride,cin", [(1, 64), (1, 128), (2, 128)])
def test_conv3x3_autograd_policies(cuda, fwd, stride, cin):
    from distributed_learning_amd.ops import conv as nconv

    torch.manual_seed(0)
    conv = nn.Conv2d(cin, 128, 3, stride, 1, bias=False).to(cuda).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(4, cin, 20, 20, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    old = dict(nconv.CONV3_POLICY)
    nconv.CONV3_POLICY.update(fwd=fwd, dgrad_native_max_cin=10**9 if fwd == "native" else 0)
    try:
        x1 = x.clone().requires_grad_(True)
        y, stats = nconv.conv3x3(x1, conv, want_stats=True)
        g = torch.randn(y.shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y.backward(g)
    finally:
        nconv.CONV3_POLICY.clear()
        nconv.CONV3_POLICY.update(old)
    xr = x.float().requires_grad_(True)
    wr = conv.weight.detach().float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, stride, 1)
    yr.backward(g.float())
    rel = lambda a, b: float((a.float() - b).norm() / b.norm())  # noqa: E731
    assert rel(y, yr.detach()) < 1e-2
    assert rel(x1.grad, xr.grad) < 2e-2
    assert rel(conv.weight.grad, wr.grad) < 2e-2
    assert conv.weight.grad.dtype == torch.bfloat16
    assert stats is not None  # want_stats forces the native forward
