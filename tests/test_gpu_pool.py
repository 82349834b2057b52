"""NHWC max-pool kernels vs PyTorch's max_pool2d in fp32 (gpu)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,k,s,p,ceil", [
    ((4, 64, 112, 112), 3, 2, 1, False),   # ResNet stem
    ((2, 64, 112, 112), 3, 2, 0, True),    # GoogLeNet maxpool1
    ((2, 480, 28, 28), 3, 1, 1, True),     # inception branch4
    ((2, 832, 14, 14), 2, 2, 0, True),     # GoogLeNet maxpool4
    ((3, 24, 9, 13), 3, 2, 1, False),
])
def test_maxpool_matches_torch(cuda, dtype, shape, k, s, p, ceil):
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.pool import max_pool2d

    torch.manual_seed(0)
    # distinct values: no ties, so the argmax (hence the gradient routing) is unambiguous
    n = torch.tensor(shape).prod().item()
    x = (torch.randperm(n, device=cuda).float() / n).reshape(shape).to(dtype)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    xr = x.detach().float().clone().requires_grad_(True)
    dnn.set_backend("native")
    try:
        y = max_pool2d(x, k, s, p, 1, ceil)
    finally:
        dnn.set_backend("torch")
    yr = F.max_pool2d(xr, k, s, p, 1, ceil)
    assert y.shape == yr.shape
    torch.testing.assert_close(y.float(), yr, rtol=0, atol=0)
    g = torch.randn(y.shape, device=cuda).to(dtype)
    y.backward(g)
    yr.backward(g.float())
    tol = dict(rtol=1e-2, atol=1e-2) if dtype == torch.bfloat16 else dict(rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)


def test_maxpool_nan_propagates(cuda):
    from distributed_learning_amd.ops import _ext

    x = torch.zeros(1, 8, 4, 4, device=cuda).contiguous(memory_format=torch.channels_last)
    x[0, 3, 1, 1] = float("nan")
    y, _ = _ext.require().maxpool_fwd(x, 2, 2, 0, False, True)
    assert torch.isnan(y[0, 3, 0, 0]) and not torch.isnan(y[0, 2, 0, 0])
