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
    ((3, 16, 9, 7), 3, 1, 0, False),        # 3x3/s1 strips with remainders, no padding
    ((2, 24, 1, 5), 3, 1, 1, False),
    ((2, 832, 14, 14), 2, 2, 0, True),     # GoogLeNet maxpool4
    ((3, 24, 9, 13), 3, 2, 1, False),
    ((2, 16, 11, 11), 5, 2, 2, False),     # runtime window size (generic path)
    ((2, 16, 12, 10), 4, 3, 1, True),      # k = 4: generic forward, 2x2-window backward
    ((40, 256, 128, 128), 3, 1, 1, False),  # > 2^24 work items: hardware-division index path
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


def _pool_reference(x, k, s, p):
    """y and the first-maximum window position in row-major order, NaN winning (first NaN), fp32."""
    n, c, h, w = x.shape
    xp = F.pad(x.float(), (p, p, p, p), value=float("-inf"))
    win = xp.unfold(2, k, s).unfold(3, k, s).reshape(n, c, (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1, k * k)
    nan = torch.isnan(win)
    idx = torch.where(nan.any(-1), nan.float().argmax(-1), torch.nan_to_num(win, nan=0.0).argmax(-1))
    return torch.gather(win, -1, idx.unsqueeze(-1)).squeeze(-1), idx


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,p", [((2, 24, 10, 9), 1), ((3, 16, 7, 7), 0), ((2, 40, 15, 1), 1), ((1, 8, 29, 4), 1)])
def test_maxpool3s1_ties_nan_inf_positions(cuda, dtype, shape, p):
    """The separable 3x3/s1 forward: values and 1-byte argmax positions equal the row-major
    first-maximum scan, with ties, NaNs and -inf in the windows; strips of 7 rows with remainders."""
    from distributed_learning_amd.ops import _ext

    torch.manual_seed(3)
    x = torch.randint(0, 4, shape, device=cuda).float()
    r = torch.rand(shape, device=cuda)
    x[r < 0.02] = float("nan")
    x[(r >= 0.02) & (r < 0.05)] = float("-inf")
    x = x.to(dtype).contiguous(memory_format=torch.channels_last)
    y, pos = _ext.require().maxpool_fwd(x, 3, 1, p, False, True)
    yr, ir = _pool_reference(x, 3, 1, p)
    assert y.shape == yr.shape
    torch.testing.assert_close(y.float(), yr, rtol=0, atol=0, equal_nan=True)
    posr = ir.permute(0, 2, 3, 1).reshape(-1).to(torch.uint8)
    assert torch.equal(pos.permute(0, 2, 3, 1).reshape(-1).cpu(), posr.cpu())


@pytest.mark.parametrize("shape,k,s,p,ceil", [
    ((4, 64, 30, 30), 3, 2, 1, False),   # ResNet stem
    ((4, 64, 29, 29), 3, 2, 0, True),    # GoogLeNet maxpool1 (odd size: the ceil window is partial)
    ((2, 192, 15, 15), 3, 2, 0, True),   # GoogLeNet maxpool2
    ((2, 64, 14, 14), 3, 2, 0, True),    # ceil mode with an even size
])
def test_stem_bn_relu_maxpool_fused_matches_unfused(cuda, shape, k, s, p, ceil):
    """Fused stem op == separate fused-BN+ReLU then max-pool: identical pooled output, running
    statistics and (up to reduction order) gradients; floor and ceil mode."""
    import torch.nn as nn

    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.bn_act import fused_bn_act, fused_bn_relu_maxpool
    from distributed_learning_amd.ops.pool import MaxPool2d, max_pool2d

    torch.manual_seed(0)
    x = torch.randn(*shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    C = shape[1]
    bn1, bn2 = nn.BatchNorm2d(C, eps=1e-3).to(cuda), nn.BatchNorm2d(C, eps=1e-3).to(cuda)
    with torch.no_grad():
        bn1.weight.uniform_(0.5, 1.5)
        bn1.bias.uniform_(-0.5, 0.5)
    bn2.load_state_dict(bn1.state_dict())
    pool = MaxPool2d(k, s, p, ceil_mode=ceil)
    dnn.set_backend("native")
    try:
        x1 = x.clone().requires_grad_(True)
        y1 = fused_bn_relu_maxpool(x1, bn1, pool)
        x2 = x.clone().requires_grad_(True)
        y2 = max_pool2d(fused_bn_act(x2, bn2, True, None), k, s, p, ceil_mode=ceil)
    finally:
        dnn.set_backend("torch")
    assert y1.shape == y2.shape and torch.equal(y1, y2)
    assert y1.grad_fn is not None and "BNReluPool" in type(y1.grad_fn).__name__  # the fused op ran
    torch.testing.assert_close(bn1.running_mean, bn2.running_mean)
    torch.testing.assert_close(bn1.running_var, bn2.running_var)
    g = torch.randn_like(y1)
    y1.backward(g)
    y2.backward(g)
    # fp32 reference with the fused op's own pooling choice (ties broken identically): the fused
    # backward sums overlapping-window gradients in fp32, the unfused max-pool backward rounds that
    # sum to bf16 first, so the fused result must be at least as close to fp32
    xr = x.float().requires_grad_(True)
    bnr = nn.BatchNorm2d(C, eps=1e-3).to(cuda)
    bnr.load_state_dict({k: v for k, v in bn2.state_dict().items()})
    with torch.no_grad():
        bnr.weight.copy_(bn1.weight)
        bnr.bias.copy_(bn1.bias)
    yr = torch.nn.functional.max_pool2d(torch.relu(bnr(xr)), k, s, p, ceil_mode=ceil)
    yr.backward(g.float())
    err = lambda a, b: float((a.float() - b).norm() / b.norm())  # noqa: E731
    assert err(bn1.weight.grad, bnr.weight.grad) <= err(bn2.weight.grad, bnr.weight.grad) * 1.5 + 1e-3
    assert err(bn1.bias.grad, bnr.bias.grad) <= err(bn2.bias.grad, bnr.bias.grad) * 1.5 + 1e-3
    assert err(x1.grad, xr.grad) <= err(x2.grad, xr.grad) * 1.5 + 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(256, 2048, 7, 7), (3, 1024, 7, 7), (2, 520, 5, 3), (4, 8, 1, 1)])
def test_global_avg_pool_matches_torch(cuda, dtype, shape):
    """Native global average pool (fwd [N, C] + channels_last backward) vs fp32 adaptive_avg_pool2d."""
    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.pool import global_avg_pool

    torch.manual_seed(0)
    x = torch.randn(shape, device=cuda).to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    xr = x.detach().float().clone().requires_grad_(True)
    dnn.set_backend("native")
    try:
        y = global_avg_pool(x)
        assert y.grad_fn is not None and "GlobalAvgPool" in type(y.grad_fn).__name__  # the native op ran
    finally:
        dnn.set_backend("torch")
    yr = torch.flatten(F.adaptive_avg_pool2d(xr, 1), 1)
    tol = dict(rtol=1e-2, atol=1e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(y.float(), yr, **tol)
    g = torch.randn(y.shape, device=cuda).to(dtype)
    y.backward(g)
    yr.backward(g.float())
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    assert _ext.require() is not None


@pytest.mark.parametrize("shape", [(2, 256, 56, 56), (3, 8, 6, 10), (1, 1024, 14, 14), (1100, 256, 56, 56)])
def test_subsample2_matches_strided_copy(cuda, shape):
    """Native stride-2 subsample (downsample-conv input) == x[:, :, ::2, ::2], bitwise; the last shape
    has > 2^24 16-byte chunks."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    x = torch.randn(shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = C.subsample2(x)
    ref = x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.shape == ref.shape
    assert torch.equal(y, ref)
