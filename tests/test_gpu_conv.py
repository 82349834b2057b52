"""Native 1x1 conv (MFMA GEMM) and the fused conv+BN(+stats) path vs PyTorch fp32 references (gpu)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,cout,stride", [((4, 64, 56, 56), 256, 1), ((2, 256, 28, 28), 64, 1),
                                               ((4, 512, 28, 28), 1024, 2), ((3, 24, 9, 9), 40, 1)])
@pytest.mark.parametrize("wdtype", [torch.float32, torch.bfloat16])
def test_conv1x1_fwd_bwd(cuda, shape, cout, stride, wdtype):
    from distributed_learning_amd.ops.conv import conv1x1

    torch.manual_seed(0)
    conv = nn.Conv2d(shape[1], cout, 1, stride=stride, bias=False).to(cuda).to(wdtype)
    conv = conv.to(memory_format=torch.channels_last)
    x = torch.randn(shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_(True)
    y, stats = conv1x1(x1, conv, want_stats=True)
    xr = x.float().clone().requires_grad_(True)
    wr = conv.weight.detach().float().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, stride)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2 * shape[1] ** 0.5 / 8)
    ysum = y.float().sum((0, 2, 3))
    torch.testing.assert_close(stats.sum(0)[:, 0], ysum, rtol=1e-3, atol=1e-1)
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    yr.backward(g.to(torch.bfloat16).float())
    rel_dx = (x1.grad.float() - xr.grad).norm() / xr.grad.norm()
    rel_dw = (conv.weight.grad.float() - wr.grad).norm() / wr.grad.norm()
    assert rel_dx < 1e-2 and rel_dw < 1e-2, (float(rel_dx), float(rel_dw))
    assert conv.weight.grad.dtype == wdtype


def test_conv_bn_act_native_vs_torch(cuda):
    from distributed_learning_amd.ops import nn as dnn

    torch.manual_seed(0)
    conv = nn.Conv2d(256, 64, 1, bias=False).to(cuda).to(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(64).to(cuda)
    conv2, bn2 = nn.Conv2d(256, 64, 1, bias=False).to(cuda), nn.BatchNorm2d(64).to(cuda)
    conv2.load_state_dict(conv.state_dict())
    bn2.load_state_dict(bn.state_dict())
    x = torch.randn(8, 256, 28, 28, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn(8, 64, 28, 28, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        y = dnn.conv_bn_act(x, conv, bn, relu=True, residual=res)
    finally:
        dnn.set_native_conv(False)
        dnn.set_backend("torch")
    yr = torch.relu(bn2(F.conv2d(x.float(), conv2.weight.float())) + res.float())
    torch.testing.assert_close(y.float(), yr, rtol=3e-2, atol=5e-2)
    torch.testing.assert_close(bn.running_mean, bn2.running_mean, rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(bn.running_var, bn2.running_var, rtol=1e-2, atol=1e-3)


def test_conv1x1_fork_sums_identity_gradient(cuda):
    """_Conv1x1Fork: dx = dgrad + d_identity fused in the GEMM epilogue equals the autograd sum of
    the two uses of x (bitwise: both round the GEMM result to bf16 before the bf16 add)."""
    from distributed_learning_amd.ops.conv import conv1x1, conv1x1_fork

    torch.manual_seed(0)
    conv = nn.Conv2d(256, 64, 1, bias=False).to(cuda).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(4, 256, 28, 28, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(4, 64, 28, 28, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gi = torch.randn(4, 256, 28, 28, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    x1 = x.clone().requires_grad_(True)
    y1, _, ident, _ = conv1x1_fork(x1, conv)
    assert ident.data_ptr() == x1.data_ptr()
    torch.autograd.backward([y1, ident], [g, gi])
    dw1 = conv.weight.grad.clone()
    conv.weight.grad = None

    x2 = x.clone().requires_grad_(True)
    y2, _ = conv1x1(x2, conv)
    torch.autograd.backward([y2, x2 * 1], [g, gi])
    assert torch.equal(y1, y2)
    assert torch.equal(x1.grad, x2.grad)
    assert torch.equal(dw1, conv.weight.grad)

    # identity gradient only (conv output unused) and conv gradient only
    x3 = x.clone().requires_grad_(True)
    _, _, ident, _ = conv1x1_fork(x3, conv)
    ident.backward(gi)
    assert torch.equal(x3.grad, gi)
