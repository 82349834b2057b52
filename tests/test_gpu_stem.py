"""Native ResNet stem conv (7x7/s2/p3, 3 input channels; csrc/kernels/stem.hip) vs fp32 PyTorch (gpu)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _inputs(cuda, n, h, w, cout=64, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, 3, h, w, generator=g).to(cuda, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, 3, 7, 7, generator=g) * 0.1).to(cuda, torch.bfloat16)
    return x, wt


@pytest.mark.parametrize("shape", [(2, 224, 224), (3, 37, 29), (1, 8, 8), (4, 64, 96),
                                   (340, 224, 224)])  # > 2^24 input pixels (only output pixels are fastdiv'd)
def test_stem_fwd_and_stats_match_torch(cuda, shape):
    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops.conv import stem_pack_weight

    C = _ext.require()
    x, wt = _inputs(cuda, *shape)
    y, stats, _ = C.stem_fwd(x, stem_pack_weight(wt), True)
    ref = F.conv2d(x.float(), wt.float(), None, 2, 3)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    # statistics of the stored bf16 values, per channel
    yf = y.float()
    s = stats.sum(0)
    torch.testing.assert_close(s[:, 0], yf.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(s[:, 1], (yf * yf).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("shape", [(2, 224, 224), (3, 37, 29)])
def test_stem_wgrad_matches_torch(cuda, shape):
    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops.conv import stem_pack_weight, stem_unpack_grad

    C = _ext.require()
    x, wt = _inputs(cuda, *shape, seed=1)
    n, _, h, w = x.shape
    dy = torch.randn(n, 64, (h - 1) // 2 + 1, (w - 1) // 2 + 1, device=cuda).to(torch.bfloat16)
    dy = dy.contiguous(memory_format=torch.channels_last)
    xs = C.stem_fwd(x, stem_pack_weight(wt), False)[2]
    dwp = C.stem_wgrad(dy, xs, h, w, torch.float32)
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), wt.float(), None, [2, 2], [3, 3], [1, 1], False,
                                              [0, 0], 1, [False, True, False])[1]
    got = stem_unpack_grad(dwp)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    # the 4 padding channels of the fold carry no gradient
    assert dwp.reshape(64, 16, 16)[:, :, 12:].abs().max().item() == 0.0


def test_stem_bn_relu_pool_end_to_end(cuda):
    """conv_bn_act_maxpool on the native stem (conv + statistics epilogue + fused BN/ReLU/pool) vs the
    torch path, forward and weight/BN-parameter gradients."""
    from distributed_learning_amd.ops import nn as dnn

    torch.manual_seed(0)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(cuda).to(memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(64).to(cuda)
    pool = nn.MaxPool2d(3, 2, 1)
    x = torch.randn(4, 3, 64, 64, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def run(backend):
        c2 = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(cuda).to(memory_format=torch.channels_last)
        c2.load_state_dict(conv.state_dict())
        c2.weight.data = c2.weight.data.to(torch.bfloat16)
        b2 = nn.BatchNorm2d(64).to(cuda)
        b2.load_state_dict(bn.state_dict())
        dnn.set_backend(backend)
        try:
            y = dnn.conv_bn_act_maxpool(x, c2, b2, pool)
            y.float().mul(torch.linspace(0, 1, y.numel(), device=cuda).reshape(y.shape)).sum().backward()
        finally:
            dnn.set_backend("torch")
        return y.float(), c2.weight.grad.float(), b2.weight.grad, b2.running_mean.clone()

    yn, gwn, gbn, rmn = run("native")
    yt, gwt, gbt, rmt = run("torch")
    torch.testing.assert_close(yn, yt, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(rmn, rmt, rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(gbn, gbt, rtol=3e-2, atol=3e-2 * gbt.abs().max().item())
    # the two convs round differently, so a few near-tie max-pool windows route their gradient to a
    # different pixel: allow a handful of outliers (4 of 9408 seen), the bulk must agree
    bad = ((gwn - gwt).abs() > 5e-2 * gwt.abs().max().item() + 5e-2 * gwt.abs()).float().mean().item()
    assert bad < 2e-3, bad
    assert (gwn - gwt).norm().item() / gwt.norm().item() < 5e-2


