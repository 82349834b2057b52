"""fp32 convolutions on the fp32 matrix cores (csrc/kernels/conv_f32.hip, ops/conv_f32.py) vs float64 PyTorch.

Forward, input gradient and weight gradient of 1x1 / 3x3 / 7x7 convolutions in channels_last fp32: channel counts
that are multiples of 4 but not of 8 or 16 (24, 20), ragged pixel counts (tiles partly past M), odd batch, both
tile sizes (the 128x128 tile above ~512 tiles, 64x64 below), split and unsplit weight-gradient reductions, the
stem's 3 input channels padded to 4 with stride 2. The kernels accumulate exact fp32 products in fp32, so the
bound is fp32 summation error: relative L2 1e-5 against float64.
"""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu

CASES = [  # N, Cin, H, W, Cout, k, pad, stride
    (4, 64, 28, 28, 192, 3, 1, 1),
    (4, 192, 28, 28, 64, 1, 0, 1),
    (2, 24, 14, 14, 64, 3, 1, 1),
    (3, 20, 9, 11, 36, 3, 1, 1),
    (8, 16, 7, 7, 48, 3, 1, 1),
    (3, 528, 14, 14, 160, 1, 0, 1),
    (32, 256, 28, 28, 128, 1, 0, 1),   # 128x128 tiles
    (16, 96, 28, 28, 128, 3, 1, 1),    # 128x128 tiles, 3x3
    (4, 3, 64, 64, 64, 7, 3, 2),       # the generic stem form (input padded 3 -> 4, stride 2, no input gradient)
    (8, 64, 28, 28, 192, 3, 1, 1),     # 192 columns: 64-wide tiles, no padded work
    (8, 192, 14, 14, 16, 1, 0, 1),     # 16 output channels: 32-wide tiles
    (8, 32, 14, 14, 96, 3, 1, 1),      # 96 columns: 32-wide tiles
]


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("case", CASES)
def test_conv_f32_matches_float64(cuda, case):
    from distributed_learning_amd.ops import conv_f32

    n, cin, h, w, cout, k, pad, stride = case
    g = torch.Generator().manual_seed(sum(case))
    conv = nn.Conv2d(cin, cout, k, stride=stride, padding=pad, bias=False)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * (cin * k * k) ** -0.5)
    conv = conv.to(cuda).to(memory_format=torch.channels_last)
    x = torch.randn(n, cin, h, w, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    need_dx = stride == 1
    x.requires_grad_(need_dx)
    old = conv_f32.STEM_NATIVE
    conv_f32.STEM_NATIVE = True
    try:
        assert conv_f32.supported(x, conv)
    finally:
        conv_f32.STEM_NATIVE = old
    y = conv_f32._ConvF32.apply(x, conv.weight, pad, stride)  # the generic form, also for the stem case
    dy = torch.randn(y.shape, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    torch.cuda.synchronize()
    xd = x.detach().double().requires_grad_(need_dx)
    wd = conv.weight.detach().double().requires_grad_(True)
    yd = torch.nn.functional.conv2d(xd, wd, None, stride, pad)
    yd.backward(dy.double())
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, yd) < 1e-5
    assert _rel(conv.weight.grad, wd.grad) < 1e-5
    assert conv.weight.grad.stride() == conv.weight.stride()
    if need_dx:
        assert _rel(x.grad, xd.grad) < 1e-5


def test_conv_f32_accumulate_into_output(cuda):
    """out += conv(x): the accumulate form the Inception gradient sums use."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 32, 10, 10, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    w = torch.randn(48, 3, 3, 32, generator=g).to(cuda)
    base = torch.randn(2, 48, 10, 10, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    out = base.clone()
    C.conv_f32_fwd(x, w, 1, 1, out)
    ref = base.double() + torch.nn.functional.conv2d(x.double(), w.permute(0, 3, 1, 2).double(), None, 1, 1)
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-5


@pytest.mark.parametrize("shape", [(4, 64, 64), (2, 224, 224), (3, 30, 42)])
def test_stem_space_to_depth_matches_float64(cuda, shape):
    """The 7x7 / stride-2 stem as a 4x4 conv over 2x2 pixel blocks (ops/conv_f32.py _StemS2D): output and weight
    gradient against float64."""
    from distributed_learning_amd.ops import conv_f32

    n, h, w = shape
    g = torch.Generator().manual_seed(h + w)
    conv = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
    conv = conv.to(cuda).to(memory_format=torch.channels_last)
    x = torch.rand(n, 3, h, w, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    assert conv_f32.stem_s2d_ok(x, conv) and conv_f32.supported(x, conv)
    y = conv_f32.conv(x, conv)
    dy = torch.randn(y.shape, generator=g).to(cuda).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    wd = conv.weight.detach().double().requires_grad_(True)
    yd = torch.nn.functional.conv2d(x.double(), wd, None, 2, 3)
    yd.backward(dy.double())
    torch.cuda.synchronize()
    assert y.shape == yd.shape
    assert _rel(y, yd) < 1e-5
    assert _rel(conv.weight.grad, wd.grad) < 1e-5
    assert conv.weight.grad.stride() == conv.weight.stride()
