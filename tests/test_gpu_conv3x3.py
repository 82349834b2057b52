"""Implicit-GEMM 3x3 convolution kernels (csrc/kernels/conv.hip) vs fp32 PyTorch convs (gpu)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


def _C():
    from distributed_learning_amd.ops import _ext

    return _ext.require()


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("N,Cin,H,W,Cout,stride", [
    (2, 64, 56, 56, 64, 1), (2, 128, 28, 28, 128, 1), (1, 256, 14, 14, 256, 1), (4, 512, 7, 7, 512, 1),
    (2, 128, 56, 56, 128, 2), (2, 64, 9, 13, 128, 1), (3, 128, 11, 7, 64, 2), (2, 256, 28, 28, 256, 2),
    # GoogLeNet's Inception 3x3s (any C % 8: a 64-deep k-step spans taps -> per-lane tap decode)
    (2, 16, 28, 28, 32, 1), (2, 96, 28, 28, 128, 1), (2, 96, 14, 14, 208, 1), (2, 24, 14, 14, 64, 1),
    (2, 112, 14, 14, 224, 1), (2, 144, 14, 14, 288, 1), (2, 160, 7, 7, 320, 1), (2, 48, 7, 7, 128, 1),
    (1, 8, 5, 7, 24, 1), (2, 64, 56, 56, 192, 1),
    # 256x256 8-wave tiles: auto-picked fwd / dgrad (>= 192 tiles, K >= 1024) and the wide wgrad
    (256, 256, 14, 14, 256, 1), (2, 512, 14, 14, 512, 2),
])
def test_conv3x3_fwd_dgrad_wgrad(cuda, N, Cin, H, W, Cout, stride):
    C = _C()
    torch.manual_seed(0)
    x = torch.randn(N, Cin, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, 3, 3, device=cuda) * (2.0 / (9 * Cin)) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, stride, 1)
    y, stats = C.conv3x3_fwd(x, w, stride, True)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
    assert _rel(y, yr) < 1e-2
    yf = y.float()
    torch.testing.assert_close(stats.sum(0)[:, 0], yf.sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(stats.sum(0)[:, 1], (yf * yf).sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    dy = torch.randn(yr.shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    yr.backward(dy.float())
    dw = C.conv3x3_wgrad(dy, x, stride, torch.float32)
    assert dw.shape == w.shape and dw.is_contiguous(memory_format=CL)
    assert _rel(dw, wr.grad) < 1e-2, _rel(dw, wr.grad)
    if stride == 1:
        dx = C.conv3x3_dgrad(dy, w)
        assert dx.shape == x.shape
        assert _rel(dx, xr.grad) < 1e-2, _rel(dx, xr.grad)
        add = torch.randn_like(x)
        assert torch.equal(C.conv3x3_dgrad(dy, w, add), dx + add)
    elif H % 2 == 0 and W % 2 == 0:
        dx = C.conv3x3s2_dgrad(dy, w, H, W)
        assert dx.shape == x.shape and dx.is_contiguous(memory_format=CL)
        assert _rel(dx, xr.grad) < 1e-2, _rel(dx, xr.grad)


@pytest.mark.parametrize("N,Cin,H,W,Cout", [(2, 64, 8, 6, 64), (1, 128, 14, 14, 64), (3, 64, 4, 10, 128),
                                           (64, 256, 28, 28, 256),  # 256x256 8-wave tiles
                                           (333, 128, 56, 56, 128)])  # 512x128: 4 x 511 tiles, partial last
def test_conv3x3s2_dgrad_every_tap(cuda, N, Cin, H, W, Cout):
    """Stride-2 data gradient (parity classes): one-hot weights per tap, exact against fp32."""
    C = _C()
    x = torch.randn(N, Cin, H, W, device=cuda)
    for tap in range(9):
        w = torch.zeros(Cout, Cin, 3, 3, device=cuda)
        w[torch.arange(Cout), (torch.arange(Cout) * 5) % Cin, tap // 3, tap % 3] = 1.0
        xr = x.clone().requires_grad_(True)
        yr = F.conv2d(xr, w, None, 2, 1)
        dy = torch.randn(yr.shape, device=cuda).to(torch.bfloat16)
        yr.backward(dy.float())
        dx = C.conv3x3s2_dgrad(dy.contiguous(memory_format=CL), w.to(torch.bfloat16).contiguous(memory_format=CL),
                               H, W)
        torch.testing.assert_close(dx.float(), xr.grad, rtol=4e-3, atol=1e-6)  # bf16 rounding of 2-term sums


@pytest.mark.parametrize("Cin,Cout", [(64, 64), (24, 40), (16, 72)])
def test_conv3x3_asymmetric_weights(cuda, Cin, Cout):
    """One-hot weights per tap catch a flipped / transposed tap order in any of the passes."""
    C = _C()
    N, H, W = 1, 6, 5
    x = torch.randn(N, Cin, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    for tap in range(9):
        w = torch.zeros(Cout, Cin, 3, 3, device=cuda)
        w[torch.arange(Cout), (torch.arange(Cout) * 7) % Cin, tap // 3, tap % 3] = 1.0
        w = w.to(torch.bfloat16).contiguous(memory_format=CL)
        y, _ = C.conv3x3_fwd(x, w, 1, False)
        torch.testing.assert_close(y.float(), F.conv2d(x.float(), w.float(), None, 1, 1), rtol=0, atol=0)
        dy = torch.randn(y.shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
        dx = C.conv3x3_dgrad(dy, w)
        ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), 1, 1)
        torch.testing.assert_close(dx.float(), ref, rtol=1e-2, atol=1e-2)
        dw = C.conv3x3_wgrad(dy, x, 1, torch.float32)
        refw = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), 1, 1)
        torch.testing.assert_close(dw.float(), refw, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("tile", [1, 2, 3, 8, 9])
@pytest.mark.parametrize("ch", [128, 256])
def test_conv3x3_tile_configs(cuda, tile, ch):
    C = _C()
    torch.manual_seed(0)
    x = torch.randn(3, ch, 14, 14, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(ch, ch, 3, 3, device=cuda) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    y_ref, s_ref = C.conv3x3_fwd(x, w, 1, True, 1)
    y, s = C.conv3x3_fwd(x, w, 1, True, tile)
    assert torch.equal(y, y_ref)
    torch.testing.assert_close(s.sum(0), s_ref.sum(0), rtol=1e-5, atol=1e-3)
    dy = torch.randn_like(y)
    assert torch.equal(C.conv3x3_dgrad(dy, w, None, tile), C.conv3x3_dgrad(dy, w, None, 1))


@pytest.mark.parametrize("stride", [1, 2])
def test_conv3x3_512x128_tile_at_stage2_rows(cuda, stride):
    """The 512x128 tile (Cout = 128, >= 1024 row tiles: ResNet stage 2 at the bench batch) against fp32 torch,
    with the BN-statistics epilogue, a partial last row tile (548,800 rows = 1071 x 512 + 448) and the data
    gradient with a fused addend."""
    C = _C()
    torch.manual_seed(0)
    N, H = 700, 28 * stride
    assert C.pick_conv_tile(N * 28 * 28, 128, 9 * 128, True) == 9  # the auto pick at these rows
    x = torch.randn(N, 128, H, H, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(128, 128, 3, 3, device=cuda) * (2.0 / (9 * 128)) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    yr = F.conv2d(x.float(), w.float(), None, stride, 1)
    y, stats = C.conv3x3_fwd(x, w, stride, True, 9)
    assert stats.shape[0] == (N * 28 * 28 + 511) // 512
    assert _rel(y, yr) < 1e-2
    y1, s1 = C.conv3x3_fwd(x, w, stride, True, 1)
    assert torch.equal(y, y1)
    torch.testing.assert_close(stats.sum(0), s1.sum(0), rtol=1e-4, atol=1.0)
    yf = y.float()
    torch.testing.assert_close(stats.sum(0)[:, 0], yf.sum((0, 2, 3)), rtol=1e-3, atol=1.0)
    if stride == 1:
        dy = torch.randn(y.shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
        add = torch.randn_like(x)
        dx = C.conv3x3_dgrad(dy, w, add, 9)
        ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), 1, 1) + add.float()
        assert _rel(dx, ref) < 1e-2
        assert torch.equal(dx, C.conv3x3_dgrad(dy, w, add, 1))


@pytest.mark.parametrize("pipe", [0, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("cin", [64, 24])
def test_conv3x3_pipelines_agree(cuda, pipe, cin):
    C = _C()
    torch.manual_seed(0)
    x = torch.randn(2, cin, 9, 13, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(128, cin, 3, 3, device=cuda) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(2, 128, 9, 13, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    old = C.mfma_pipeline()
    try:
        C.set_mfma_pipeline(0)
        ref = [C.conv3x3_fwd(x, w, 1, True)[0], C.conv3x3_dgrad(dy, w), C.conv3x3_wgrad(dy, x, 1, torch.float32),
               C.conv3x3_fwd(x, w, 2, False)[0]]
        C.set_mfma_pipeline(pipe)
        got = [C.conv3x3_fwd(x, w, 1, True)[0], C.conv3x3_dgrad(dy, w), C.conv3x3_wgrad(dy, x, 1, torch.float32),
               C.conv3x3_fwd(x, w, 2, False)[0]]
    finally:
        C.set_mfma_pipeline(old)
    for r, g in zip(ref, got):
        assert torch.equal(r, g)


_HALO_SCRIPT = r"""
import sys, torch, torch.nn.functional as F
sys.path.insert(0, %r)
from distributed_learning_amd.ops import _ext
C = _ext.require()
CL = torch.channels_last
dev = torch.device("cuda:0")
for N, H, W in [(2, 56, 56), (3, 9, 13), (2, 7, 63), (1, 1, 1), (5, 56, 56)]:
    torch.manual_seed(0)
    x = torch.randn(N, 64, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(64, 64, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    y, s = C.conv3x3_fwd(x, w, 1, True, 0)           # halo kernel (DLA_HALO=2)
    y1, s1 = C.conv3x3_fwd(x, w, 1, True, 1)         # forced 128x128 implicit GEMM
    assert torch.equal(y, y1), (N, H, W)              # same tap / k order -> bitwise
    torch.testing.assert_close(s.sum(0), s1.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(y.float(), F.conv2d(x.float(), w.float(), None, 1, 1), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(s.sum(0)[:, 0], y.float().sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    dy = torch.randn_like(y)
    dx = C.conv3x3_dgrad(dy, w)                       # halo kernel, flipped / transposed weights
    refx = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), 1, 1)
    torch.testing.assert_close(dx.float(), refx, rtol=1e-2, atol=2e-2)
    add = torch.randn_like(x)
    assert torch.equal(C.conv3x3_dgrad(dy, w, add), dx + add)  # fused addend == unfused bf16 add
print("halo ok")
"""


# 3: variant 2 forward, variant 1 data gradient; "d": the variant-1 data gradient stored from registers, "f": the
# forward (tile and statistics) from registers (variant 2, or variant 1 through dla_mfma.h epilogue_direct)
@pytest.mark.parametrize("version", ["1", "2", "3", "1d", "3d", "2f", "3df", "1f", "1df"])
def test_conv3x3_halo_c64(cuda, version):
    """64 -> 64 channel stride-1 3x3 convs on the halo-tiled persistent kernel, forward and data
    gradient, both kernel variants (a fresh process with DLA_HALO=2, read once): forward bitwise equal to the
    implicit-GEMM kernel, statistics and the data gradient against fp32 PyTorch."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DLA_HALO="2", DLA_HALO_V=version[0], DLA_HALO_DIRECT="1" if "d" in version else "0",
               DLA_HALO_DIRECT_FWD="1" if "f" in version else "0")
    r = subprocess.run([sys.executable, "-c", _HALO_SCRIPT % root], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "halo ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.parametrize("N,H,stride", [(2, 28, 1), (3, 13, 1), (2, 56, 2), (64, 28, 1)])
def test_conv3x3_wgrad_128x256_tiles(cuda, N, H, stride):
    """128x256 four-wave weight-gradient tiles for Cout = 128 (set_wgrad_w4): the last column tile covers taps
    past the 9th (masked), against fp32 PyTorch and the 128x128 tiles."""
    C = _C()
    torch.manual_seed(0)
    x = torch.randn(N, 128, H, H, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    oh = (H - 1) // stride + 1
    dy = torch.randn(N, 128, oh, oh, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    try:
        C.set_wgrad_w4(0)
        ref_tile = C.conv3x3_wgrad(dy, x, stride, torch.float32)
        C.set_wgrad_w4(1)
        got = C.conv3x3_wgrad(dy, x, stride, torch.float32)
    finally:
        C.set_wgrad_w4(-1)
    ref = torch.nn.grad.conv2d_weight(x.float(), (128, 128, 3, 3), dy.float(), stride, 1)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=CL)
    assert _rel(got, ref) < 1e-2
    assert _rel(got, ref_tile) < 1e-5  # same products, another split of the pixel sum
