"""Halo-tiled 64-channel 3x3 weight gradient (csrc/kernels/conv_halo_wgrad.hip) vs fp32 PyTorch and vs
the implicit-GEMM weight gradient: odd image sizes (the padded position space and its zero halo),
batches whose strips straddle images, a block count that leaves blocks with no strips, bf16 and fp32
outputs."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(2, 56, 56), (3, 17, 23), (1, 7, 9), (5, 56, 56), (16, 28, 28)]


@pytest.fixture
def C():
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    yield C
    C.set_halo_wgrad(-1)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
def test_halo_wgrad(cuda, C, shape, odt):
    n, h, w = shape
    g = torch.Generator().manual_seed(n * 1000 + h * 10 + w)
    x = torch.randn(n, 64, h, w, generator=g).to(cuda, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, 64, h, w, generator=g).to(cuda, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    C.set_halo_wgrad(1)
    assert C.halo_wgrad_eligible(64, 64, w, 1)
    dw = C.conv3x3_wgrad(dy, x, 1, odt)
    C.set_halo_wgrad(0)
    dw_ref_kernel = C.conv3x3_wgrad(dy, x, 1, torch.float32)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.float(), (64, 64, 3, 3), dy.float(), padding=1)
    assert dw.shape == ref.shape and dw.dtype == odt
    assert _rel(dw, ref) < (5e-3 if odt == torch.bfloat16 else 1e-4), _rel(dw, ref)
    # the same bf16 products summed in another order: fp32-rounding-level agreement
    assert _rel(dw_ref_kernel, ref) < 1e-4
    if odt == torch.float32:
        assert _rel(dw, dw_ref_kernel) < 1e-4


def test_not_eligible(C):
    C.set_halo_wgrad(1)
    assert not C.halo_wgrad_eligible(128, 128, 28, 1)
    assert not C.halo_wgrad_eligible(64, 64, 56, 2)
    assert not C.halo_wgrad_eligible(64, 64, 100, 1)  # halo + 3 strips exceed the 512-row ring
