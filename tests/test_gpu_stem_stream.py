"""The ResNet stem forward on the persistent streaming GEMM (csrc/kernels/gemm_stream.hip kStem: implicit im2col
over the space-to-depth image, BN statistics in registers) vs the 128x64 implicit-GEMM tile kernel (stem.hip) and
fp32 PyTorch (gpu)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("n,h,w", [(4, 224, 224), (3, 100, 98), (2, 64, 96), (1280, 224, 224)])
def test_stem_stream_matches_tile_and_torch(cuda, n, h, w):
    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops.conv import stem_pack_weight

    C = _ext.require()
    g = torch.Generator(device=cuda).manual_seed(0)
    x = torch.randn(n, 3, h, w, generator=g, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    wt = (torch.randn(64, 3, 7, 7, generator=g, device=cuda) * 0.1).to(torch.bfloat16)
    wpk = stem_pack_weight(wt)
    try:
        C.set_stem_stream(0)
        y0, s0, _ = C.stem_fwd(x, wpk, True)
        C.set_stem_stream(1)
        y1, s1, _ = C.stem_fwd(x, wpk, True)
    finally:
        C.set_stem_stream(-1)
    torch.cuda.synchronize()
    assert y1.shape == y0.shape and y1.is_contiguous(memory_format=CL)
    assert s1.shape[1:] == (64, 2) and s1.shape[0] <= s0.shape[0]
    assert _rel(y1, y0) < 1e-3  # same bf16 products, another accumulation order inside the MFMA
    k = min(n, 2)  # fp32 reference on the last images (the tail row tile included)
    ref = F.conv2d(x[-k:].float(), wt.float(), None, 2, 3)
    assert _rel(y1[-k:], ref) < 1e-2
    yf = y1.float()
    torch.testing.assert_close(s1.sum(0)[:, 0], yf.sum((0, 2, 3)), rtol=1e-3, atol=1e-2 * yf.numel() ** 0.5)
    torch.testing.assert_close(s1.sum(0)[:, 1], (yf * yf).sum((0, 2, 3)), rtol=1e-3, atol=1e-2 * yf.numel() ** 0.5)
