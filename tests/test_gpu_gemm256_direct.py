"""256x256 statistics forwards stored from the registers (dla_mfma.h epilogue_direct, DLA_GEMM256_DIRECT) vs the
LDS-staged epilogue and fp32 PyTorch (gpu). The transposed product has the same bf16 products in the same k order,
so the outputs must be bit-identical; the statistics partials are summed in another order."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(20000, 256, 1024), (9001, 512, 2048), (5001, 256, 512), (62720, 512, 2048), (300, 1024, 256)]


@pytest.mark.parametrize("shape", SHAPES)
def test_direct_256_forward_matches_staged_and_torch(cuda, shape):
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    M, K, N = shape
    g = torch.Generator(device=cuda).manual_seed(0)
    a = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=cuda) * K ** -0.5).to(torch.bfloat16)
    try:
        C.set_gemm256_direct(0)
        y0, s0 = C.gemm_nt(a, w, True, None, False, 8)  # forced 256x256 tile
        C.set_gemm256_direct(1)
        y1, s1 = C.gemm_nt(a, w, True, None, False, 8)
    finally:
        C.set_gemm256_direct(-1)
    torch.cuda.synchronize()
    assert torch.equal(y1, y0)
    assert s1.shape == s0.shape == ((M + 255) // 256, N, 2)
    torch.testing.assert_close(s1, s0, rtol=1e-4, atol=1e-3)
    yf = y1.float()
    torch.testing.assert_close(s1.sum(0)[:, 0], yf.sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)
    torch.testing.assert_close(s1.sum(0)[:, 1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2 * M ** 0.5)
    rows = slice(max(0, M - 300), M)  # the partial last row tile against fp32
    ref = a[rows].float() @ w.float().t()
    assert ((yf[rows] - ref).norm() / ref.norm()).item() < 5e-3
