"""Register-stored 128x128 1x1 GEMM tiles (csrc/kernels/gemm_direct.hip) vs fp32 PyTorch and vs the LDS-staged
tile kernel (gemm.hip) they replace.

The direct kernel computes the transposed product (same bf16 products, same k order per output element), so
its outputs must equal the staged kernel's bit for bit; its BatchNorm-statistics partials are summed in another
order, so they are checked against the column sums of the stored output. Shapes cover ragged M (last row tile
partly out of range), a column tile partly past N, the register-staged main loop (K <= 512), the 2-stage
LDS-DMA loop (K > 512) and the buffer-DMA loop (forced PIPE 6), weights [N][K] (forward) and k-major [K][N]
(data gradient), with and without the masked identity-gradient addend. The streaming kernel is turned off so
the short-K shapes reach the tile dispatch, and the statistics forwards are held on the 128x128 tiles (their
default moves to 256x256 from K = 256).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, K, N)
    (3000, 64, 256), (20000, 256, 1024), (5001, 512, 128), (9000, 1024, 384), (12345, 128, 320),
    (250880, 256, 1024),  # stage-3 conv3 at bs1280
]


@pytest.fixture
def C():
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    C.set_gemm_stream(0)
    C.set_tile256_min_k_stats(1 << 30)  # keep the statistics forwards on the 128x128 tiles under test
    yield C
    C.set_tile256_min_k_stats(-1)
    C.set_gemm_stream(-1)
    C.set_gemm_direct(-1)
    C.set_mfma_pipeline(-1)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _both(C, fn):
    C.set_gemm_direct(1)
    new = fn()
    C.set_gemm_direct(0)
    old = fn()
    C.set_gemm_direct(1)
    torch.cuda.synchronize()
    return new, old


@pytest.mark.parametrize("pipe", [-1, 6])
@pytest.mark.parametrize("kmajor", [False, True])
@pytest.mark.parametrize("shape", SHAPES)
def test_direct_forward_statistics(cuda, C, shape, kmajor, pipe):
    M, K, N = shape
    g = torch.Generator().manual_seed(M + K + N)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(cuda, torch.bfloat16)
    B = W.t().contiguous() if kmajor else W
    C.set_mfma_pipeline(pipe)
    poison = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    del poison  # a skipped store would leave NaN behind
    (out, st), (ref_tile, st_tile) = _both(C, lambda: C.gemm_nt(A, B, True, None, kmajor))
    assert torch.isfinite(out).all()
    assert torch.equal(out, ref_tile)
    ref = A.float() @ W.float().t()
    assert _rel(out, ref) < 5e-3
    assert st.shape == st_tile.shape == ((M + 127) // 128, N, 2)
    tot = st.double().sum(0)
    of = out.double()
    torch.testing.assert_close(tot[:, 0], of.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(tot[:, 1], (of * of).sum(0), rtol=1e-4, atol=1e-3)
    # per row tile, too (bn_stats_finalize reduces the rows in a fixed order; a tile's partial is its own)
    torch.testing.assert_close(st.double(), st_tile.double(), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("pipe", [-1, 6])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("shape", SHAPES)
def test_direct_dgrad_addend(cuda, C, shape, masked, pipe):
    """C = bf16(bf16(dY W) + (bit ? D : 0)), bit for bit the staged kernel's."""
    M, K, N = shape
    g = torch.Generator().manual_seed(M + 3 * K + N)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    B = (torch.randn(K, N, generator=g) * K ** -0.5).to(cuda, torch.bfloat16)
    D = torch.randn(M, N, generator=g).to(cuda, torch.bfloat16)
    mask = torch.randint(0, 256, ((M * N + 7) // 8,), generator=g, dtype=torch.uint8).to(cuda) if masked else None
    C.set_mfma_pipeline(pipe)
    (out, _), (ref, _) = _both(C, lambda: C.gemm_nt(A, B, False, D, True, 0, mask))
    assert torch.equal(out, ref)
    bits = torch.ones(M * N, device=cuda) if mask is None else \
        torch.stack([(mask >> j) & 1 for j in range(8)], 1).reshape(-1)[: M * N].float()
    exp = ((A.float() @ B.float()).to(torch.bfloat16).float() + D.float() * bits.view(M, N)).to(torch.bfloat16)
    assert float((out.float() - exp.float()).abs().max()) <= float(exp.float().abs().max()) * 2 ** -6


@pytest.mark.parametrize("kmajor", [False, True])
@pytest.mark.parametrize("shape", SHAPES[:4])
def test_direct_plain_writes_every_row(cuda, C, shape, kmajor):
    M, K, N = shape
    g = torch.Generator().manual_seed(M * 3 + K + N)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(cuda, torch.bfloat16)
    B = W.t().contiguous() if kmajor else W
    poison = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    del poison
    (out, _), (ref, _) = _both(C, lambda: C.gemm_nt(A, B, False, None, kmajor))
    assert torch.isfinite(out).all(), f"{int((~torch.isfinite(out)).any(1).sum())} rows never written"
    assert torch.equal(out, ref)
    assert _rel(out, A.float() @ W.float().t()) < 5e-3


def test_direct_row_strided_output(cuda, C):
    """The output written into a channel slice of a wider tensor (ldc > N) is refused by gemm_nt's API
    (it allocates C), so the direct path is reached through conv1x1 with an input slice instead:
    A row-strided, C contiguous."""
    M, K, N = 7000, 256, 512
    g = torch.Generator().manual_seed(11)
    wide = torch.randn(M, 2 * K, generator=g).to(cuda, torch.bfloat16)
    A = wide[:, K:]
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(cuda, torch.bfloat16)
    (out, st), (ref, _) = _both(C, lambda: C.gemm_nt(A, W, True, None, False))
    assert torch.equal(out, ref)
    assert _rel(out, A.float() @ W.float().t()) < 5e-3
