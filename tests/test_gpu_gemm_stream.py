"""Persistent streaming 1x1 GEMM (csrc/kernels/gemm_stream.hip) vs fp32 PyTorch, and vs the tile kernel.

Shapes cover every instantiation (K = 64 / 128 / 256 -> 1 / 2 / 4 ring chunks per tile, 128- and 64-wide
column panels, weights [N][K] and k-major [K][N]), ragged M (last tile partly out of range: zero-filled
loads, dropped stores), several column panels per row group, row-strided A (a channel slice) and the
BatchNorm-statistics epilogue, whose partial rows must sum to the column sums of the stored bf16 output.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, K, N)
    (9000, 64, 64), (9000, 64, 256), (20000, 128, 512), (5001, 256, 128), (70000, 256, 64), (33333, 128, 128),
    (131072, 64, 256),
]


@pytest.fixture
def C():
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    yield C
    C.set_gemm_stream(-1)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("kmajor", [False, True])
@pytest.mark.parametrize("shape", SHAPES)
def test_stream_matches_fp32_and_tile_kernel(cuda, C, shape, kmajor):
    M, K, N = shape
    g = torch.Generator().manual_seed(M + K + N)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(cuda, torch.bfloat16)
    B = W.t().contiguous() if kmajor else W  # dgrad form: [K][N]
    C.set_gemm_stream(1)
    rows = C.gemm_stream_rows(M, N, K, K, N, kmajor)
    assert rows > 0, "shape not served by the streaming kernel"
    out, st = C.gemm_nt(A, B, True, None, kmajor)
    C.set_gemm_stream(0)
    ref_tile, _ = C.gemm_nt(A, B, False, None, kmajor)
    torch.cuda.synchronize()
    ref = A.float() @ W.float().t()
    assert _rel(out, ref) < 5e-3
    # same fp32 accumulation of the same bf16 products: the two kernels agree to bf16 rounding
    assert float((out.float() - ref_tile.float()).abs().max()) <= float(ref.abs().max()) * 2 ** -7
    assert st.shape[0] == rows and st.shape[1:] == (N, 2)
    tot = st.double().sum(0)
    of = out.double()
    torch.testing.assert_close(tot[:, 0], of.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(tot[:, 1], (of * of).sum(0), rtol=1e-4, atol=1e-3)


def test_stream_row_strided_input(cuda, C):
    """A is a channel slice of a wider tensor (lda > K), as for a branch of a concatenated block input."""
    M, K, N = 12345, 64, 128
    g = torch.Generator().manual_seed(7)
    wide = torch.randn(M, 3 * K, generator=g).to(cuda, torch.bfloat16)
    A = wide[:, K:2 * K]
    W = (torch.randn(N, K, generator=g) * 0.1).to(cuda, torch.bfloat16)
    C.set_gemm_stream(1)
    if C.gemm_stream_rows(M, N, K, A.stride(0), N) == 0:
        pytest.skip("strided input not served")
    out, _ = C.gemm_nt(A, W, False)
    torch.cuda.synchronize()
    assert _rel(out, A.float() @ W.float().t()) < 5e-3


def test_small_m_stays_on_tile_kernel(cuda, C):
    C.set_gemm_stream(1)
    # fewer than 2 tiles per row group: the tile kernel serves it (nothing for the ring to overlap)
    assert C.gemm_stream_rows(1000, 256, 64, 64, 256) == 0
    assert C.gemm_stream_rows(100000, 256, 512, 512, 256) == 0  # K = 512: not served
    # default policy (environment mode): forward K = 256 stays on the tile kernel, dgrad K = 256 streams
    C.set_gemm_stream(-1)
    assert C.gemm_stream_rows(802816, 512, 256, 256, 512, True, True) == 0  # addend form: K <= 128
    assert C.gemm_stream_rows(802816, 512, 256, 256, 512, False) == 0
    assert C.gemm_stream_rows(802816, 512, 256, 256, 512, True) > 0


@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("shape", [(9000, 64, 256), (20000, 128, 512), (5001, 128, 128), (70000, 64, 64)])
def test_stream_dgrad_addend_matches_tile_kernel(cuda, C, shape, masked):
    """The fused identity-gradient epilogue: C = bf16(bf16(dY W) + (bit ? D : 0)); same bf16 products in
    the same k order as the tile kernel, so the two agree bit for bit."""
    M, K, N = shape
    g = torch.Generator().manual_seed(M + 3 * K + N)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    B = (torch.randn(K, N, generator=g) * K ** -0.5).to(cuda, torch.bfloat16)
    D = torch.randn(M, N, generator=g).to(cuda, torch.bfloat16)
    mask = torch.randint(0, 256, ((M * N + 7) // 8,), generator=g, dtype=torch.uint8).to(cuda) if masked else None
    C.set_gemm_stream(1)
    assert C.gemm_stream_rows(M, N, K, K, N, True, True) > 0
    out, _ = C.gemm_nt(A, B, False, D, True, 0, mask)
    C.set_gemm_stream(0)
    ref, _ = C.gemm_nt(A, B, False, D, True, 0, mask)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # and against the definition
    bits = torch.ones(M * N, device=cuda) if mask is None else \
        torch.stack([(mask >> j) & 1 for j in range(8)], 1).reshape(-1)[: M * N].float()
    exp = ((A.float() @ B.float()).to(torch.bfloat16).float() + D.float() * bits.view(M, N)).to(torch.bfloat16)
    assert float((out.float() - exp.float()).abs().max()) <= float(exp.float().abs().max()) * 2 ** -6


@pytest.mark.parametrize("kmajor", [False, True])
@pytest.mark.parametrize("shape", SHAPES + [(12544, 128, 64)])
def test_stream_without_statistics_writes_every_row(cuda, C, shape, kmajor):
    """The statistics-free instantiations (data gradients, plain forwards). The output block is poisoned
    with NaN first, so a tile whose stores were skipped cannot pass on stale correct values left in a
    recycled allocation (the K = 128 instantiation skipped every tile after the peeled prologue while an
    inline-asm M0 advance clobbered the SCC branch condition; dla_mfma.h bglds)."""
    M, K, N = shape
    g = torch.Generator().manual_seed(M * 3 + K + N)
    A = torch.randn(M, K, generator=g).to(cuda, torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(cuda, torch.bfloat16)
    B = W.t().contiguous() if kmajor else W
    C.set_gemm_stream(1)
    assert C.gemm_stream_rows(M, N, K, K, N, kmajor) > 0
    poison = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
    del poison  # the caching allocator hands this block to the next [M, N] bf16 output
    out, st = C.gemm_nt(A, B, False, None, kmajor)
    torch.cuda.synchronize()
    assert st is None or st.numel() == 0
    assert torch.isfinite(out).all(), f"{int((~torch.isfinite(out)).any(1).sum())} rows never written"
    assert _rel(out, A.float() @ W.float().t()) < 5e-3
