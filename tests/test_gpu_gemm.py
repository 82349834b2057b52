"""bf16 MFMA GEMMs vs an fp32 PyTorch reference (gpu)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from distributed_learning_amd.ops import _ext

    return _ext.require()


@pytest.mark.parametrize("M,N,K", [(128, 64, 64), (1000, 64, 256), (777, 136, 72), (12544, 512, 2048),
                                   (4096, 256, 64), (130, 8, 8), (50176, 1024, 256),
                                   # >= 2048 tiles with K <= 256: the persistent short-K kernel
                                   (262181, 200, 136), (300000, 64, 64), (131072, 512, 128)])
def test_gemm_nt(cuda, M, N, K):
    C = _C()
    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    B = torch.randn(N, K, device=cuda).to(torch.bfloat16)
    out, stats = C.gemm_nt(A, B, True)
    ref = A.float() @ B.float().t()
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2 * (K ** 0.5))
    # fused column statistics of the rounded outputs
    s = stats.sum(0)
    o = out.float()
    torch.testing.assert_close(s[:, 0], o.sum(0), rtol=1e-4, atol=1e-2 * M ** 0.5)
    torch.testing.assert_close(s[:, 1], (o * o).sum(0), rtol=1e-4, atol=1e-1)


def test_gemm_nt_asymmetric_identity(cuda):
    """A = I with an asymmetric B catches a transposed C/D mapping (cdna_hip_programming.md §3)."""
    C = _C()
    n = 128
    A = torch.eye(n, device=cuda).to(torch.bfloat16)
    B = (torch.arange(n * n, device=cuda).reshape(n, n) % 251).to(torch.bfloat16)
    out, _ = C.gemm_nt(A, B, False)
    torch.testing.assert_close(out.float(), B.float().t())


@pytest.mark.parametrize("K,Mo,No", [(802816, 64, 256), (1000, 64, 64), (12544, 512, 2048), (333, 136, 72),
                                     (50176, 256, 1024), (3333, 512, 256), (131072, 8, 8), (65536, 24, 40), (200704, 64, 64)])
def test_gemm_tn(cuda, K, Mo, No):
    C = _C()
    torch.manual_seed(0)
    A = torch.randn(K, Mo, device=cuda).to(torch.bfloat16)
    B = torch.randn(K, No, device=cuda).to(torch.bfloat16)
    out = C.gemm_tn(A, B, torch.float32, 0.5)
    ref = (A.float().t() @ B.float()) * 0.5
    torch.testing.assert_close(out, ref, rtol=1e-3, atol=1e-3 * K ** 0.5)
    outb = C.gemm_tn(A, B, torch.bfloat16, 1.0)
    torch.testing.assert_close(outb.float(), ref * 2, rtol=1e-2, atol=2e-3 * K ** 0.5)


@pytest.mark.parametrize("M,N,K", [(1000, 64, 256), (777, 136, 72), (12544, 512, 2048), (130, 8, 8),
                                   (50176, 256, 1024), (262181, 200, 136), (300000, 64, 64)])
def test_gemm_nt_kmajor_b_and_addend(cuda, M, N, K):
    """b_kmajor: C = A @ B with B [K, N] (dgrad with the weight as stored); the fused addend gives
    bf16(bf16(A @ B) + D) exactly like the unfused add."""
    C = _C()
    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    B = torch.randn(K, N, device=cuda).to(torch.bfloat16)
    D = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    out, _ = C.gemm_nt(A, B, False, None, True)
    ref = A.float() @ B.float()
    torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-2 * (K ** 0.5))
    # same accumulation order as the n-major form -> bitwise equal
    out_t, _ = C.gemm_nt(A, B.t().contiguous(), False)
    assert torch.equal(out, out_t)
    out_d, _ = C.gemm_nt(A, B, False, D, True)
    assert torch.equal(out_d, out + D)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 8])
@pytest.mark.parametrize("M,N,K", [(1000, 64, 256), (777, 136, 72), (4096, 512, 128), (1300, 520, 640),
                                   (70000, 512, 256)])
def test_gemm_nt_tile_configs(cuda, tile, M, N, K):
    C = _C()
    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    B = torch.randn(N, K, device=cuda).to(torch.bfloat16)
    out, stats = C.gemm_nt(A, B, True, None, False, tile)
    ref, _ = C.gemm_nt(A, B, False, None, False, 1)
    assert torch.equal(out, ref)  # same k order in every tile shape
    torch.testing.assert_close(stats.sum(0)[:, 0], out.float().sum(0), rtol=1e-4, atol=1e-2 * M ** 0.5)
    outk, _ = C.gemm_nt(A, B.t().contiguous(), False, None, True, tile)
    if tile == 0 and C.gemm_nt_splitk_splits(M, N, K) > 1:  # auto without statistics may split K: other order
        assert float((outk.float() - ref.float()).abs().max()) <= float(ref.float().abs().max()) * 2 ** -7
    else:
        assert torch.equal(outk, ref)


def test_auto_tile_policy():
    """256x256 tiles from K = 1024 (N % 256 == 0, enough tiles to fill the chip), 128-row tiles otherwise;
    the threshold setter moves it (A/B runs)."""
    C = _C()
    # pick_tile(M, N, K, wide_ok)
    assert C.pick_tile(250880, 512, 1024, True) == 8
    assert C.pick_tile(1003520, 256, 512, True) == 1
    assert C.pick_tile(1003520, 512, 128, True) == 1
    assert C.pick_tile(4014080, 64, 256, True) == 2
    assert C.pick_tile(2000, 512, 1024, True) == 1  # 16 tiles: too few for 256 CUs
    assert C.pick_tile(250880, 512, 1024, False) == 1
    try:
        C.set_tile256_min_k(256)
        assert C.pick_tile(1003520, 512, 256, True) == 8
    finally:
        C.set_tile256_min_k(0)
    assert C.pick_tile(1003520, 512, 256, True) == 1


@pytest.mark.parametrize("pipe", [0, 2, 3, 4, 5, 6])
def test_mfma_pipelines_agree(cuda, pipe):
    """Register-staged and LDS-DMA (2/3-stage) main loops: identical results for every kernel
    family (same MFMA order), including ragged edges and the transposed-read operands."""
    C = _C()
    torch.manual_seed(0)
    A = torch.randn(1000, 200, device=cuda).to(torch.bfloat16)
    B = torch.randn(136, 200, device=cuda).to(torch.bfloat16)
    Bk = torch.randn(200, 136, device=cuda).to(torch.bfloat16)
    T1 = torch.randn(3000, 136, device=cuda).to(torch.bfloat16)
    T2 = torch.randn(3000, 72, device=cuda).to(torch.bfloat16)
    old = C.mfma_pipeline()
    try:
        C.set_mfma_pipeline(0)
        ref = [C.gemm_nt(A, B, True)[0], C.gemm_nt(A, Bk, False, None, True)[0], C.gemm_tn(T1, T2)]
        C.set_mfma_pipeline(pipe)
        got = [C.gemm_nt(A, B, True)[0], C.gemm_nt(A, Bk, False, None, True)[0], C.gemm_tn(T1, T2)]
    finally:
        C.set_mfma_pipeline(old)
    for r, g in zip(ref, got):
        assert torch.equal(r, g)
    torch.testing.assert_close(got[0].float(), A.float() @ B.float().t(), rtol=1e-2, atol=0.15)


@pytest.mark.parametrize("M,N,K,kmajor,addend", [(128, 1024, 2048, False, "bias"), (512, 1000, 2048, False, "bias"),
                                                (512, 2048, 1000, True, None), (300, 136, 1000, True, None),
                                                (8, 64, 4096, False, "bias")])
def test_gemm_nt_splitk_heads(cuda, M, N, K, kmajor, addend):
    """Few output tiles + long K take the split-K path (fp32 slabs, fixed-order reduce with the addend)."""
    C = _C()
    assert C.gemm_nt_splitk_splits(M, N, K) > 1
    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    W = torch.randn(N, K, device=cuda).to(torch.bfloat16)
    B = W.t().contiguous() if kmajor else W
    D = None
    if addend == "bias":
        D = torch.randn(N, device=cuda).to(torch.bfloat16).expand(M, N)
    elif addend == "rows":
        D = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    y, _ = C.gemm_nt(A, B, False, D, kmajor)
    ref = A.float() @ W.float().t() + (D.float() if D is not None else 0)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=2e-3 * K ** 0.5)
    y2, _ = C.gemm_nt(A, B, False, D, kmajor)
    assert torch.equal(y, y2)  # fixed-order reduction
