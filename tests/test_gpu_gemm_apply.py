"""1x1-conv forward over a deferred BN(+residual)+ReLU output (csrc/kernels/gemm_apply.hip, ops/bn_act.py
PendingApply) vs the unfused apply pass + GEMM and vs fp32 PyTorch (gpu).

The fused kernel stages its A operand as relu(BN(y) + r) (or relu(BN(y) + BN_d(y_d))) with the apply kernel's
arithmetic, so the written block output, its ReLU mask, the GEMM output and the BN-statistics partials must equal
the unfused pair bit for bit (same 128-row register-staged tile, same k order). Shapes: ragged M, N = 64 / 128 /
256 (two column panels: only panel 0 writes the output), K = 256 / 512, identity and downsample (dual) residuals,
and the stage-1 shape of ResNet-50 at bench.py's batch. The model test runs a ResNet-50 training step with the
deferral on and off.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, K, N)
    (3000, 256, 64), (5001, 512, 128), (20000, 256, 128), (12345, 512, 256), (777, 256, 64),
]


def _case(cuda, M, K, N, dual, seed=0):
    g = torch.Generator(device=cuda).manual_seed(seed)
    y = torch.randn(M, K, generator=g, device=cuda).to(torch.bfloat16)
    r = (torch.randn(M, K, generator=g, device=cuda) * 0.7).to(torch.bfloat16)
    ws = torch.zeros(7 * K, device=cuda)
    ws[2 * K:3 * K] = torch.rand(K, generator=g, device=cuda) + 0.5
    ws[3 * K:4 * K] = torch.rand(K, generator=g, device=cuda) - 0.5
    wsd = None
    if dual:
        wsd = torch.zeros(7 * K, device=cuda)
        wsd[2 * K:3 * K] = torch.rand(K, generator=g, device=cuda) + 0.5
        wsd[3 * K:4 * K] = torch.rand(K, generator=g, device=cuda) - 0.5
    w = (torch.randn(N, K, generator=g, device=cuda) * K ** -0.5).to(torch.bfloat16)
    return y, r, ws, wsd, w


def _as4d(t):  # [M, K] rows as a channels_last [1, K, M, 1] tensor (bn_apply_deferred's input form)
    M, K = t.shape
    return t.view(1, M, 1, K).permute(0, 3, 1, 2)


@pytest.fixture
def wide_k():
    """Serve K up to 2048 and keep the unfused reference GEMM on the same register-staged main loop."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    C.set_gemm_apply_max_k(2048)
    C.set_mfma_pipeline(0)
    yield
    C.set_gemm_apply_max_k(-1)
    C.set_mfma_pipeline(-1)


@pytest.mark.parametrize("dual", [False, True])
@pytest.mark.parametrize("shape", SHAPES + [(4097, 1024, 256), (3001, 2048, 512), (1000, 1024, 512)])
def test_apply_gemm_matches_unfused_and_torch(cuda, wide_k, shape, dual):
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    M, K, N = shape
    y, r, ws, wsd, w = _case(cuda, M, K, N, dual)
    assert C.gemm_nt_apply_ok(M, N, K)
    out = torch.full((M, K), float("nan"), device=cuda, dtype=torch.bfloat16)
    mask = torch.zeros((M * K + 7) // 8, device=cuda, dtype=torch.uint8)
    c, st = C.gemm_nt_apply(y, r, ws, wsd, w, True, out, mask)
    # unfused: the apply pass, then the same 128-row register-staged tile over its output
    out_u = torch.empty_like(out)
    mask_u = torch.zeros_like(mask)
    C.bn_apply_deferred(_as4d(y), _as4d(r), ws, wsd, _as4d(out_u), mask_u)
    tile = 2 if N <= 64 else 1  # kTile128x64 / kTile128x128
    c_u, st_u = C.gemm_nt(out_u, w, True, None, False, tile)
    torch.cuda.synchronize()
    assert torch.equal(out, out_u)
    assert torch.equal(mask, mask_u)
    assert torch.equal(c, c_u)
    assert st.shape == st_u.shape == ((M + 127) // 128, N, 2)
    assert torch.equal(st, st_u)
    # fp32 PyTorch of the same op
    sc, sh = ws[2 * K:3 * K], ws[3 * K:4 * K]
    res = r.float() * wsd[2 * K:3 * K] + wsd[3 * K:4 * K] if dual else r.float()
    ref_out = torch.relu(y.float() * sc + sh + res)
    assert ((out.float() - ref_out).abs().max() <= 1e-2 * ref_out.abs().max()).item()
    ref_c = out.float() @ w.float().t()
    assert ((c.float() - ref_c).norm() / ref_c.norm()).item() < 5e-3
    bits = torch.stack([(mask >> j) & 1 for j in range(8)], 1).reshape(-1)[: M * K].reshape(M, K)
    assert torch.equal(bits.bool(), (y.float() * sc + sh + res) > 0) or \
        (bits.bool() != ((y.float() * sc + sh + res) > 0)).float().mean().item() < 1e-4  # fma vs mul+add ties
    csum = c.float().sum(0)
    assert torch.allclose(st[:, :, 0].sum(0), csum, rtol=1e-3, atol=1e-2 * csum.abs().max().item())


@pytest.mark.parametrize("n,H,W,K,N,dual", [(3, 14, 10, 256, 128, False), (2, 28, 28, 512, 256, True),
                                            (5, 6, 8, 256, 64, False)])
def test_apply_gemm_writes_stride2_subsample(cuda, n, H, W, K, N, dual):
    """At a stage transition the fused kernel also writes out[:, ::2, ::2] (the downsample conv's input)."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    M = n * H * W
    y, r, ws, wsd, w = _case(cuda, M, K, N, dual, seed=3)
    out = torch.empty((M, K), device=cuda, dtype=torch.bfloat16)
    mask = torch.empty((M * K + 7) // 8, device=cuda, dtype=torch.uint8)
    xs = torch.full((n, K, H // 2, W // 2), float("nan"), device=cuda, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    c, st = C.gemm_nt_apply(y, r, ws, wsd, w, True, out, mask, xs, H, W)
    c0, st0 = C.gemm_nt_apply(y, r, ws, wsd, w, True, torch.empty_like(out), torch.empty_like(mask))
    torch.cuda.synchronize()
    ref = out.view(n, H, W, K)[:, ::2, ::2].permute(0, 3, 1, 2)
    assert torch.equal(xs, ref)
    assert torch.equal(c, c0) and torch.equal(st, st0)


def test_apply_gemm_stage1_bench_shape(cuda):
    """conv1 of ResNet-50 layer1 blocks 2-3 at bench.py's batch (M = 1280 x 56 x 56, K 256, N 64)."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    M, K, N = 1280 * 56 * 56, 256, 64
    y, r, ws, wsd, w = _case(cuda, M, K, N, False, seed=1)
    out = torch.empty((M, K), device=cuda, dtype=torch.bfloat16)
    mask = torch.empty((M * K + 7) // 8, device=cuda, dtype=torch.uint8)
    xs = torch.empty((1280, K, 28, 28), device=cuda, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    c, st = C.gemm_nt_apply(y, r, ws, None, w, True, out, mask, xs, 56, 56)
    out_u = torch.empty_like(out)
    mask_u = torch.empty_like(mask)
    C.bn_apply_deferred(_as4d(y), _as4d(r), ws, None, _as4d(out_u), mask_u)
    del y, r
    assert torch.equal(xs, C.subsample2(out_u.view(1280, 56, 56, K).permute(0, 3, 1, 2)))
    c_u, st_u = C.gemm_nt(out_u, w, True, None, False, 2)
    torch.cuda.synchronize()
    assert torch.equal(out, out_u)
    assert torch.equal(mask, mask_u)
    assert torch.equal(c, c_u)
    assert torch.equal(st, st_u)
    tail = slice(M - 300, M)  # the last (partial) row tile against fp32
    ref = out[tail].float() @ w.float().t()
    assert ((c[tail].float() - ref).norm() / ref.norm()).item() < 5e-3


@pytest.mark.parametrize("M,K,N", [(20000, 64, 256), (50001, 128, 512), (1280 * 56 * 56, 64, 256)])
def test_stream_apply_matches_unfused_and_torch(cuda, M, K, N):
    """The streaming GEMM with a deferred BN+ReLU on its operand (gemm_stream.hip kAp): the written operand, the
    output and the statistics equal the apply pass + the same streaming kernel bit for bit."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    assert C.gemm_nt_stream_apply_ok(M, N, K)
    y, _, ws, _, w = _case(cuda, M, K, N, False, seed=5)
    out = torch.full((M, K), float("nan"), device=cuda, dtype=torch.bfloat16)
    c, st = C.gemm_nt_stream_apply(y, ws, w, out)
    out_u = torch.empty_like(out)
    C.bn_apply_deferred(_as4d(y), None, ws, None, _as4d(out_u), None)
    c_u, st_u = C.gemm_nt(out_u, w, True)  # the same streaming kernel without the transform
    torch.cuda.synchronize()
    assert torch.equal(out, out_u)
    assert torch.equal(c, c_u)
    assert st.shape == st_u.shape and torch.equal(st, st_u)
    rows = slice(M - 500, M)  # the last (partial) row tile against fp32
    ref_out = torch.relu(y[rows].float() * ws[2 * K:3 * K] + ws[3 * K:4 * K])
    assert ((out[rows].float() - ref_out).abs().max() <= 1e-2 * ref_out.abs().max()).item()
    ref_c = out[rows].float() @ w.float().t()
    assert ((c[rows].float() - ref_c).norm() / ref_c.norm()).item() < 5e-3
    csum = c.float().sum(0)
    assert torch.allclose(st[:, :, 0].sum(0), csum, rtol=1e-3, atol=1e-2 * csum.abs().max().item())


def _resnet_step(cuda, defer: bool, max_k: int = -1, mid: bool = False):
    from distributed_learning_amd import knobs
    from distributed_learning_amd.models.resnet import resnet50
    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops import bn_act
    from distributed_learning_amd.ops import conv as nconv
    from distributed_learning_amd.ops import nn as dnn

    C = _ext.require()
    torch.manual_seed(0)
    model = resnet50(num_classes=100).to(cuda).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    x = torch.randn(16, 3, 96, 96, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    tgt = torch.randint(0, 100, (16,), device=cuda)
    old = knobs._CACHE.get("DEFER_APPLY"), knobs._CACHE.get("DEFER_MID")
    knobs._CACHE["DEFER_APPLY"] = "1" if defer else "0"
    knobs._CACHE["DEFER_MID"] = "1" if mid else "0"
    C.set_tile256_min_k_stats(1 << 30)  # the same statistics tiles on both paths (bitwise comparison)
    C.set_gemm_apply_max_k(max_k)
    if max_k > 512:
        C.set_mfma_pipeline(0)  # the unfused K > 512 forwards on the fused kernel's main loop too
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    before = dict(bn_act.CALLS), nconv.CALLS["1x1_apply"], nconv.CALLS["1x1_stream_apply"]
    try:
        out = model(x)
        loss = torch.nn.functional.cross_entropy(out.float(), tgt)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
        C.set_tile256_min_k_stats(-1)
        C.set_gemm_apply_max_k(-1)
        C.set_mfma_pipeline(-1)
        for k, v in zip(("DEFER_APPLY", "DEFER_MID"), old):
            if v is None:
                knobs._CACHE.pop(k, None)
            else:
                knobs._CACHE[k] = v
    used = {k: bn_act.CALLS[k] - before[0][k] for k in bn_act.CALLS}
    used["fused"] = nconv.CALLS["1x1_apply"] - before[1]
    used["stream_fused"] = nconv.CALLS["1x1_stream_apply"] - before[2]
    grads = [p.grad.float().clone() for p in model.parameters()]
    stats = [b.clone() for b in model.buffers()]
    return out.float(), loss.item(), grads, stats, used


def test_resnet50_step_with_deferred_apply_matches(cuda):
    out_d, loss_d, g_d, s_d, used_d = _resnet_step(cuda, True)
    out_u, loss_u, g_u, s_u, used_u = _resnet_step(cuda, False)
    # 15 block outputs feed a next bottleneck; the 7 with K <= 512 are written by their consumer's GEMM
    assert used_d["deferred"] == 15 and used_d["fused"] == 7 and used_d["materialised"] == 8, used_d
    assert used_u["deferred"] == 0 and used_u["fused"] == 0, used_u
    assert loss_d == loss_u
    assert torch.equal(out_d, out_u)
    for a, b in zip(s_d, s_u):
        assert torch.equal(a, b)
    for i, (a, b) in enumerate(zip(g_d, g_u)):
        assert torch.equal(a, b), i


def test_resnet50_step_with_every_chained_output_deferred_matches(cuda):
    out_d, loss_d, g_d, s_d, used_d = _resnet_step(cuda, True, 2048)
    out_u, loss_u, g_u, s_u, used_u = _resnet_step(cuda, False, 2048)
    assert used_d["deferred"] == 15 and used_d["fused"] == 15 and used_d["materialised"] == 0, used_d
    assert loss_d == loss_u
    assert torch.equal(out_d, out_u)
    for a, b in zip(s_d, s_u):
        assert torch.equal(a, b)
    for i, (a, b) in enumerate(zip(g_d, g_u)):
        assert torch.equal(a, b), i


def test_resnet50_step_with_deferred_mid_bn_matches(cuda):
    """bn2 + ReLU written by conv3's streaming GEMM as well (DLA_DEFER_MID): bitwise the undeferred step."""
    out_d, loss_d, g_d, s_d, used_d = _resnet_step(cuda, True, mid=True)
    out_u, loss_u, g_u, s_u, used_u = _resnet_step(cuda, False, mid=False)
    # 16 bn2 outputs deferred on top of the 15 block outputs; the streaming kernel serves the stage-1 / 2 conv3s
    assert used_d["deferred"] == 31 and used_d["fused"] == 7 and used_d["stream_fused"] > 0, used_d
    assert used_d["materialised"] == 31 - 7 - used_d["stream_fused"], used_d
    assert loss_d == loss_u
    assert torch.equal(out_d, out_u)
    for a, b in zip(s_d, s_u):
        assert torch.equal(a, b)
    for i, (a, b) in enumerate(zip(g_d, g_u)):
        assert torch.equal(a, b), i


def test_deferred_output_is_materialised_for_other_consumers(cuda):
    """A bottleneck called on its own (outside ResNet.forward's deferral scope) never defers, and a hook on a
    chained block makes it write its output itself."""
    from distributed_learning_amd.models.resnet import resnet50
    from distributed_learning_amd.ops import bn_act
    from distributed_learning_amd.ops import nn as dnn

    torch.manual_seed(0)
    model = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    x = torch.randn(4, 3, 64, 64, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    from distributed_learning_amd import knobs

    seen = []
    old = knobs._CACHE.get("DEFER_APPLY"), knobs._CACHE.get("DEFER_MID")
    knobs._CACHE["DEFER_APPLY"] = "1"
    knobs._CACHE["DEFER_MID"] = "0"  # count the block outputs only
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        h = model.layer1[0].register_forward_hook(lambda m, i, o: seen.append(o.float().abs().sum().item()))
        before = bn_act.CALLS["deferred"]
        out = model(x)
        out.float().sum().backward()
        deferred = bn_act.CALLS["deferred"] - before
        h.remove()
        blk = model.layer1[1]
        t = torch.randn(4, 256, 16, 16, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        t.requires_grad_(True)
        before = bn_act.CALLS["deferred"]
        o = blk(t)
        alone = bn_act.CALLS["deferred"] - before
        torch.cuda.synchronize()
    finally:
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
        for k, v in zip(("DEFER_APPLY", "DEFER_MID"), old):
            if v is None:
                knobs._CACHE.pop(k, None)
            else:
                knobs._CACHE[k] = v
    assert deferred == 14  # the hooked block wrote its own output
    assert alone == 0 and bn_act.pending_of(o) is None
    assert seen and all(v == v and v > 0 for v in seen)
