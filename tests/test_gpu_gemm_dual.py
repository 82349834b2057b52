"""One-pass data + weight gradient of a stride-1 1x1 conv (csrc/kernels/gemm_dual.hip) vs the separate
kernels and fp32 PyTorch (gpu).

Shapes: the ResNet-50 stage-1 / stage-2 shapes it serves ((Cin, Cout) = (64, 256), (128 / 256, 512), the
latter as 64-channel slices sharing the dY tiles), ragged row counts (last tile partly
past the end: zero-filled loads, dropped stores), row groups with one tile fewer than others; then the
conv autograd path with the kernel on and off."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def C():
    from distributed_learning_amd.ops import _ext

    return _ext.require()


@pytest.mark.parametrize("M,ci,co", [(65536, 64, 256), (70001, 64, 256), (200003, 64, 256), (1 << 20, 64, 256),
                                     (16384, 128, 512), (50001, 128, 512), (40003, 256, 512), (131072, 256, 512)])
@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
def test_dual_matches_separate_kernels_and_fp32(cuda, C, M, ci, co, odt):
    g = torch.Generator().manual_seed(M + ci)
    dy = torch.randn(M, co, generator=g).to(cuda, torch.bfloat16)
    x = torch.randn(M, ci, generator=g).to(cuda, torch.bfloat16)
    w = (torch.randn(co, ci, generator=g) * co ** -0.5).to(cuda, torch.bfloat16)
    assert C.conv1x1_dual_blocks(M, ci, co) == 256
    dx, dw = C.conv1x1_dual(dy, x, w, odt)
    dx_ref, _ = C.gemm_nt(dy, w, False, None, True)  # the data gradient as the step runs it otherwise
    torch.cuda.synchronize()
    ref = dy.float() @ w.float()
    scale = float(ref.abs().max())
    assert float((dx.float() - dx_ref.float()).abs().max()) <= scale * 2 ** -7
    assert float((dx.float() - ref).norm() / ref.norm()) < 5e-3
    dw_ref = dy.double().t() @ x.double()
    assert dw.dtype == odt and dw.shape == (co, ci)
    rel = float((dw.double() - dw_ref).norm() / dw_ref.norm())
    assert rel < (1e-5 if odt == torch.float32 else 5e-3), rel
    dw_tn = C.gemm_tn(dy, x, odt, 1.0)
    assert float((dw.double() - dw_tn.double()).norm() / dw_ref.norm()) < (1e-5 if odt == torch.float32 else 8e-3)


def test_dual_not_served_shapes(C):
    assert C.conv1x1_dual_blocks(1000, 64, 256) == 0  # too few tiles
    assert C.conv1x1_dual_blocks(1 << 20, 256, 1024) == 0  # weight panel too large for LDS
    assert C.conv1x1_dual_blocks(1 << 20, 256, 64) == 0
    assert C.conv1x1_dual_blocks(1 << 20, 512, 512) == 0
    assert C.conv1x1_dual_bn_ok(1 << 20, 64, 256) and not C.conv1x1_dual_bn_ok(1 << 20, 128, 512)


def test_conv_autograd_uses_dual_and_matches(cuda):
    """_Conv1x1.backward with the one-pass kernel vs the separate kernels: same data gradient (same
    MFMA order), weight gradient to fp32 summation-order noise."""
    import torch.nn as nn

    from distributed_learning_amd.ops import conv as nconv

    torch.manual_seed(0)
    m = nn.Conv2d(64, 256, 1, bias=False).to(cuda).to(memory_format=torch.channels_last)
    m.weight.data = m.weight.data.to(torch.bfloat16)
    x0 = torch.randn(24, 64, 56, 56, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(24, 256, 56, 56, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def run(flag):
        old = nconv.DUAL_1X1
        nconv.DUAL_1X1 = flag
        try:
            m.weight.grad = None
            x = x0.clone().requires_grad_(True)
            y, _ = nconv.conv1x1(x, m)
            y.backward(gy)
            return x.grad.float(), m.weight.grad.float()
        finally:
            nconv.DUAL_1X1 = old

    dx1, dw1 = run(True)
    dx0, dw0 = run(False)
    assert float((dx1 - dx0).abs().max()) <= float(dx0.abs().max()) * 2 ** -7
    assert float((dw1 - dw0).norm() / dw0.norm()) < 1e-2


@pytest.mark.parametrize("M,ci,co", [(65536, 64, 256), (100003, 64, 256)])
def test_dual_with_bn_apply_matches_separate(cuda, C, M, ci, co):
    """kBN: the consuming BN(+residual)+ReLU's backward apply inside the kernel (gradient, BN input, bit mask,
    finalized coefficients) == bn_act_bwd's apply pass followed by the plain one-pass kernel."""
    g = torch.Generator().manual_seed(M + ci)
    dout = torch.randn(M, co, generator=g).to(cuda, torch.bfloat16)
    ybn = (torch.randn(M, co, generator=g) * 2 + 0.5).to(cuda, torch.bfloat16)
    x = torch.randn(M, ci, generator=g).to(cuda, torch.bfloat16)
    w = (torch.randn(co, ci, generator=g) * co ** -0.5).to(cuda, torch.bfloat16)
    mask = torch.randint(0, 256, ((M * co + 7) // 8,), generator=g, dtype=torch.uint8).to(cuda)
    gamma = (torch.rand(co, generator=g) + 0.5).to(cuda)
    yf = ybn.float()
    ws = torch.zeros(7 * co, device=cuda)
    ws[:co] = yf.mean(0)
    ws[co:2 * co] = (yf.var(0, unbiased=False) + 1e-5).rsqrt()
    ws_a, ws_b = ws.clone(), ws.clone()
    assert C.conv1x1_dual_bn_ok(M, ci, co)
    dY, _, dg, db = C.bn_act_bwd(dout, None, mask, ybn, ws_a, gamma, 2, False, None)
    dx_ref, dw_ref = C.conv1x1_dual(dY, x, w, torch.float32)
    _, _, dg2, db2 = C.bn_act_bwd(dout, None, mask, ybn, ws_b, gamma, 2, False, None, False)
    dx, dw = C.conv1x1_dual(dout, x, w, torch.float32, ybn, ws_b, mask)
    torch.cuda.synchronize()
    assert torch.equal(ws_a, ws_b) and torch.equal(dg, dg2) and torch.equal(db, db2)
    scale = float(dx_ref.float().abs().max())
    assert float((dx.float() - dx_ref.float()).abs().max()) <= scale * 2 ** -7
    ref = dY.float() @ w.float()
    assert float((dx.float() - ref).norm() / ref.norm()) < 5e-3
    assert float((dw - dw_ref).norm() / dw_ref.norm()) < 1e-5


def test_resnet_with_and_without_fused_bn_apply(cuda):
    """Whole ResNet-50 step: the BN-apply hand-off (BN backward stops after its reduction, the conv3 backward
    applies it inside the one-pass kernel) reproduces the unfused gradients up to fp32 summation order."""
    from distributed_learning_amd.models import resnet50
    from distributed_learning_amd.ops import conv as nconv
    from distributed_learning_amd.ops import nn as dnn

    CL = torch.channels_last

    def run(flag):
        torch.manual_seed(0)
        m = resnet50(10).to(cuda).to(memory_format=CL)
        dnn.bf16_weights(m)
        x = torch.randn(24, 3, 224, 224, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
        old = nconv.DUAL_BN
        nconv.DUAL_BN = flag
        before = nconv.CALLS["1x1_dual_bn"]
        try:
            m(x).float().square().mean().backward()
        finally:
            nconv.DUAL_BN = old
        # stage 1: the conv3 of blocks 1 and 2, and block 0's conv3 + downsample conv (its dual BN hands both over)
        assert (nconv.CALLS["1x1_dual_bn"] - before == 4) == flag
        return {n: p.grad.float().clone() for n, p in m.named_parameters()}

    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        g1, g0 = run(True), run(False)
    finally:
        dnn.set_native_conv(False)
        dnn.set_backend("torch")
    rels = sorted(float((g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-20)) for n in g0)
    assert rels[len(rels) // 2] < 2e-2 and rels[-1] < 0.2, rels[-5:]


def test_bn_handoff_falls_back_when_output_has_other_consumers(cuda):
    """The conv output feeding the block-final BN is ALSO used elsewhere: autograd sums the BN's placeholder
    gradient with the other one, the conv backward sees a different tensor, materialises the BN's gradient and
    adds it -- the same gradients as without the hand-off."""
    import torch.nn as nn

    from distributed_learning_amd.ops import bn_act
    from distributed_learning_amd.ops import conv as nconv
    from distributed_learning_amd.ops import nn as dnn

    CL = torch.channels_last
    torch.manual_seed(0)
    c1 = nn.Conv2d(256, 64, 1, bias=False).to(cuda).to(memory_format=CL)
    c3 = nn.Conv2d(64, 256, 1, bias=False).to(cuda).to(memory_format=CL)
    for c in (c1, c3):
        c.weight.data = c.weight.data.to(torch.bfloat16)
    bn = nn.BatchNorm2d(256).to(cuda)
    x0 = torch.randn(24, 256, 56, 56, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    h0 = torch.randn(24, 64, 56, 56, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    wgt = torch.randn(24, 256, 56, 56, device=cuda).contiguous(memory_format=CL)

    def run(flag, extra):
        old = nconv.DUAL_BN
        nconv.DUAL_BN = flag
        try:
            for p in (c1.weight, c3.weight, bn.weight, bn.bias):
                p.grad = None
            x = x0.clone().requires_grad_(True)
            h = h0.clone().requires_grad_(True)
            _, _, ident, _ = nconv.conv1x1_fork(x, c1)          # the identity alias with its residual hand-off
            y3, st = nconv.conv1x1(h, c3, want_stats=True)      # carries the BN hand-off link when flag
            out = bn_act.fused_bn_act(y3, bn, True, ident, st)
            loss = (out.float() * wgt).sum()
            if extra:
                loss = loss + (y3.float() * wgt).square().mean()  # a second consumer of the conv output
            before = nconv.CALLS["1x1_dual_bn"]
            loss.backward()
            fused = nconv.CALLS["1x1_dual_bn"] - before
            # (conv1's own output is unused here: only its identity alias carries a gradient)
            return fused, [t.float().clone() for t in (x.grad, h.grad, c3.weight.grad, bn.weight.grad, bn.bias.grad)]
        finally:
            nconv.DUAL_BN = old

    dnn.set_backend("native")
    n_alone, g_alone = run(True, False)
    n_extra, g_extra = run(True, True)
    _, g_ref_alone = run(False, False)
    _, g_ref_extra = run(False, True)
    assert n_alone == 1 and n_extra == 0  # fused when the BN is the only consumer; materialised otherwise
    for a, b in zip(g_extra, g_ref_extra):
        assert float((a - b).norm() / b.norm().clamp_min(1e-20)) < 1e-2
    for a, b in zip(g_alone, g_ref_alone):
        assert float((a - b).norm() / b.norm().clamp_min(1e-20)) < 1e-2


def _two_bn_setup(cuda):
    import torch.nn as nn

    CL = torch.channels_last
    torch.manual_seed(1)
    convs = [nn.Conv2d(256, 64, 1, bias=False), nn.Conv2d(256, 64, 1, bias=False), nn.Conv2d(64, 256, 1, bias=False)]
    convs = [c.to(cuda).to(memory_format=CL) for c in convs]
    for c in convs:
        c.weight.data = c.weight.data.to(torch.bfloat16)
    bns = [nn.BatchNorm2d(256).to(cuda), nn.BatchNorm2d(256).to(cuda)]
    mk = lambda *s: torch.randn(*s, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)  # noqa: E731
    return convs, bns, mk(24, 256, 56, 56), mk(24, 256, 56, 56), mk(24, 64, 56, 56), \
        torch.randn(24, 256, 56, 56, device=cuda).contiguous(memory_format=CL)


def test_bn_handoff_one_conv_output_two_bns(cuda):
    """one conv output consumed by TWO fused BN(+residual)+ReLU calls. Only the first BN may claim the
    conv's hand-off link (a second park would overwrite the first BN's parked gradient and lose it); the second
    runs the normal path. Gradients must equal the run without the hand-off. With retain_grad() on the conv
    output, nothing is handed off and the retained gradient is the real one, not the placeholder's zeros."""
    from distributed_learning_amd.ops import bn_act
    from distributed_learning_amd.ops import conv as nconv
    from distributed_learning_amd.ops import nn as dnn

    (c1a, c1b, c3), (bn1, bn2), xa0, xb0, h0, wgt = _two_bn_setup(cuda)

    def run(flag, retain):
        old = nconv.DUAL_BN
        nconv.DUAL_BN = flag
        try:
            for p in (c1a.weight, c1b.weight, c3.weight, bn1.weight, bn1.bias, bn2.weight, bn2.bias):
                p.grad = None
            xa, xb, h = (t.clone().requires_grad_(True) for t in (xa0, xb0, h0))
            _, _, ia, _ = nconv.conv1x1_fork(xa, c1a)
            _, _, ib, _ = nconv.conv1x1_fork(xb, c1b)
            y3, st = nconv.conv1x1(h, c3, want_stats=True)
            if retain:
                y3.retain_grad()
            out = bn_act.fused_bn_act(y3, bn1, True, ia, st) + bn_act.fused_bn_act(y3, bn2, True, ib, st)
            before = nconv.CALLS["1x1_dual_bn"]
            (out.float() * wgt).sum().backward()
            fused = nconv.CALLS["1x1_dual_bn"] - before
            gs = [t.float().clone() for t in (xa.grad, xb.grad, h.grad, c3.weight.grad, bn1.weight.grad,
                                              bn2.weight.grad, bn1.bias.grad, bn2.bias.grad)]
            return fused, gs, (y3.grad.float().clone() if retain else None)
        finally:
            nconv.DUAL_BN = old

    dnn.set_backend("native")
    try:
        n_on, g_on, _ = run(True, False)
        n_ret, g_ret, y_ret = run(True, True)
        _, g_ref, y_ref = run(False, True)
    finally:
        dnn.set_backend("torch")
    assert n_on == 0 and n_ret == 0  # two consumers: the conv sees a summed gradient and materialises
    for got in (g_on, g_ret):
        for a, b in zip(got, g_ref):
            assert float((a - b).norm() / b.norm().clamp_min(1e-20)) < 1e-2
    assert float(y_ret.abs().max()) > 0 and float((y_ret - y_ref).norm() / y_ref.norm()) < 1e-2
