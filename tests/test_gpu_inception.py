"""Native Inception block (ops/inception.py): concat-free BN+ReLU into channel slices, strided-dy BN
backward, and the fan-in node that sums x's four gradients in GEMM epilogues (gpu)."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def test_bn_act_into_slice_and_strided_dy(cuda):
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    torch.manual_seed(0)
    x = torch.randn(3, 24, 7, 9, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.rand(24, device=cuda) + 0.5
    b = torch.randn(24, device=cuda)
    rm, rv = torch.zeros(24, device=cuda), torch.ones(24, device=cuda)
    y_ref, ws_ref, _ = C.bn_act_fwd(x, None, g, b, rm.clone(), rv.clone(), True, 0.1, 1e-3, True)
    out = torch.full((3, 64, 7, 9), 7.0, device=cuda, dtype=torch.bfloat16).contiguous(memory_format=CL)
    y, ws, _ = C.bn_act_fwd(x, None, g, b, rm.clone(), rv.clone(), True, 0.1, 1e-3, True, None, out, 16)
    assert torch.equal(out[:, 16:40], y_ref) and torch.equal(y, y_ref)
    assert bool((out[:, :16] == 7).all()) and bool((out[:, 40:] == 7).all())  # neighbours untouched
    dout = torch.randn(3, 64, 7, 9, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    dsl = dout[:, 16:40]
    a = C.bn_act_bwd(dsl, None, None, x, ws.clone(), g, 1, False, None)
    r = C.bn_act_bwd(dsl.contiguous(memory_format=CL), None, None, x, ws.clone(), g, 1, False, None)
    for u, v in zip(a, r):
        if u is not None:
            assert torch.equal(u, v)


@pytest.mark.parametrize("shape", [(4, 7, 9), (35, 80, 50)])  # the second has > 1024 epilogue row tiles (fold path)
def test_bn_concat_matches_per_branch(cuda, shape):
    """Grouped BN+ReLU over concatenated branches == one bn_act_fwd / bn_act_bwd chain per branch."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    torch.manual_seed(0)
    n, h, w = shape
    chans = [64, 96, 24, 208]
    ys, sts, gs, bs, rms, rvs = [], [], [], [], [], []
    for c in chans:
        a = torch.randn(n * h * w, 32, device=cuda).to(torch.bfloat16)
        wt = torch.randn(c, 32, device=cuda).to(torch.bfloat16)
        y2, st = C.gemm_nt(a, wt, True)  # the conv epilogue's statistics, as in the fused block
        ys.append(y2.view(n, h, w, c).permute(0, 3, 1, 2))
        sts.append(st)
        gs.append(torch.rand(c, device=cuda) + 0.5)
        bs.append(torch.randn(c, device=cuda))
        rms.append(torch.randn(c, device=cuda))
        rvs.append(torch.rand(c, device=cuda) + 0.5)
    ctot = sum(chans)
    out_g = torch.zeros(n, ctot, h, w, device=cuda, dtype=torch.bfloat16).contiguous(memory_format=CL)
    out_r = torch.zeros_like(out_g)
    rm_g, rv_g = [t.clone() for t in rms], [t.clone() for t in rvs]
    wss_g = C.bn_concat_fwd(ys, gs, bs, rm_g, rv_g, [0.1] * 4, [1e-3] * 4, sts, out_g)
    wss_r, off = [], 0
    for i, c in enumerate(chans):
        _, ws, _ = C.bn_act_fwd(ys[i], None, gs[i], bs[i], rms[i], rvs[i], True, 0.1, 1e-3, True, sts[i], out_r, off)
        wss_r.append(ws)
        off += c
    assert torch.equal(out_g, out_r)
    for a, b in zip(rm_g + rv_g, rms + rvs):
        assert torch.equal(a, b)
    for a, b in zip(wss_g, wss_r):
        assert torch.equal(a[:4 * a.numel() // 7], b[:4 * b.numel() // 7])
    dout = torch.randn(n, ctot, h, w, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    got = C.bn_concat_bwd(dout, ys, gs, wss_g)
    off = 0
    for i, c in enumerate(chans):
        dx, _, dg, db = C.bn_act_bwd(dout[:, off:off + c], None, None, ys[i], wss_r[i], gs[i], 1, False, None)
        gdx, gdg, gdb = got[3 * i:3 * i + 3]
        assert gdx.shape == dx.shape and gdx.is_contiguous(memory_format=CL)
        assert _rel(gdx, dx) < 1e-2 and _rel(gdg, dg) < 1e-4 and _rel(gdb, db) < 1e-4, (i, _rel(gdx, dx))
        off += c


@pytest.mark.parametrize("shape", [(4, 7, 9), (35, 80, 50)])
def test_bn_group_separate_outputs_with_epilogue_partials(cuda, shape):
    """bn_group_fwd / bn_group_bwd (the two reduction-branch BNs) == per-branch bn_act_fwd / bn_act_bwd,
    with the backward's reduction partials coming from the consumer GEMM's dgrad epilogue."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    torch.manual_seed(1)
    n, h, w = shape
    chans = [96, 16]
    ys, sts, gs, bs, rms, rvs = [], [], [], [], [], []
    for c in chans:
        a = torch.randn(n * h * w, 32, device=cuda).to(torch.bfloat16)
        wt = torch.randn(c, 32, device=cuda).to(torch.bfloat16)
        y2, st = C.gemm_nt(a, wt, True)
        ys.append(y2.view(n, h, w, c).permute(0, 3, 1, 2))
        sts.append(st)
        gs.append(torch.rand(c, device=cuda) + 0.5)
        bs.append(torch.randn(c, device=cuda))
        rms.append(torch.zeros(c, device=cuda))
        rvs.append(torch.ones(c, device=cuda))
    res = C.bn_group_fwd(ys, gs, bs, [t.clone() for t in rms], [t.clone() for t in rvs], [0.1] * 2, [1e-3] * 2, sts)
    outs, wss = res[:2], res[2:]
    for i in range(2):
        y_r, ws_r, _ = C.bn_act_fwd(ys[i], None, gs[i], bs[i], rms[i].clone(), rvs[i].clone(), True, 0.1, 1e-3, True,
                                    sts[i])
        assert torch.equal(outs[i], y_r) and outs[i].is_contiguous(memory_format=CL)
        assert torch.equal(wss[i][:4 * chans[i]], ws_r[:4 * chans[i]])
    # each BN's dy comes from a consumer GEMM (dgrad of a 1x1 conv) whose epilogue also emits the
    # BN backward partials (mode 1: ReLU recomputed from the BN input)
    dys, parts = [], []
    for i, c in enumerate(chans):
        g2 = torch.randn(n * h * w, 64, device=cuda).to(torch.bfloat16)
        wk = torch.randn(64, c, device=cuda).to(torch.bfloat16)
        dy2, part = C.gemm_nt_bn(g2, wk, None, True, ys[i].permute(0, 2, 3, 1).reshape(-1, c), wss[i], None, 1,
                                 None, None, 0, 0)
        dys.append(dy2.view(n, h, w, c).permute(0, 3, 1, 2))
        parts.append(part)
    for exts in (parts, []):
        got = C.bn_group_bwd(dys, ys, gs, [ws.clone() for ws in wss], exts)
        for i in range(2):
            dx, _, dg, db = C.bn_act_bwd(dys[i], None, None, ys[i], wss[i].clone(), gs[i], 1, False,
                                         parts[i] if exts else None)
            gdx, gdg, gdb = got[3 * i:3 * i + 3]
            assert _rel(gdx, dx) < 1e-2 and _rel(gdg, dg) < 1e-4 and _rel(gdb, db) < 1e-4, (i, len(exts))


@pytest.mark.parametrize("shape", [(4, 7, 9), (35, 80, 50)])
def test_bn_group_strided_inputs_and_dx_slices(cuda, shape):
    """Branch inputs, their statistics and the dx outputs as channel slices of wider tensors (the
    fused fan-in GEMM's layout) give bit-identical results to the contiguous call."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    torch.manual_seed(2)
    n, h, w = shape
    chans = [64, 96, 16]
    ctot = sum(chans)
    a = torch.randn(n * h * w, 32, device=cuda).to(torch.bfloat16)
    wt = torch.randn(ctot, 32, device=cuda).to(torch.bfloat16)
    ycat, scat = C.gemm_nt(a, wt, True)
    y4 = ycat.view(n, h, w, ctot).permute(0, 3, 1, 2)
    offs = [0, 64, 160]
    ys_s = [y4[:, o:o + c] for o, c in zip(offs, chans)]
    st_s = [scat[:, o:o + c] for o, c in zip(offs, chans)]
    ys_c = [y.contiguous(memory_format=CL) for y in ys_s]
    st_c = [st.contiguous() for st in st_s]
    gs = [torch.rand(c, device=cuda) + 0.5 for c in chans]
    bs = [torch.randn(c, device=cuda) for c in chans]
    rm = [torch.zeros(c, device=cuda) for c in chans]
    rv = [torch.ones(c, device=cuda) for c in chans]
    args = ([0.1] * 3, [1e-3] * 3)
    rs = C.bn_group_fwd(ys_s, gs, bs, [t.clone() for t in rm], [t.clone() for t in rv], *args, st_s)
    rc = C.bn_group_fwd(ys_c, gs, bs, [t.clone() for t in rm], [t.clone() for t in rv], *args, st_c)
    for i, c in enumerate(chans):
        assert torch.equal(rs[i], rc[i])
        assert torch.equal(rs[3 + i][:4 * c], rc[3 + i][:4 * c])  # ws: [mean, invstd, scale, shift | bwd]
    dys = [torch.randn(n, c, h, w, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL) for c in chans]
    buf = torch.full((n, ctot, h, w), 7.0, device=cuda, dtype=torch.bfloat16).contiguous(memory_format=CL)
    outs = [buf[:, o:o + c] for o, c in zip(offs, chans)]
    gs_ = C.bn_group_bwd(dys, ys_s, gs, rs[3:], [], outs)
    gc_ = C.bn_group_bwd(dys, ys_c, gs, rc[3:], [])
    for i in range(3):
        assert gs_[3 * i].data_ptr() == outs[i].data_ptr()
        for u, v in zip(gs_[3 * i:3 * i + 3], gc_[3 * i:3 * i + 3]):
            assert torch.equal(u, v)


def test_dgrad_bn_epilogue_reads_strided_bn_input(cuda):
    """The 3x3 dgrad's BN-backward epilogue reading its BN input as a channel slice (fused fan-in
    layout) == reading a contiguous copy, bitwise."""
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    torch.manual_seed(4)
    n, h, w, cin, ctot, off = 4, 14, 14, 96, 176, 64
    big = torch.randn(n, ctot, h, w, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    xs = big[:, off:off + cin]
    xc = xs.contiguous(memory_format=CL)
    ws = torch.cat([torch.randn(cin, device=cuda) * 0.1, torch.rand(cin, device=cuda) + 0.5,
                    torch.rand(cin, device=cuda) + 0.5, torch.randn(cin, device=cuda) * 0.1,
                    torch.zeros(3 * cin, device=cuda)])
    dy = torch.randn(n, 128, h, w, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    wt = torch.randn(128, cin, 3, 3, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    a = C.conv3x3_dgrad_bn(dy, wt, None, xs, ws, None, 1)
    b = C.conv3x3_dgrad_bn(dy, wt, None, xc, ws, None, 1)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def _block():
    from distributed_learning_amd.models.googlenet import Inception
    from distributed_learning_amd.ops import nn as dnn

    torch.manual_seed(1)
    m = Inception(192, 64, 96, 128, 16, 32, 32).cuda().to(memory_format=CL)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            with torch.no_grad():
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.3, 0.3)
    dnn.bf16_weights(m)
    return m


def _run(m, x, g, fused):
    from distributed_learning_amd.ops import inception as ninc
    from distributed_learning_amd.ops import nn as dnn

    orig = ninc.supported
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    if not fused:
        ninc.supported = lambda *a: False
    try:
        assert ninc.supported(m, x) == fused
        xi = x.clone().requires_grad_(True)
        y = m(xi)
        y.backward(g)
        from distributed_learning_amd.ops.bn_act import flush_bn_counters

        flush_bn_counters()
    finally:
        ninc.supported = orig
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
    return y.detach(), xi.grad, {n: p.grad.clone() for n, p in m.named_parameters()}


def test_fused_inception_matches_unfused_and_fp32(cuda):
    base = _block()
    mf, mu = copy.deepcopy(base), copy.deepcopy(base)
    ref = copy.deepcopy(base)
    for p in ref.parameters():
        p.data = p.data.float()
    torch.manual_seed(2)
    x = torch.randn(4, 192, 14, 14, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    g = torch.randn(4, 256, 14, 14, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    yf, dxf, gf = _run(mf, x, g, True)
    yu, dxu, gu = _run(mu, x, g, False)
    # same convs, same statistics, same apply kernel: the forward output is bit-identical
    assert yf.shape == (4, 256, 14, 14) and yf.is_contiguous(memory_format=CL)
    assert torch.equal(yf, yu)
    for (n, a), (_, b) in zip(mf.named_buffers(), mu.named_buffers()):
        torch.testing.assert_close(a, b, rtol=0, atol=0, msg=n)
    # fp32 reference of the whole block
    xr = x.float().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g.float())
    assert _rel(yf, yr) < 2e-2
    # gradients: the fused fan-in sums x's four gradients in fp32 epilogues (unfused: bf16 adds)
    assert _rel(dxf, xr.grad) <= 1.5 * _rel(dxu, xr.grad) + 1e-3, (_rel(dxf, xr.grad), _rel(dxu, xr.grad))
    for n, p in ref.named_parameters():
        ef, eu = _rel(gf[n].float(), p.grad), _rel(gu[n].float(), p.grad)
        assert ef <= 1.5 * eu + 2e-3, (n, ef, eu)


def test_googlenet_uses_fused_blocks(cuda):
    """Every Inception block of GoogLeNet takes the fused path with native kernels."""
    from distributed_learning_amd.models import googlenet
    from distributed_learning_amd.ops import inception as ninc
    from distributed_learning_amd.ops import nn as dnn

    m = googlenet(10).cuda().to(memory_format=CL)
    dnn.bf16_weights(m)
    calls = []
    orig = ninc.inception_forward

    def spy(block, x):
        calls.append(block)
        return orig(block, x)

    ninc.inception_forward = spy
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        x = torch.rand(2, 3, 96, 96, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
        out = m(x)
        F.cross_entropy(out.float(), torch.tensor([1, 2], device=cuda)).backward()
    finally:
        ninc.inception_forward = orig
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
    assert len(calls) == 9
    assert all(p.grad is not None for n, p in m.named_parameters() if not n.startswith("aux"))
