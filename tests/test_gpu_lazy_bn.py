"""relu(BN2) of a bottleneck normalised on load by its conv3 instead of written to HBM (gpu).

Kernels: the streaming GEMM's kNrm forward (gemm_stream.hip) and the one-pass gradient kernel's kXN X tiles
(gemm_dual.hip, plain and with the consuming BN's apply fused) against the same kernels fed the activation
materialised by bn_apply_ws -- bitwise, since both apply bn_apply's arithmetic to the same bf16 inputs.
Model: a ResNet-50 step with the lazy hand-off on and off gives bitwise equal gradients, running statistics
and BN counters. Fallback: shapes the kernels do not serve materialise the activation."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture
def C():
    from distributed_learning_amd.ops import _ext

    return _ext.require()


def _bn_input(cuda, C, M, ch, seed):
    """A channels_last [M/16, ch, 4, 4] BN input and its finalized training workspace."""
    g = torch.Generator().manual_seed(seed)
    y = (torch.randn(M // 16, 4, 4, ch, generator=g) * 1.5 + 0.2).to(cuda, torch.bfloat16).permute(0, 3, 1, 2)
    gamma = (torch.rand(ch, generator=g) + 0.5).to(cuda)
    beta = (torch.randn(ch, generator=g) * 0.3).to(cuda)
    rm, rv = torch.zeros(ch, device=cuda), torch.ones(ch, device=cuda)
    ws = C.bn_stats_ws(y, gamma, beta, rm, rv, 0.1, 1e-5, None)
    return y, ws, gamma


def _rows(t):
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


@pytest.mark.parametrize("M,K,N", [(100000, 64, 256), (200000, 64, 256), (50000, 128, 512), (80000, 128, 128),
                                   (40000, 64, 64)])
@pytest.mark.parametrize("stats", [True, False])
def test_stream_normalise_on_load_is_bitwise(cuda, C, M, K, N, stats):
    y, ws, _ = _bn_input(cuda, C, M, K, M + K)
    a = C.bn_apply_ws(y, ws, True)
    ref = torch.relu(y.float() * ws[2 * K:3 * K].view(1, K, 1, 1) + ws[3 * K:4 * K].view(1, K, 1, 1))
    assert float((a.float() - ref).abs().max()) <= float(ref.abs().max()) * 2 ** -7
    w = (torch.randn(N, K, device=cuda) * K ** -0.5).to(torch.bfloat16)
    assert C.gemm_stream_rows(M, N, K, K, N, False) > 0
    out = C.gemm_nt_norm(_rows(y), w, stats, ws)
    c0, s0 = C.gemm_nt(_rows(a), w, stats)
    torch.cuda.synchronize()
    assert out and torch.equal(out[0], c0)
    if stats:
        assert torch.equal(out[1], s0)
    fp = _rows(a).float() @ w.float().t()
    assert float((out[0].float() - fp).norm() / fp.norm()) < 5e-3


def test_stream_normalise_not_served(cuda, C):
    y, ws, _ = _bn_input(cuda, C, 1024, 64, 1)
    w = torch.randn(256, 64, device=cuda).to(torch.bfloat16)
    assert C.gemm_nt_norm(_rows(y), w, True, ws) == []  # too few rows for the persistent grid
    y2, ws2, _ = _bn_input(cuda, C, 100000, 256, 2)
    assert C.gemm_nt_norm(_rows(y2), torch.randn(512, 256, device=cuda).to(torch.bfloat16), True, ws2) == []  # K 256


@pytest.mark.parametrize("M,ci,co", [(65536, 64, 256), (70001, 64, 256), (50001, 128, 512), (40003, 256, 512)])
def test_dual_normalise_x_is_bitwise(cuda, C, M, ci, co):
    M16 = M // 16 * 16
    y, ws, _ = _bn_input(cuda, C, M16, ci, M)
    a = C.bn_apply_ws(y, ws, True)
    g = torch.Generator().manual_seed(M + 1)
    dy = torch.randn(M16, co, generator=g).to(cuda, torch.bfloat16)
    w = (torch.randn(co, ci, generator=g) * co ** -0.5).to(cuda, torch.bfloat16)
    assert C.conv1x1_dual_blocks(M16, ci, co) > 0
    dx, dw = C.conv1x1_dual(dy, _rows(y), w, torch.float32, None, None, None, ws)
    dx0, dw0 = C.conv1x1_dual(dy, _rows(a), w, torch.float32)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx0) and torch.equal(dw, dw0)
    ref = dy.double().t() @ _rows(a).double()
    assert float((dw.double() - ref).norm() / ref.norm()) < 1e-5


@pytest.mark.parametrize("M", [65536, 100000])
def test_dual_bn_apply_with_normalised_x_is_bitwise(cuda, C, M):
    ci, co = 64, 256
    y, ws, _ = _bn_input(cuda, C, M, ci, M + 7)
    a = C.bn_apply_ws(y, ws, True)
    g = torch.Generator().manual_seed(M)
    dout = torch.randn(M, co, generator=g).to(cuda, torch.bfloat16)
    ybn = (torch.randn(M, co, generator=g) * 2 + 0.5).to(cuda, torch.bfloat16)
    w = (torch.randn(co, ci, generator=g) * co ** -0.5).to(cuda, torch.bfloat16)
    mask = torch.randint(0, 256, ((M * co + 7) // 8,), generator=g, dtype=torch.uint8).to(cuda)
    ws3 = torch.zeros(7 * co, device=cuda)
    ws3[:co] = ybn.float().mean(0)
    ws3[co:2 * co] = (ybn.float().var(0, unbiased=False) + 1e-5).rsqrt()
    gamma3 = (torch.rand(co, generator=g) + 0.5).to(cuda)
    C.bn_act_bwd(dout, None, mask, ybn, ws3, gamma3, 2, False, None, False)  # finalize k1 / m1 / k2 into ws3
    assert C.conv1x1_dual_bn_ok(M, ci, co)
    dx, dw = C.conv1x1_dual(dout, _rows(y), w, torch.float32, ybn, ws3, mask, ws)
    dx0, dw0 = C.conv1x1_dual(dout, _rows(a), w, torch.float32, ybn, ws3, mask)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx0) and torch.equal(dw, dw0)


def _resnet_step(cuda, lazy, batch=24):
    from distributed_learning_amd.models import resnet50
    from distributed_learning_amd.ops import bn_act
    from distributed_learning_amd.ops import conv as nconv

    torch.manual_seed(0)
    from distributed_learning_amd.ops import nn as dnn

    m = resnet50(10).to(cuda).to(memory_format=CL)
    dnn.bf16_weights(m)
    x = torch.randn(batch, 3, 224, 224, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    old = nconv.LAZY_BN_ACT
    nconv.LAZY_BN_ACT = lazy
    before = nconv.CALLS["1x1_norm"]
    try:
        loss = m(x).float().square().mean()
        loss.backward()
        bn_act.flush_bn_counters()
    finally:
        nconv.LAZY_BN_ACT = old
    grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    bufs = {n: b.clone() for n, b in m.named_buffers()}
    return float(loss), grads, bufs, nconv.CALLS["1x1_norm"] - before


def test_resnet_lazy_bn2_is_bitwise(cuda):
    """Stage-1/2 bottlenecks (7 conv3s) normalise relu(BN2) on load; everything else is unchanged, and so are
    the loss, every gradient and every running statistic, bit for bit."""
    from distributed_learning_amd.ops import nn as dnn

    dnn.set_backend("native")
    dnn.set_native_conv(True)
    try:
        l1, g1, b1, n1 = _resnet_step(cuda, True)
        l0, g0, b0, n0 = _resnet_step(cuda, False)
    finally:
        dnn.set_native_conv(False)
        dnn.set_backend("torch")
    assert n1 == 7 and n0 == 0
    assert l1 == l0
    bad = [n for n in g0 if not torch.equal(g1[n], g0[n])]
    assert not bad, bad[:5]
    badb = [n for n in b0 if not torch.equal(b1[n], b0[n])]
    assert not badb, badb[:5]


def test_lazy_conv_fallback_materialises(cuda):
    """A shape neither kernel serves (few rows): _BNActConv1x1 materialises the activation with bn_apply's
    arithmetic and runs the tile GEMMs -- the same bits as the BN+ReLU followed by the 1x1 conv."""
    import torch.nn as nn

    from distributed_learning_amd.ops import bn_act
    from distributed_learning_amd.ops import conv as nconv
    from distributed_learning_amd.ops import nn as dnn

    torch.manual_seed(0)
    conv = nn.Conv2d(64, 256, 1, bias=False).to(cuda).to(memory_format=CL)
    conv.weight.data = conv.weight.data.to(torch.bfloat16)
    y0 = torch.randn(2, 64, 14, 14, device=cuda).to(torch.bfloat16).contiguous(memory_format=CL)
    gy = torch.randn(2, 256, 14, 14, device=cuda).contiguous(memory_format=CL)

    def run(lazy):
        bn = nn.BatchNorm2d(64).to(cuda)
        torch.manual_seed(1)
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.uniform_(-0.3, 0.3)
        conv.weight.grad = None
        y = y0.clone().requires_grad_(True)
        st = torch.stack([y.float().sum((0, 2, 3)), y.float().square().sum((0, 2, 3))], 1).unsqueeze(0).contiguous()
        if lazy:
            out, _ = nconv.conv1x1(nconv.LazyBNAct(y, bn, st), conv)
        else:
            out, _ = nconv.conv1x1(bn_act.fused_bn_act(y, bn, True, None, st), conv)
        (out.float() * gy).sum().backward()
        bn_act.flush_bn_counters()
        return out, y.grad, conv.weight.grad, bn.weight.grad, bn.bias.grad, bn.running_mean, bn.running_var

    dnn.set_backend("native")
    try:
        r1, r0 = run(True), run(False)
    finally:
        dnn.set_backend("torch")
    for a, b in zip(r1, r0):
        assert torch.equal(a, b)
