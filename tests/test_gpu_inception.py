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
