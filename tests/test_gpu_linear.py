"""Native fully connected layer (ops/linear.py: MFMA GEMMs, bias as a stride-0 epilogue addend)
vs an fp32 PyTorch reference (gpu)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("B,fin,fout,bias", [(2, 2048, 1000, True), (512, 2048, 1000, True), (7, 1024, 1000, True),
                                             (64, 1024, 1024, False), (130, 128, 16, True),
                                             (128, 2048, 1024, True), (128, 1024, 1000, True)])
def test_native_linear_matches_fp32(cuda, B, fin, fout, bias):
    from distributed_learning_amd.ops.linear import linear, supported

    torch.manual_seed(0)
    fc = nn.Linear(fin, fout, bias=bias).to(cuda)
    with torch.no_grad():
        if bias:
            fc.bias.uniform_(-1, 1)
    fc_bf = nn.Linear(fin, fout, bias=bias).to(cuda)
    fc_bf.load_state_dict(fc.state_dict())
    fc_bf.to(torch.bfloat16)
    x = torch.randn(B, fin, device=cuda).to(torch.bfloat16)
    assert supported(x, fc_bf)
    xn = x.clone().requires_grad_(True)
    y = linear(xn, fc_bf)
    assert y.dtype == torch.bfloat16 and y.shape == (B, fout)
    xr = x.float().requires_grad_(True)
    w_r = fc_bf.weight.detach().float().requires_grad_(True)
    b_r = fc_bf.bias.detach().float().requires_grad_(True) if bias else None
    yr = F.linear(xr, w_r, b_r)
    assert _rel(y, yr) < 1e-2
    g = torch.randn(B, fout, device=cuda).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    assert _rel(xn.grad, xr.grad) < 1e-2
    assert fc_bf.weight.grad.dtype == torch.bfloat16 and _rel(fc_bf.weight.grad, w_r.grad) < 1e-2
    if bias:
        assert fc_bf.bias.grad.shape == (fout,) and _rel(fc_bf.bias.grad, b_r.grad) < 1e-2
