"""fp32 Inception block with its three 1x1 convs on x as one GEMM (ops/inception_f32.py) vs float64 PyTorch.

Output, input gradient, every parameter gradient (the concatenated conv weights and BN affine parameters split
back to their modules through autograd) and the running statistics (the modules' buffers are views of one
concatenated buffer that the fused BN kernel updates) of one training-mode forward/backward, against the same
block in float64 on the stock torch path.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("cfg", [(192, 64, 96, 128, 16, 32, 32, 28), (480, 192, 96, 208, 16, 48, 64, 14),
                                 (832, 384, 192, 384, 48, 128, 128, 7)])
def test_inception_f32_matches_float64(cuda, cfg):
    from distributed_learning_amd.models.googlenet import Inception
    from distributed_learning_amd.ops import bn_act
    from distributed_learning_amd.ops import inception_f32
    from distributed_learning_amd.ops import nn as dnn

    cin, c1, c2r, c2, c3r, c3, cp, hw = cfg
    torch.manual_seed(sum(cfg))
    ref = Inception(cin, c1, c2r, c2, c3r, c3, cp).to(cuda)
    for m in ref.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    nat = copy.deepcopy(ref).to(memory_format=torch.channels_last)
    ref = ref.double()
    x = torch.randn(4, cin, hw, hw, device=cuda)
    xn = x.clone().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    xr = x.double().requires_grad_(True)
    dnn.set_backend("native")
    dnn.set_native_conv_f32(True)
    try:
        assert inception_f32.supported(nat, xn)
        yn = nat(xn)
        bn_act.flush_bn_counters()
    finally:
        dnn.set_backend("torch")
        dnn.set_native_conv_f32(False)
    yr = ref(xr)
    dy = torch.randn(yr.shape, device=cuda)
    yn.backward(dy.contiguous(memory_format=torch.channels_last))
    yr.backward(dy.double())
    torch.cuda.synchronize()
    assert _rel(yn, yr) < 1e-5
    assert _rel(xn.grad, xr.grad) < 1e-4
    for (n, pn), (_, pr) in zip(nat.named_parameters(), ref.named_parameters()):
        assert pn.grad is not None, n
        assert _rel(pn.grad, pr.grad) < 1e-4, n
    for (n, bn_n), (_, bn_r) in zip(nat.named_buffers(), ref.named_buffers()):
        if "running" in n:
            assert _rel(bn_n, bn_r) < 1e-5, n
        elif "num_batches" in n:
            assert int(bn_n) == int(bn_r) == 1, n
