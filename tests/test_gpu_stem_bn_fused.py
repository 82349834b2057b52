"""Stem weight gradient with the BN+ReLU+max-pool backward apply fused (csrc/kernels/stem.hip
stem_wgrad_bn_kernel; ops/conv.py StemBNLink) vs the unfused pair and fp32 PyTorch (gpu)."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _stem_bn_case(cuda, n, h, w, seed=0):
    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops.conv import stem_pack_weight

    C = _ext.require()
    g = torch.Generator(device=cuda).manual_seed(seed)  # device-side draws: the bench-batch case is 2 GB of dY
    x = torch.randn(n, 3, h, w, generator=g, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(64, 3, 7, 7, generator=g, device=cuda) * 0.1).to(torch.bfloat16)
    y, stats, xs = C.stem_fwd(x, stem_pack_weight(wt), True)
    gamma = torch.rand(64, generator=g, device=cuda) + 0.5
    beta = torch.rand(64, generator=g, device=cuda) - 0.5
    yp, ws, pos = C.bn_relu_maxpool_fwd(y, gamma, beta, None, None, 0.1, 1e-5, 3, 2, 1, stats, False)
    dyp = torch.randn(yp.shape, generator=g, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    return C, x, wt, y, xs, gamma, ws, pos, dyp


@pytest.mark.parametrize("shape", [(4, 224, 224), (3, 100, 100), (2, 64, 96), (1, 8, 8),
                                   (1280, 224, 224)])  # bench.py's batch: 512 splits, 16 M conv-output pixels
def test_stem_wgrad_bn_matches_unfused_and_torch(cuda, shape):
    from distributed_learning_amd.ops.conv import stem_unpack_grad

    C, x, wt, y, xs, gamma, ws, pos, dyp = _stem_bn_case(cuda, *shape)
    n, _, h, w = x.shape
    # unfused: the quad apply writes the conv output's gradient, stem_wgrad reads it
    dy, dg, db = C.bn_relu_maxpool_bwd(dyp, pos, y, ws.clone(), gamma, 3, 2, 1)
    ref_pk = C.stem_wgrad(dy, xs, h, w, torch.float32)
    # fused: reduce + finalize only, then the weight gradient computes dY itself
    ws2 = ws.clone()
    none, dg2, db2 = C.bn_relu_maxpool_bwd(dyp, pos, y, ws2, gamma, 3, 2, 1, want_dx=False)
    assert none is None
    torch.testing.assert_close(dg2, dg, rtol=0, atol=0)
    torch.testing.assert_close(db2, db, rtol=0, atol=0)
    got_pk = C.stem_wgrad_bn(dyp, pos, y, ws2, xs, h, w, torch.float32)
    # same bf16 dY values, different summation order only
    rel = ((got_pk - ref_pk).norm() / ref_pk.norm().clamp_min(1e-30)).item()
    assert rel < 1e-5, rel
    # against fp32 PyTorch of the same op: the weight gradient of the 7x7 / s2 conv from that dY
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), wt.float(), None, [2, 2], [3, 3], [1, 1], False,
                                              [0, 0], 1, [False, True, False])[1]
    got = stem_unpack_grad(got_pk)
    assert ((got - ref).norm() / ref.norm()).item() < 1e-4
    assert got_pk.reshape(64, 16, 16)[:, :, 12:].abs().max().item() == 0.0
    bf = C.stem_wgrad_bn(dyp, pos, y, ws2, xs, h, w, torch.bfloat16)
    assert bf.dtype == torch.bfloat16
    torch.testing.assert_close(bf.float(), got_pk, rtol=1e-2, atol=1e-2 * got_pk.abs().max().item())


def test_want_dx_false_refused_outside_quad_form(cuda):
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    y = torch.randn(2, 64, 30, 30, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gamma, beta = torch.ones(64, device=cuda), torch.zeros(64, device=cuda)
    yp, ws, pos = C.bn_relu_maxpool_fwd(y, gamma, beta, None, None, 0.1, 1e-5, 3, 2, 0, None, False)  # pad 0
    dyp = torch.randn(yp.shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError, match="quad form"):
        C.bn_relu_maxpool_bwd(dyp, pos, y, ws, gamma, 3, 2, 0, want_dx=False)


def _model_step(cuda, fused: bool, observe: bool = False, second: bool = False):
    from distributed_learning_amd.ops import conv as nconv
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.bn_act import fused_bn_relu_maxpool

    torch.manual_seed(0)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(cuda).to(memory_format=torch.channels_last)
    conv.weight.data = conv.weight.data.to(torch.bfloat16)
    bn = nn.BatchNorm2d(64).to(cuda)
    pool = nn.MaxPool2d(3, 2, 1)
    x = torch.randn(8, 3, 128, 128, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    before = nconv.CALLS["stem_bn"]
    old = nconv.STEM_BN
    nconv.STEM_BN = fused
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    seen = []
    try:
        extra = None
        if observe:  # a hook on the conv output must see the real gradient, so the fusion stands down
            y, stats = nconv.stem_conv(x, conv, want_stats=True)
            y.register_hook(lambda g: seen.append(g.float().norm().item()))
            out = fused_bn_relu_maxpool(y, bn, pool, stats)
        elif second:  # the conv output also feeds another consumer: its gradient adds to the parked one
            y, stats = nconv.stem_conv(x, conv, want_stats=True)
            out = fused_bn_relu_maxpool(y, bn, pool, stats)
            extra = y.float().mul(torch.linspace(-0.5, 0.5, y.numel(), device=cuda).reshape(y.shape)).sum()
        else:
            out = dnn.conv_bn_act_maxpool(x, conv, bn, pool)
        loss = out.float().mul(torch.linspace(-1, 1, out.numel(), device=cuda).reshape(out.shape)).sum()
        (loss if extra is None else loss + extra).backward()
        torch.cuda.synchronize()
    finally:
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
        nconv.STEM_BN = old
    return conv.weight.grad.float().clone(), bn.weight.grad.clone(), nconv.CALLS["stem_bn"] - before, seen


def test_stem_bn_fused_model_path_matches_unfused(cuda):
    gw_f, gg_f, used_f, _ = _model_step(cuda, True)
    gw_u, gg_u, used_u, _ = _model_step(cuda, False)
    assert used_f == 1 and used_u == 0
    torch.testing.assert_close(gg_f, gg_u, rtol=0, atol=0)
    assert ((gw_f - gw_u).norm() / gw_u.norm()).item() < 1e-4


def test_stem_bn_fusion_stands_down_for_observed_output(cuda):
    gw_o, _, used_o, seen = _model_step(cuda, True, observe=True)
    gw_u, _, _, _ = _model_step(cuda, False)
    assert used_o == 0 and len(seen) == 1 and seen[0] > 0
    assert ((gw_o - gw_u).norm() / gw_u.norm()).item() < 1e-4


def test_stem_bn_fusion_with_a_second_consumer_of_the_conv_output(cuda):
    """advisor r5: the stem conv output feeds the fused BN+ReLU+max-pool AND a second consumer. The parked gradient
    is materialised (StemBNLink.materialise re-runs the quad apply on the already finalized workspace) and added to
    the other consumer's gradient: dW and dgamma must match the unfused path."""
    gw_f, gg_f, used_f, _ = _model_step(cuda, True, second=True)
    gw_u, gg_u, used_u, _ = _model_step(cuda, False, second=True)
    assert used_u == 0
    torch.testing.assert_close(gg_f, gg_u, rtol=0, atol=0)
    assert ((gw_f - gw_u).norm() / gw_u.norm()).item() < 1e-4
