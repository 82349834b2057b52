"""Native HIP kernels vs plain PyTorch fp32 references (run on an MI355X: ``pytest -m gpu``)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from distributed_learning_amd.ops import _ext

    return _ext.require()


@pytest.mark.parametrize("grad_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kw", [dict(momentum=0.5), dict(momentum=0.9, nesterov=True, weight_decay=1e-4),
                                dict(momentum=0.9, dampening=0.2), dict(momentum=0.0, weight_decay=0.01)])
def test_sgd_table_vs_torch(cuda, grad_dtype, kw):
    C = _C()
    torch.manual_seed(0)
    shapes = [(5000,), (4096,), (17,), (123457,), (64, 3, 7, 7)]
    ps = [torch.randn(s, device=cuda) for s in shapes]
    ps[-1] = ps[-1].contiguous(memory_format=torch.channels_last)
    refp = [p.clone() for p in ps]
    mom = kw.get("momentum", 0.0)
    ms = [torch.zeros_like(p) for p in ps] if mom else []
    refm = [torch.zeros_like(p) for p in ps]
    tab = C.SgdTable(ps, [torch.empty_like(p, dtype=grad_dtype) for p in ps], ms, [])
    del tab
    for step in range(3):
        gs = [torch.randn_like(p).to(grad_dtype) for p in ps]
        tab = C.SgdTable(ps, gs, ms, [])
        tab.step(0.1, mom, kw.get("dampening", 0.0), kw.get("weight_decay", 0.0), kw.get("nesterov", False), 0.5,
                 step == 0)
        for i, (p, g) in enumerate(zip(refp, gs)):
            d = g.float() * 0.5 + kw.get("weight_decay", 0.0) * p
            if mom:
                refm[i] = d.clone() if step == 0 else refm[i] * mom + (1 - kw.get("dampening", 0.0)) * d
                d = d + mom * refm[i] if kw.get("nesterov") else refm[i]
            p.add_(d, alpha=-0.1)
    for p, r in zip(ps, refp):
        torch.testing.assert_close(p, r, rtol=1e-5, atol=1e-6)


def test_fused_sgd_optimizer_gpu(cuda):
    from distributed_learning_amd.ops.optim import FusedSGD

    torch.manual_seed(0)
    ps = [torch.randn(n, device=cuda, requires_grad=True) for n in (10, 4096 * 3 + 5, 77)]
    qs = [p.detach().clone().requires_grad_(True) for p in ps]
    a, b = FusedSGD(ps, lr=0.05, momentum=0.9), torch.optim.SGD(qs, lr=0.05, momentum=0.9)
    for _ in range(4):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad, q.grad = g.clone(), g.clone()
        a.step()
        b.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("flat_dtype", [torch.float32, torch.bfloat16])
def test_pack_unpack(cuda, flat_dtype):
    C = _C()
    torch.manual_seed(1)
    gs = [torch.randn(n, device=cuda) for n in (1, 63, 4096, 10000, 5)]
    gs.append(torch.randn(8, 16, 3, 3, device=cuda).contiguous(memory_format=torch.channels_last))
    offs, o = [], 0
    for g in gs:
        offs.append(o)
        o += (g.numel() + 63) // 64 * 64
    flat = torch.full((o,), 7.0, device=cuda, dtype=flat_dtype)
    t = C.PackTable(gs, offs)
    t.pack(flat, 2.0)
    for g, off in zip(gs, offs):
        raw = g.permute(0, 2, 3, 1).reshape(-1) if g.dim() == 4 else g.reshape(-1)
        torch.testing.assert_close(flat[off:off + g.numel()].float(), (raw * 2).to(flat_dtype).float())
    orig = [g.clone() for g in gs]
    t.unpack(flat, 0.5)
    for g, og in zip(gs, orig):
        tol = dict(rtol=1e-2, atol=1e-2) if flat_dtype == torch.bfloat16 else dict(rtol=0, atol=0)
        torch.testing.assert_close(g, og, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nsrc", [0, 1, 3, 8])
def test_reduce_sum(cuda, dtype, nsrc):
    C = _C()
    for n in (1, 7, 1000, 1_000_003):
        dst = torch.randn(n, device=cuda).to(dtype)
        srcs = [torch.randn(n, device=cuda).to(dtype) for _ in range(nsrc)]
        ref = (dst.float() + sum((s.float() for s in srcs), torch.zeros(n, device=cuda))) * 0.25
        C.reduce_sum_(dst, srcs, True, 0.25)
        tol = dict(rtol=1e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(dst.float(), ref, **tol)
    # unaligned view (scalar path)
    base = torch.randn(1001, device=cuda)
    v, s = base[1:], torch.randn(1000, device=cuda)
    ref = (v + s).clone()
    C.reduce_sum_(v, [s], True, 1.0)
    torch.testing.assert_close(v, ref)


def test_philox_synthetic(cuda):
    C = _C()
    a = torch.empty(1 << 20, device=cuda)
    b = torch.empty_like(a)
    C.uniform_(a, 42, 0, 0.0, 1.0)
    C.uniform_(b, 42, 0, 0.0, 1.0)
    assert torch.equal(a, b)  # counter-based: reproducible
    assert 0.0 <= float(a.min()) and float(a.max()) < 1.0
    assert abs(float(a.mean()) - 0.5) < 2e-3 and abs(float(a.var()) - 1 / 12) < 2e-3
    C.uniform_(b, 43, 0, 0.0, 1.0)
    assert not torch.equal(a, b)
    y = torch.empty(100_000, device=cuda, dtype=torch.long)
    C.randint_(y, 1000, 7, 0)
    assert int(y.min()) >= 0 and int(y.max()) < 1000
    assert abs(float(y.float().mean()) - 499.5) < 10
    from distributed_learning_amd.data import SyntheticBatches

    x, t = SyntheticBatches(8, (3, 224, 224), 1000, cuda, channels_last=True).next()
    assert x.is_contiguous(memory_format=torch.channels_last) and x.shape == (8, 3, 224, 224)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,Cn", [(256, 1000), (3, 10), (129, 4097)])
def test_xent_vs_torch(cuda, dtype, B, Cn):
    from distributed_learning_amd.ops.loss import cross_entropy

    torch.manual_seed(0)
    x = (torch.randn(B, Cn, device=cuda) * 3).to(dtype).requires_grad_(True)
    y = torch.randint(0, Cn, (B,), device=cuda)
    if B > 3:
        y[1] = -100  # ignored row
    loss = cross_entropy(x, y)
    loss.backward()
    xr = x.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(xr, y, ignore_index=-100)
    ref.backward()
    torch.testing.assert_close(loss.float(), ref, rtol=1e-5, atol=1e-5)
    tol = dict(rtol=2e-2, atol=1e-4) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
