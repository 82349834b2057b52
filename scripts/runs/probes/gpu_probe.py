"""First GPU probe: native kernel sanity + stock-PyTorch ResNet-50 baseline throughput."""
import sys, time, json
import torch
sys.path.insert(0, ".")
from distributed_learning_amd.ops import _ext
from distributed_learning_amd.models import resnet50

C = _ext.require()
dev = torch.device("cuda:0")
print(torch.cuda.get_device_name(0), torch.version.hip, flush=True)

# --- kernel sanity ---
ps = [torch.randn(n, device=dev) for n in (5000, 4096, 17, 123457)]
gs = [torch.randn_like(p) for p in ps]
ms = [torch.randn_like(p) for p in ps]
ref_p = [p.clone() for p in ps]; ref_m = [m.clone() for m in ms]
t = C.SgdTable(ps, gs, ms, [])
t.step(0.1, 0.9, 0.0, 1e-4, False, 0.5, False)
for p, g, m, rp, rm in zip(ps, gs, ms, ref_p, ref_m):
    d = g * 0.5 + 1e-4 * rp
    rm.mul_(0.9).add_(d)
    rp.add_(rm, alpha=-0.1)
    print("sgd maxerr", (p - rp).abs().max().item(), (m - rm).abs().max().item())
flat = torch.zeros(sum(g.numel() for g in gs) + 64 * 4, device=dev)
offs, o = [], 0
for g in gs:
    offs.append(o); o += (g.numel() + 63) // 64 * 64
pt = C.PackTable(gs, offs)
pt.pack(flat, 2.0)
print("pack err", max((flat[off:off + g.numel()] - 2 * g).abs().max().item() for g, off in zip(gs, offs)))
x = torch.randn(1000003, device=dev); y = torch.randn_like(x); z = x.clone()
C.reduce_sum_(z, [y], True, 0.5)
print("reduce err", (z - (x + y) * 0.5).abs().max().item())
u = torch.empty(10**6, device=dev, dtype=torch.bfloat16); C.uniform_(u, 1, 0, 0.0, 1.0)
print("uniform mean", u.float().mean().item(), u.float().min().item(), u.float().max().item())
lg = torch.randn(256, 1000, device=dev, dtype=torch.bfloat16); tg = torch.randint(0, 1000, (256,), device=dev)
loss, ws = C.xent_fwd(lg, tg)
ref = torch.nn.functional.cross_entropy(lg.float(), tg)
print("xent", loss[0].item(), ref.item())
torch.cuda.synchronize()

# --- baseline ResNet-50 stock pytorch ---
torch.backends.cudnn.benchmark = True
res = {}
for bs in (128, 256):
    model = resnet50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9)
    data = torch.rand(bs, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    target = torch.randint(0, 1000, (bs,), device=dev)
    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(data)
            loss = torch.nn.functional.cross_entropy(out, target)
        loss.backward()
        opt.step()
    for _ in range(8):
        step()
    torch.cuda.synchronize()
    t0 = time.time()
    n = 20
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.time() - t0) / n
    res[bs] = (dt * 1000, bs / dt)
    print(f"bs={bs} {dt*1000:.1f} ms/step {bs/dt:.1f} img/s", flush=True)
    del model, opt
print(json.dumps(res))
