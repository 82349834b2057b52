#!/usr/bin/env python3
"""Op-by-op fp32 parity of the native kernels against stock PyTorch (the reference-precision path).

Each op runs native (channels_last fp32) and stock (torch / MIOpen, fp32) on the same input and output
gradient; prints one JSON line per op with the relative L2 error of the output, the input gradient and the
parameter gradients. Used to localise a whole-model fp32 gradient difference (tests/test_gpu_fp32_path.py).

usage: python scripts/fp32_op_parity.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def main() -> None:
    import torch
    import torch.nn as nn
    import torch.nn.functional as F

    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.bn_act import fused_bn_act
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.pool import global_avg_pool, max_pool2d

    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cudnn.deterministic = True
    dev = torch.device("cuda:0")
    CL = torch.channels_last
    dnn.set_backend("native")
    torch.manual_seed(0)

    def run(name, fn_nat, fn_ref, x, params=()):
        xn = x.detach().clone().contiguous(memory_format=CL).requires_grad_(True)
        xr = x.detach().clone().requires_grad_(True)
        yn = fn_nat(xn)
        yr = fn_ref(xr)
        g = torch.randn_like(yr)
        for p in params:
            p.grad = None
        yn.backward(g.contiguous(memory_format=CL) if g.dim() == 4 else g)
        gn = [p.grad.clone() for p in params]
        for p in params:
            p.grad = None
        yr.backward(g)
        gr = [p.grad.clone() for p in params]
        out = {"op": name, "out": rel(yn, yr), "dx": rel(xn.grad, xr.grad)}
        out["dparams"] = [rel(a, b) for a, b in zip(gn, gr)]
        print(json.dumps(out), flush=True)

    x = torch.randn(16, 64, 28, 28, device=dev) * 2 + 0.5
    bn = nn.BatchNorm2d(64, eps=1e-3).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn_ref = nn.BatchNorm2d(64, eps=1e-3).to(dev)
    bn_ref.load_state_dict(bn.state_dict())
    params = [bn.weight, bn.bias]
    xn = x.detach().clone().contiguous(memory_format=CL).requires_grad_(True)
    xr = x.detach().clone().requires_grad_(True)
    yn = fused_bn_act(xn, bn, True)
    yr = F.relu(bn_ref(xr))
    g = torch.randn_like(yr)
    yn.backward(g.contiguous(memory_format=CL))
    yr.backward(g)
    print(json.dumps({"op": "bn_relu C64", "out": rel(yn, yr), "dx": rel(xn.grad, xr.grad),
                      "dgamma": rel(bn.weight.grad, bn_ref.weight.grad), "dbeta": rel(bn.bias.grad, bn_ref.bias.grad)}),
          flush=True)
    xp = F.relu(torch.randn(16, 64, 28, 28, device=dev))
    run("maxpool 3/2/0 ceil", lambda t: max_pool2d(t, 3, 2, 0, 1, True), lambda t: F.max_pool2d(t, 3, 2, 0, 1, True), xp)
    run("maxpool 3/1/1 ceil", lambda t: max_pool2d(t, 3, 1, 1, 1, True), lambda t: F.max_pool2d(t, 3, 1, 1, 1, True), xp)
    run("maxpool 3/2/1", lambda t: max_pool2d(t, 3, 2, 1), lambda t: F.max_pool2d(t, 3, 2, 1), xp)
    run("global avg pool", lambda t: global_avg_pool(t), lambda t: torch.flatten(F.adaptive_avg_pool2d(t, 1), 1),
        torch.randn(16, 64, 7, 7, device=dev))
    logits = torch.randn(16, 100, device=dev)
    y = torch.randint(0, 100, (16,), device=dev)
    ln, lr = logits.clone().requires_grad_(True), logits.clone().requires_grad_(True)
    a, b = cross_entropy(ln, y), F.cross_entropy(lr, y)
    a.backward()
    b.backward()
    print(json.dumps({"op": "cross_entropy", "out": abs(float(a) - float(b)), "dx": rel(ln.grad, lr.grad)}), flush=True)


if __name__ == "__main__":
    main()
