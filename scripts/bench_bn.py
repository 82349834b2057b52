#!/usr/bin/env python3
"""Micro-benchmark of the fused BatchNorm passes at the headline batch's stage-1 shapes (ResNet-50, bs1280).

Cases (M = 1280 * 56 * 56 rows): the block-output BN (C = 256, identity residual, ReLU, 1-bit mask) in
training mode with GEMM-epilogue statistics, the same apply in eval mode (no statistics, no mask: the mask's
cost), bn1/bn2 (C = 64, ReLU recomputed), and the backward reduce + apply of both. Each op runs ``--iters``
times, so ``rocprofv3 --kernel-trace --stats`` of this script gives per-kernel times; one JSON line with
the median ms of each op and its TB/s of compulsory bytes.

usage: python scripts/bench_bn.py [--batch 1280] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    import torch

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--batch", type=int, default=1280)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    dev = torch.device("cuda:0")
    CL = torch.channels_last
    out = {"batch": a.batch}
    for ch, res in ((256, True), (64, False)):
        x = (torch.randn(a.batch, ch, 56, 56, device=dev) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
        r = torch.randn_like(x) if res else None
        g = torch.rand(ch, device=dev) + 0.5
        b = torch.randn(ch, device=dev) * 0.1
        rm, rv = torch.zeros(ch, device=dev), torch.ones(ch, device=dev)
        M = x.numel() // ch
        T = x.numel() * 2 / 1e9  # GB of one bf16 activation
        # GEMM-epilogue style statistics partials: one row per 128-row tile
        xr = x.permute(0, 2, 3, 1).reshape(M, ch).float()
        st = torch.stack([xr.view(-1, 128, ch).sum(1), xr.view(-1, 128, ch).square().sum(1)], 2).contiguous()
        del xr
        key = f"c{ch}"
        fwd = lambda: C.bn_act_fwd(x, r, g, b, rm, rv, True, 0.1, 1e-5, True, st, None, 0)  # noqa: E731
        out[key + "_fwd_train_ms"] = timeit(fwd, a.iters)
        out[key + "_fwd_eval_ms"] = timeit(lambda: C.bn_act_fwd(x, r, g, b, rm, rv, False, 0.1, 1e-5, True, None,
                                                                 None, 0), a.iters)
        y, ws, mask = fwd()
        dy = torch.randn_like(x)
        mode = 2 if res else 1
        out[key + "_bwd_ms"] = timeit(lambda: C.bn_act_bwd(dy, None, mask if res else None, x, ws, g, mode,
                                                            res, None), a.iters)
        nread_fwd = 2 if res else 1
        out[key + "_fwd_train_TBps"] = round((nread_fwd + 1) * T / out[key + "_fwd_train_ms"], 2)
        # backward: reduce reads dy + x, apply reads dy + x and writes dx (+ dres)
        out[key + "_bwd_TBps"] = round((5 + (1 if res else 0)) * T / out[key + "_bwd_ms"], 2)
        del x, r, y, dy, mask, st
        torch.cuda.empty_cache()
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
