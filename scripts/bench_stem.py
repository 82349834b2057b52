#!/usr/bin/env python3
"""Micro-benchmark of the ResNet stem at the headline batch: the native conv 7x7/s2 + BN + ReLU + max-pool
(ops/nn.py conv_bn_act_maxpool: fold, stem_fwd with the statistics epilogue, the fused BN+ReLU+pool forward,
the quad BN+pool backward, the stem weight gradient) run forward + backward ``--iters`` times, so a
``rocprofv3 --kernel-trace --stats`` of this script gives the stem's per-kernel times in isolation, and the
whole op's time per iteration (HIP events, median) is printed as one JSON line with the compulsory-bytes
roofline of each stage at the measured ~6 TB/s.

usage: python scripts/bench_stem.py [--batch 1280] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--batch", type=int, default=1280)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    import torch.nn as nn

    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops import nn as dnn

    _ext.require()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev).to(memory_format=torch.channels_last)
    conv.weight.data = conv.weight.data.to(torch.bfloat16)
    bn = nn.BatchNorm2d(64).to(dev)
    pool = nn.MaxPool2d(3, 2, 1)
    x = torch.rand(a.batch, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    g = None
    times = {"fwd": [], "bwd": []}
    for it in range(a.iters + 3):
        conv.weight.grad = None
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        y = dnn.conv_bn_act_maxpool(x, conv, bn, pool)
        e[1].record()
        if g is None:
            g = torch.randn_like(y)
        y.backward(g)
        e[2].record()
        torch.cuda.synchronize()
        if it >= 3:
            times["fwd"].append(e[0].elapsed_time(e[1]))
            times["bwd"].append(e[1].elapsed_time(e[2]))
    med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
    N = a.batch
    GB = 1e9
    xin, xs, yc, yp = N * 224 * 224 * 3 * 2, N * 112 * 112 * 16 * 2, N * 112 * 112 * 64 * 2, N * 56 * 56 * 64 * 2
    roof = {  # compulsory bytes per stage (one read of each operand, one write of each result) at 6 TB/s
        "fold": (xin + xs) / GB, "conv_fwd": (xs + yc) / GB, "bn_relu_pool_fwd": (yc + yp + N * 56 * 56 * 64) / GB,
        "pool_bn_bwd": (2 * yc + 2 * yp) / GB, "wgrad": (yc + xs) / GB}
    print(json.dumps({"batch": N, "fwd_ms": round(med["fwd"], 3), "bwd_ms": round(med["bwd"], 3),
                      "roofline_ms_at_6TBps": {k: round(v / 6.0, 3) for k, v in roof.items()},
                      "roofline_total_ms": round(sum(roof.values()) / 6.0, 3)}), flush=True)


if __name__ == "__main__":
    main()
