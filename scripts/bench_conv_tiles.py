#!/usr/bin/env python3
"""Per-tile timing of the 3x3 implicit-GEMM convolutions at the headline batch (ResNet-50, bs1280).

For every stride-1 3x3 shape of the step (stage 1: halo-tiled 64-channel kernels under ``auto``; stages
2-4: the tile kernels) the forward with the BN-statistics epilogue and the data gradient are timed with
``auto`` and with every tile configuration the shape admits, plus the weight gradient; medians of 15, one
process, interleaved by shape. Prints one JSON line per shape with ms and achieved TFLOP/s.

usage: python scripts/bench_conv_tiles.py [--batch 1280]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TILES = {"auto": 0, "128x128": 1, "128x64": 2, "256x128": 4, "256x128w4": 5, "128x256w4": 6, "256x256": 8,
         "512x128": 9}


def timeit(fn, iters=15):
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
    a = ap.parse_args()
    import torch

    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    dev = torch.device("cuda:0")
    CL = torch.channels_last
    for C_, H in ((64, 56), (128, 28), (256, 14), (512, 7)):
        N = a.batch
        x = torch.randn(N, C_, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(C_, C_, 3, 3, device=dev) * (2.0 / (9 * C_)) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=CL)
        dy = torch.randn(N, C_, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        gflop = 2 * N * H * H * C_ * C_ * 9 / 1e9
        r = {"C": C_, "H": H, "M": N * H * H, "gflop": round(gflop, 1)}
        for name, t in TILES.items():
            if t == 8 and C_ % 256:
                continue
            if t == 9 and C_ != 128:
                continue
            if t == 2 and C_ > 64:
                continue
            try:
                r[f"fwd_{name}"] = round(timeit(lambda: C.conv3x3_fwd(x, w, 1, True, t)), 4)
            except RuntimeError as e:
                r[f"fwd_{name}"] = str(e)[:50]
            try:
                r[f"dgrad_{name}"] = round(timeit(lambda: C.conv3x3_dgrad(dy, w, None, t)), 4)
            except RuntimeError as e:
                r[f"dgrad_{name}"] = str(e)[:50]
        r["wgrad"] = round(timeit(lambda: C.conv3x3_wgrad(dy, x, 1, torch.float32)), 4)
        for k in ("fwd_auto", "dgrad_auto", "wgrad"):
            if isinstance(r.get(k), float):
                r[k + "_tflops"] = round(gflop / r[k], 1)
        print(json.dumps(r), flush=True)
        del x, w, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
