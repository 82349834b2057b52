"""Halo vs implicit-GEMM 3x3 weight gradient at the ResNet-50 stage-1 shape (64 -> 64, 56x56), interleaved.

    python scripts/bench_halo_wgrad.py [--batch 1024]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_learning_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=15):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    C = _ext.require()
    dev = torch.device("cuda", 0)
    x = torch.randn(a.batch, 64, 56, 56, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(a.batch, 64, 56, 56, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    flop = 2.0 * a.batch * 56 * 56 * 64 * 64 * 9
    r = {"batch": a.batch}
    for rep in range(2):
        for mode in (1, 0):
            C.set_halo_wgrad(mode)
            ms = timeit(lambda: C.conv3x3_wgrad(dy, x, 1, torch.float32))
            key = "halo" if mode else "implicit"
            r[f"{key}_ms_{rep}"] = round(ms, 4)
            r[f"{key}_TFs_{rep}"] = round(flop / ms / 1e9, 1)
    C.set_halo_wgrad(-1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
