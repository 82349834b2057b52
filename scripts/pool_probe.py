"""Max-pool microbenchmark at GoogLeNet's Inception branch-4 shapes (3x3 / s1 / p1, ceil mode) on one GPU.

Times the native maxpool_fwd / maxpool_bwd kernels against a same-size copy (the HBM reference) and
torch's own max_pool2d, and prints effective TB/s of the bytes each must move (x read once, y and
the 1-byte argmax written once; backward: dy + pos read, dx written).

    python scripts/pool_probe.py [--batch 128] [--iters 50]
"""
import argparse
import os
import sys
import json

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(28, 192), (28, 256), (14, 480), (14, 512), (14, 528), (7, 832)]


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    dev = torch.device("cuda:0")
    for hw, c in SHAPES:
        x = torch.randn(a.batch, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y, pos = C.maxpool_fwd(x, 3, 1, 1, True, True)
        dy = torch.randn_like(y)
        nbytes = x.numel() * 2
        t_fwd = timed(lambda: C.maxpool_fwd(x, 3, 1, 1, True, True), a.iters)
        t_bwd = timed(lambda: C.maxpool_bwd(dy, pos, hw, hw, 3, 1, 1), a.iters)
        buf = torch.empty_like(x)
        t_copy = timed(lambda: buf.copy_(x), a.iters)
        t_torch = timed(lambda: F.max_pool2d(x, 3, 1, 1, ceil_mode=True), a.iters)
        rec = {"hw": hw, "c": c, "batch": a.batch, "MB": round(nbytes / 1e6, 1),
               "fwd_us": round(t_fwd, 1), "fwd_TBps": round(2.5 * nbytes / t_fwd / 1e6, 2),
               "bwd_us": round(t_bwd, 1), "bwd_TBps": round(2.5 * nbytes / t_bwd / 1e6, 2),
               "copy_us": round(t_copy, 1), "copy_TBps": round(2 * nbytes / t_copy / 1e6, 2),
               "torch_fwd_us": round(t_torch, 1)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
