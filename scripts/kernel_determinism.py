#!/usr/bin/env python3
"""Bitwise run-to-run determinism of single native kernels (race diagnosis).

Each op runs --reps times on fixed inputs; the count of repetitions whose output differs from the
first (and the largest difference) is printed per op and per MFMA pipeline (0 = register staging,
2 = LDS-DMA). Inputs are rotated through fresh allocations between repetitions so stale memory
differs from run to run (an uninitialised read shows up as a mismatch).

    python scripts/kernel_determinism.py [--reps 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops.conv import stem_pack_weight

    C = _ext.require()
    dev = torch.device("cuda:0")
    CL = torch.channels_last
    g = torch.Generator(device="cpu").manual_seed(0)

    def rnd(*shape, scale=1.0):
        return (torch.randn(*shape, generator=g) * scale).to(dev, torch.bfloat16)

    x3 = rnd(16, 3, 224, 224).contiguous(memory_format=CL)
    w7 = rnd(64, 3, 7, 7, scale=0.1)
    wpk = stem_pack_weight(w7)
    x64 = rnd(16, 64, 56, 56).contiguous(memory_format=CL)
    w33 = rnd(64, 64, 3, 3, scale=0.05).contiguous(memory_format=CL)
    w128 = rnd(128, 128, 3, 3, scale=0.05).contiguous(memory_format=CL)
    x128 = rnd(16, 128, 28, 28).contiguous(memory_format=CL)
    A = rnd(50176, 256)
    B = rnd(256, 256, scale=0.05)
    dy64 = rnd(16, 64, 112, 112).contiguous(memory_format=CL)
    ops = {
        "stem_fwd": lambda: torch.cat([t.reshape(-1).float() for t in C.stem_fwd(x3, wpk, True)[:2]]),
        "stem_wgrad": lambda: C.stem_wgrad(dy64, C.stem_fwd(x3, wpk, False)[2], 224, 224, torch.float32),
        "conv3x3_fwd_64": lambda: torch.cat([t.reshape(-1).float() for t in C.conv3x3_fwd(x64, w33, 1, True)]),
        "conv3x3_fwd_128": lambda: torch.cat([t.reshape(-1).float() for t in C.conv3x3_fwd(x128, w128, 1, True)]),
        "conv3x3_dgrad_64": lambda: C.conv3x3_dgrad(x64, w33),
        "conv3x3_wgrad_64": lambda: C.conv3x3_wgrad(x64, x64, 1, torch.float32),
        "gemm_nt_stats": lambda: torch.cat([t.reshape(-1).float() for t in C.gemm_nt(A, B, True)]),
        "gemm_tn": lambda: C.gemm_tn(A, A, torch.float32, 1.0),
    }
    junk = []
    for pipe in (2, 0):
        C.set_mfma_pipeline(pipe)
        for name, fn in ops.items():
            ref = fn().clone()
            bad, worst = 0, 0.0
            for _ in range(a.reps):
                junk.append(torch.randn(1 << 22, device=dev))  # churn the allocator: fresh memory contents
                if len(junk) > 8:
                    junk.pop(0)
                out = fn()
                if not torch.equal(out, ref):
                    bad += 1
                    worst = max(worst, (out.float() - ref.float()).abs().max().item())
            torch.cuda.synchronize()
            print(f"pipe {pipe} {name:18s}: {bad:3d} / {a.reps} repetitions differ (max |diff| {worst:.3e})", flush=True)
    C.set_mfma_pipeline(-1)


if __name__ == "__main__":
    main()
