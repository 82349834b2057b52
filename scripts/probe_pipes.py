#!/usr/bin/env python3
"""Main-loop (PIPE) sweep of the step's 3x3 forward / data-gradient and 1x1 weight-gradient (gemm_tn) shapes at
ResNet-50 bs1280, after the round-5 swizzled operand images: median of 30 per (shape, pipe), two repetitions,
results checked against the default. One JSON line per measurement. usage: python scripts/probe_pipes.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv_tiles import timeit  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30)).item()


def main():
    import torch
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    dev = torch.device("cuda:0")
    CL = torch.channels_last
    N = 1280
    for C_, H, pipes in ((128, 28, (0, 2, 3, 4, 6)), (256, 14, (2, 6)), (512, 7, (2, 6))):
        x = torch.randn(N, C_, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(C_, C_, 3, 3, device=dev) * 0.03).to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn(N, C_, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        C.set_mfma_pipeline(-1)
        yr = C.conv3x3_fwd(x, w, 1, True, 0)[0]
        dr = C.conv3x3_dgrad(dy, w, None, 0)
        timeit(lambda: C.conv3x3_fwd(x, w, 1, True, 0), 10)
        for rep in range(2):
            for p in (-1,) + pipes:
                C.set_mfma_pipeline(p)
                e = max(rel(C.conv3x3_fwd(x, w, 1, True, 0)[0], yr), rel(C.conv3x3_dgrad(dy, w, None, 0), dr))
                f = timeit(lambda: C.conv3x3_fwd(x, w, 1, True, 0), 30)
                d = timeit(lambda: C.conv3x3_dgrad(dy, w, None, 0), 30)
                print(json.dumps({"op": "conv3x3", "C": C_, "H": H, "rep": rep, "pipe": p, "fwd_ms": round(f, 4),
                                  "dgrad_ms": round(d, 4), "rel_err": e}), flush=True)
        C.set_mfma_pipeline(-1)
        del x, w, dy, yr, dr
        torch.cuda.empty_cache()
    # 1x1 weight gradients not served by the one-pass kernel (stages 3-4 and the strided downsamples): dW = dY^T X
    for M, Co, Ci in ((250880, 1024, 256), (250880, 256, 1024), (62720, 2048, 512), (62720, 512, 2048),
                      (250880, 1024, 512), (62720, 2048, 1024), (1003520, 512, 256)):
        a = torch.randn(M, Co, device=dev).to(torch.bfloat16)
        b = torch.randn(M, Ci, device=dev).to(torch.bfloat16)
        C.set_mfma_pipeline(-1)
        ref = C.gemm_tn(a, b, torch.float32)
        for rep in range(2):
            for p in (-1, 0, 2, 4, 6):
                C.set_mfma_pipeline(p)
                e = rel(C.gemm_tn(a, b, torch.float32), ref)
                t = timeit(lambda: C.gemm_tn(a, b, torch.float32), 30)
                print(json.dumps({"op": "gemm_tn", "M": M, "Cout": Co, "Cin": Ci, "rep": rep, "pipe": p,
                                  "ms": round(t, 4), "rel_err": e}), flush=True)
        C.set_mfma_pipeline(-1)
        del a, b, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
