#!/usr/bin/env python3
"""Stage-2 (C = 128, 28x28, bs1280) 3x3 probe: measurement-order check of the auto vs explicit 128x128 forward
tile (same kernel), and the weight gradient of every 3x3 shape of the step under each main loop (g49: 512 split-K blocks best). One JSON line per
measurement. usage: python scripts/probe_c128.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv_tiles import timeit  # noqa: E402


def main():
    import torch
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    dev = torch.device("cuda:0")
    CL = torch.channels_last
    N, C_, H = 1280, 128, 28
    x = torch.randn(N, C_, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(C_, C_, 3, 3, device=dev) * 0.03).to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(N, C_, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    for rep in range(3):
        for t in (0, 1):
            print(json.dumps({"rep": rep, "fwd_tile": t, "ms": round(timeit(lambda: C.conv3x3_fwd(x, w, 1, True, t), 30), 4)}), flush=True)
            print(json.dumps({"rep": rep, "dgrad_tile": t, "ms": round(timeit(lambda: C.conv3x3_dgrad(dy, w, None, t), 30), 4)}), flush=True)
    del x, dy
    # weight gradients of every 3x3 shape of the step (stride-2: the first block of stages 2-4), per main loop
    for C_, H, s in ((128, 28, 1), (128, 56, 2), (256, 14, 1), (256, 28, 2), (512, 7, 1), (512, 14, 2)):
        OH = H // s
        x = torch.randn(N, C_, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn(N, C_, OH, OH, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        ref = C.conv3x3_wgrad(dy, x, s, torch.float32)
        for rep in range(2):
            for pipe in (-1, 2, 4):
                C.set_mfma_pipeline(pipe)
                out = C.conv3x3_wgrad(dy, x, s, torch.float32)
                err = ((out - ref).abs().max() / ref.abs().max()).item()
                ms = timeit(lambda: C.conv3x3_wgrad(dy, x, s, torch.float32), 30)
                print(json.dumps({"C": C_, "H": H, "stride": s, "rep": rep, "pipe": pipe, "ms": round(ms, 4),
                                  "rel_err": err}), flush=True)
        C.set_mfma_pipeline(-1)
        del x, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
