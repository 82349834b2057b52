#!/usr/bin/env python3
"""Stage-2 3x3 passes (Cout = 128, 28x28 output, bs1280) on the 512x128 tile vs the 128x128 tile: forward with the
BN-statistics epilogue (stride 1 and 2) and data gradient, interleaved, medians of 30 after a warm-up pass.
usage: [PROBE_N=512] python scripts/probe_tile512.py  (explicit tiles: the auto-pick threshold does not apply)"""
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
    N = int(os.environ.get("PROBE_N", "1280"))
    w = (torch.randn(128, 128, 3, 3, device=dev) * 0.03).to(torch.bfloat16).contiguous(memory_format=CL)
    for stride in (1, 2):
        H = 28 * stride
        x = torch.randn(N, 128, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn(N, 128, 28, 28, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
        timeit(lambda: C.conv3x3_fwd(x, w, stride, True, 1), 10)
        for rep in range(3):
            for t in (1, 9, 0):
                r = {"stride": stride, "rep": rep, "tile": t,
                     "fwd_ms": round(timeit(lambda: C.conv3x3_fwd(x, w, stride, True, t), 30), 4)}
                if stride == 1:
                    r["dgrad_ms"] = round(timeit(lambda: C.conv3x3_dgrad(dy, w, None, t), 30), 4)
                print(json.dumps(r), flush=True)
        del x, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
