#!/usr/bin/env python3
"""Stride-2 3x3 data gradient of ResNet-50 stage 2 (Cin = Cout = 128, 56x56 input, bs1280): median of 30, three
repetitions, one JSON line (the tile follows DLA_TILE512 of the process). usage: python scripts/probe_s2dgrad.py"""
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
    w = (torch.randn(128, 128, 3, 3, device=dev) * 0.03).to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(1280, 128, 28, 28, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    timeit(lambda: C.conv3x3s2_dgrad(dy, w, 56, 56), 10)
    ms = [round(timeit(lambda: C.conv3x3s2_dgrad(dy, w, 56, 56), 30), 4) for _ in range(3)]
    print(json.dumps({"tile512": os.environ.get("DLA_TILE512", "default"), "ms": ms}), flush=True)


if __name__ == "__main__":
    main()
