#!/usr/bin/env python3
"""Per-layer fp32 convolution time, native fp32 MFMA kernels vs MIOpen (TF32 off), GoogLeNet bs128 shapes.

Each distinct conv of the GoogLeNet (torchvision v0.6 layout) step: forward, input gradient and weight gradient
timed separately (median of 15, interleaved in one process), with the achieved TFLOP/s. One JSON line per layer.

usage: python scripts/bench_conv_f32.py [--batch 128] [--out FILE.jsonl]
"""
import argparse
import json
import sys

import torch
import torch.nn as nn

sys.path.insert(0, ".")
from distributed_learning_amd.ops import conv_f32  # noqa: E402

# (Cin, H, Cout, k, pad, stride, calls per step)
LAYERS = {}


def add(cin, h, cout, k, pad=0, stride=1):
    key = (cin, h, cout, k, pad, stride)
    LAYERS[key] = LAYERS.get(key, 0) + 1


def googlenet():
    add(3, 224, 64, 7, 3, 2)
    add(64, 56, 64, 1)
    add(64, 56, 192, 3, 1)
    blocks = [(192, 28, 64, 96, 128, 16, 32, 32), (256, 28, 128, 128, 192, 32, 96, 64),
              (480, 14, 192, 96, 208, 16, 48, 64), (512, 14, 160, 112, 224, 24, 64, 64),
              (512, 14, 128, 128, 256, 24, 64, 64), (512, 14, 112, 144, 288, 32, 64, 64),
              (528, 14, 256, 160, 320, 32, 128, 128), (832, 7, 256, 160, 320, 32, 128, 128),
              (832, 7, 384, 192, 384, 48, 128, 128)]
    for cin, h, c1, c3r, c3, c5r, c5, pp in blocks:
        add(cin, h, c1, 1)
        add(cin, h, c3r, 1)
        add(c3r, h, c3, 3, 1)
        add(cin, h, c5r, 1)
        add(c5r, h, c5, 3, 1)
        add(cin, h, pp, 1)


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
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cudnn.benchmark = False
    googlenet()
    dev = torch.device("cuda:0")
    out = open(a.out, "w") if a.out else None
    from distributed_learning_amd.ops import _ext

    C = _ext.require()
    tot = {"native2": 0.0, "native1": 0.0, "miopen": 0.0}
    for (cin, h, cout, k, pad, stride), calls in LAYERS.items():
        conv = nn.Conv2d(cin, cout, k, stride=stride, padding=pad, bias=False).to(dev).to(memory_format=torch.channels_last)
        x = torch.randn(a.batch, cin, h, h, device=dev).contiguous(memory_format=torch.channels_last)
        x.requires_grad_(stride == 1)
        y = conv(x)
        dy = torch.randn_like(y)
        oh = y.shape[2]
        flop = 2.0 * a.batch * oh * oh * cout * cin * k * k
        row = {"layer": f"{cin}x{h}x{h}->{cout} k{k}s{stride}", "calls": calls}
        for name, fwd in (("native2", lambda: conv_f32.conv(x, conv)), ("native1", lambda: conv_f32.conv(x, conv)),
                          ("miopen", lambda: conv(x))):
            C.set_conv_f32_buffers(1 if name == "native1" else 2)

            def step(fwd=fwd):
                conv.weight.grad = None
                if x.grad is not None:
                    x.grad = None
                fwd().backward(dy)
            tf = timeit(lambda fwd=fwd: fwd())
            tt = timeit(step)
            row[name] = {"fwd_ms": round(tf, 4), "fwd_bwd_ms": round(tt, 4),
                         "tflops": round(flop * (3 if stride == 1 else 2) / tt / 1e9, 1)}
            tot[name] += tt * calls
        print(json.dumps(row), flush=True)
        if out:
            out.write(json.dumps(row) + "\n")
    print(json.dumps({"total_fwd_bwd_ms_per_step": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
