#!/usr/bin/env python3
"""One fp32 conv pass in a loop (counter runs): conv_f32_one.py N Cin H Cout k pad fwd|wgrad [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from distributed_learning_amd.ops import _ext

    n, cin, h, cout, k, pad = (int(v) for v in sys.argv[1:7])
    kind = sys.argv[7]
    iters = int(sys.argv[8]) if len(sys.argv) > 8 else 10
    C = _ext.require()
    dev = torch.device("cuda:0")
    x = torch.randn(n, cin, h, h, device=dev).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, k, k, cin, device=dev)
    y = C.conv_f32_fwd(x, w, pad, 1)
    for _ in range(iters):
        if kind == "fwd":
            C.conv_f32_fwd(x, w, pad, 1)
        else:
            C.conv_f32_wgrad(y, x, k, k, pad, 1)
    torch.cuda.synchronize()
    print("ok", sys.argv[1:], flush=True)


if __name__ == "__main__":
    main()
