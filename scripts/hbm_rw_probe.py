#!/usr/bin/env python3
"""HBM write / read / copy rates on this box (torch kernels, 2 GiB buffers): the ceiling a write-dominated
kernel (a 1x1 GEMM whose output is 4x its input) can reach. Median of 10."""
import torch


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(it):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


n = 1 << 29  # 2 GiB of fp32
x = torch.empty(n, device="cuda")
y = torch.empty(n, device="cuda")
x.fill_(1.0)
gb = n * 4 / 1e9
w = t(lambda: y.fill_(2.0))
r = t(lambda: x.sum())
c = t(lambda: y.copy_(x))
print(f"write-only {gb / w:.2f} TB/s  read-only {gb / r:.2f} TB/s  copy {2 * gb / c:.2f} TB/s (read+write)", flush=True)
