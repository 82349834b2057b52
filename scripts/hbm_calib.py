"""HBM calibration on one MI355X: write-only (fill), read-only (sum), copy and read+write ratios with
torch's own streaming kernels, so the GEMM epilogues' write-heavy traffic can be priced against
what the memory system actually delivers. Prints one JSON line per case."""
import json

import torch

dev = torch.device("cuda:0")


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / it


n = 1 << 29  # 1 GiB of bf16
x = torch.empty(n, dtype=torch.bfloat16, device=dev).normal_()
y = torch.empty_like(x)
z = torch.empty(n // 4, dtype=torch.bfloat16, device=dev).normal_()
cases = {
    "write_fill": (lambda: y.fill_(1.0), 2 * n),
    "read_sum": (lambda: x.sum(dtype=torch.float32), 2 * n),
    "copy": (lambda: y.copy_(x), 4 * n),
    "read1_write4 (expand)": (lambda: y.view(-1, 4).copy_(z.view(-1, 1).expand(-1, 4)), 2 * n + n // 2),
}
for k, (fn, byts) in cases.items():
    ms = t(fn)
    print(json.dumps({"case": k, "ms": round(ms, 4), "GB": round(byts / 1e9, 3), "TBps": round(byts / ms / 1e9, 3)}))
