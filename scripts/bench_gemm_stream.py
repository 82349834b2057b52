"""Streaming vs tile 1x1 GEMM at the ResNet-50 bs1024 shapes (interleaved in one process).

fwd = Y = X W^T with BN statistics (the forward conv), dgrad = dX = dY W (k-major weights, no addend).
Bytes = A read + C written (+ weights); TB/s against that logical traffic.

    python scripts/bench_gemm_stream.py [--batch 1024] [--out gpurun_out/x.jsonl]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_learning_amd.ops import _ext  # noqa: E402


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
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    C = _ext.require()
    dev = torch.device("cuda", 0)
    b = a.batch
    # (name, pixels per image, K, N): forward shapes (K = Cin, N = Cout); the dgrad of a conv with
    # (Cin, Cout) is the GEMM (K = Cout, N = Cin)
    convs = [("l1.conv1", 3136, 256, 64), ("l1.conv3", 3136, 64, 256), ("l1.b0.conv1", 3136, 64, 64),
             ("l2.b0.conv1", 3136, 256, 128), ("l2.conv3", 784, 128, 512), ("l2.ds", 784, 256, 512),
             ("l3.conv3", 196, 256, 1024), ("l3.b0.conv1", 784, 512, 256)]
    rows = []
    for name, px, cin, cout in convs:
        M = b * px
        for kind, K, N in (("fwd", cin, cout), ("dgrad", cout, cin), ("dgrad_fork", cout, cin)):
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)
            if kind == "fwd":
                B, km, st = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16), False, True
            else:
                B, km, st = (torch.randn(K, N, device=dev) * 0.05).to(torch.bfloat16), True, False
            # the fork's data gradient: + the identity gradient, masked by the ReLU bits
            D = torch.randn(M, N, device=dev).to(torch.bfloat16) if kind == "dgrad_fork" else None
            mk = torch.randint(0, 256, ((M * N + 7) // 8,), device=dev, dtype=torch.uint8) if D is not None else None
            C.set_gemm_stream(1)
            served = C.gemm_stream_rows(M, N, K, K, N, km, D is not None) > 0
            r = {"layer": name, "pass": kind, "M": M, "K": K, "N": N, "stream_served": served}
            byts = (M * K + M * N + K * N) * 2 + ((M * N * 2 + M * N // 8) if D is not None else 0)
            for mode in ((1, 0) if served else (0,)):
                C.set_gemm_stream(mode)
                ms = timeit(lambda: C.gemm_nt(A, B, st, D, km, 0, mk))
                key = "stream" if mode else "tile"
                r[f"{key}_ms"] = round(ms, 4)
                r[f"{key}_TBps"] = round(byts / ms / 1e9, 3)
            C.set_gemm_stream(-1)
            rows.append(r)
            print(json.dumps(r), flush=True)
            del A, B, D, mk
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
