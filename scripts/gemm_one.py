#!/usr/bin/env python3
"""One 1x1 GEMM shape in a loop (for counter passes): ``gemm_one.py M K N fwd|dgrad [iters]``; forward with
BN statistics, data gradient with k-major weights, the production dispatch (tile=0)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from distributed_learning_amd.ops import _ext

    M, K, N, kind = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    C = _ext.require()
    dev = torch.device("cuda:0")
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = (torch.randn(N, K, device=dev) if kind == "fwd" else torch.randn(K, N, device=dev)).to(torch.bfloat16)
    for _ in range(iters):
        C.gemm_nt(A, B, kind == "fwd", None, kind == "dgrad", 0)
    torch.cuda.synchronize()
    print("ok", M, K, N, kind, iters, flush=True)


if __name__ == "__main__":
    main()
