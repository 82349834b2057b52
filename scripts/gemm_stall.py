#!/usr/bin/env python3
"""One 1x1 GEMM launch shape in a loop, for stall-attribution counter passes (verdict r5 item 1a).

  gemm_stall.py M K N fwd|dgrad|dgrad_add [iters] [tile]

fwd: forward with the BN-statistics epilogue (A [M, K], W [N, K]); fwdns: the same without statistics; dgrad: data gradient with k-major
weights; dgrad_add: data gradient with the fused identity-gradient addend [M, N] (the conv1 data
gradients of the bottleneck blocks, which the streaming kernel does not take at K = 256). tile 0 = the
production dispatch (pick_tile / streaming), else a forced TileCfg.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from distributed_learning_amd.ops import _ext

    M, K, N, kind = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    tile = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    C = _ext.require()
    if os.environ.get("STALL_PIPE"):  # MFMA main-loop pipeline override (A/B)
        C.set_mfma_pipeline(int(os.environ["STALL_PIPE"]))
    if os.environ.get("STALL_STREAM"):  # streaming-kernel mode override (1: every K <= 256)
        C.set_gemm_stream(int(os.environ["STALL_STREAM"]))
    dev = torch.device("cuda:0")
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    fwd = kind.startswith("fwd")
    B = (torch.randn(N, K, device=dev) if fwd else torch.randn(K, N, device=dev)).to(torch.bfloat16)
    D = torch.randn(M, N, device=dev).to(torch.bfloat16) if kind == "dgrad_add" else None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(iters):
        if i == iters // 2:
            e0.record()
        C.gemm_nt(A, B, kind == "fwd", D, not fwd, tile, None, None, 0, 0)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / (iters - iters // 2)
    gb = (M * K + M * N * (2 if D is not None else 1) + N * K) * 2 / 1e9
    print(f"ok {M} {K} {N} {kind} tile={tile} {ms:.4f} ms {gb / ms:.2f} TB/s (compulsory bytes)", flush=True)


if __name__ == "__main__":
    main()
