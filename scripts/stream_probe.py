"""Which output rows of the streaming 1x1 GEMM come out wrong or unwritten, per variant (round 3 g28)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
torch.manual_seed(0)


def rnd(*shape):
    return torch.randn(*shape, device=dev).to(torch.bfloat16)


for M, K, N in [(12544, 128, 64), (12544, 128, 256), (12544, 64, 64), (12544, 256, 64)]:
    for kmajor in (True, False):
        for stats in (False, True):
            A = rnd(M, K)
            B = rnd(K, N) if kmajor else rnd(N, K)
            C.set_gemm_stream(0)
            ref = C.gemm_nt(A, B, stats, None, kmajor)[0].float()
            C.set_gemm_stream(1)
            torch.cuda.synchronize()
            # poison the caching allocator's next block of this size so unwritten rows are visible
            junk = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
            del junk
            got = C.gemm_nt(A, B, stats, None, kmajor)[0].float()
            C.set_gemm_stream(-1)
            badrows = (~torch.isclose(got, ref, rtol=2e-2, atol=2e-2)).any(1).nonzero().flatten()
            tiles = sorted(set((badrows // 128).tolist()))
            print(f"M={M} K={K} N={N} kmajor={kmajor} stats={stats}: bad rows {badrows.numel()}, "
                  f"bad 128-row tiles {len(tiles)} first {tiles[:10]}", flush=True)
