"""Run one native conv / GEMM kernel shape repeatedly (target for rocprofv3 --pmc passes).

  python scripts/conv_one.py fwd|dgrad|wgrad Cin H Cout stride [iters] [pipe] [tile]
  python scripts/conv_one.py gemm M Cin Cout 1 [iters] [pipe] [tile]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
CL = torch.channels_last
op = sys.argv[1]
a, b, c, s = (int(v) for v in sys.argv[2:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 50
if len(sys.argv) > 7:
    C.set_mfma_pipeline(int(sys.argv[7]))
tile = int(sys.argv[8]) if len(sys.argv) > 8 else 0
N = int(os.environ.get("CONV_ONE_N", "256"))  # batch (the bench runs 1280)
if op == "gemm":
    M, Cin, Cout = a, b, c
    X = torch.randn(M, Cin, device=dev).to(torch.bfloat16)
    W = (torch.randn(Cout, Cin, device=dev) * 0.05).to(torch.bfloat16)
    fn = lambda: C.gemm_nt(X, W, True, None, False, tile)  # noqa: E731
else:
    Cin, H, Cout, stride = a, b, c, s
    x = torch.randn(N, Cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    OH = (H - 1) // stride + 1
    dy = torch.randn(N, Cout, OH, OH, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    fn = {"fwd": lambda: C.conv3x3_fwd(x, w, stride, True, tile),
          "dgrad": lambda: C.conv3x3_dgrad(dy, w),
          "wgrad": lambda: C.conv3x3_wgrad(dy, x, stride, torch.bfloat16)}[op]
for _ in range(iters):
    fn()
torch.cuda.synchronize()
print("done", op, sys.argv[2:])
