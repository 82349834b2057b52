"""A/B of MFMA tile configurations (operands rotated through 2 GiB of copies: HBM-cold, as in the model) (dla_kernels.h TileCfg) at the ResNet-50 bs256 shapes, in one
process with interleaved rounds; also checks each variant's output against the default tile's.

  python scripts/bench_tiles.py [tiles, default "1,4"]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
CL = torch.channels_last
tiles = [int(t) for t in (sys.argv[1] if len(sys.argv) > 1 else "1,4").split(",")]
if len(sys.argv) > 2:  # force the MFMA main-loop pipeline (0 / 2 / 3) for every variant
    C.set_mfma_pipeline(int(sys.argv[2]))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters, 4)


ROT_BYTES = 2 << 30  # rotate operand copies through 2 GiB so they are not Infinity-Cache (256 MB) hot


def copies(t):
    n = max(1, min(16, ROT_BYTES // max(1, t.numel() * t.element_size())))
    return [t] + [t.clone() for _ in range(n - 1)]


def timeit_rot(fn, ops, iters=20):
    """fn(*operand tuple); ops = list of tuples cycled per call."""
    for i in range(3):
        fn(*ops[i % len(ops)])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(*ops[i % len(ops)])
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters, 4)


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


for (Cin, H, Cout, stride) in [(64, 56, 64, 1), (128, 56, 128, 2), (128, 28, 128, 1), (256, 28, 256, 2),
                               (256, 14, 256, 1), (512, 14, 512, 2), (512, 7, 512, 1)]:
    N = 256
    x = torch.randn(N, Cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    OH = (H - 1) // stride + 1
    dy = torch.randn(N, Cout, OH, OH, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    flops = 2 * N * OH * OH * Cout * Cin * 9
    r = {"conv": f"{Cin}x{H}->{Cout}/s{stride}"}
    xs, dys = copies(x), copies(dy)
    ref_y = C.conv3x3_fwd(x, w, stride, True, tiles[0])
    ref_dx = C.conv3x3_dgrad(dy, w, None, tiles[0]) if stride == 1 else None
    for t in tiles:
        y = C.conv3x3_fwd(x, w, stride, True, t)
        r[f"fwd_t{t}"] = timeit_rot(lambda xx: C.conv3x3_fwd(xx, w, stride, True, t), [(c,) for c in xs])
        r[f"fwd_t{t}_TF"] = round(flops / r[f"fwd_t{t}"] / 1e9)
        r[f"fwd_t{t}_err"] = round(rel(y[0], ref_y[0]), 5)
        r[f"stats_t{t}_err"] = round(rel(y[1].sum(0), ref_y[1].sum(0)), 5)
        if stride == 1:
            dx = C.conv3x3_dgrad(dy, w, None, t)
            r[f"dgrad_t{t}"] = timeit_rot(lambda d: C.conv3x3_dgrad(d, w, None, t), [(c,) for c in dys])
            r[f"dgrad_t{t}_err"] = round(rel(dx, ref_dx), 5)
    print(json.dumps(r), flush=True)

for M, Cin, Cout in [(802816, 64, 256), (802816, 256, 64), (200704, 512, 128), (200704, 128, 512),
                     (50176, 1024, 256), (50176, 256, 1024), (12544, 2048, 512), (12544, 512, 2048)]:
    X = torch.randn(M, Cin, device=dev).to(torch.bfloat16)
    W = (torch.randn(Cout, Cin, device=dev) * 0.05).to(torch.bfloat16)
    dY = torch.randn(M, Cout, device=dev).to(torch.bfloat16)
    r = {"gemm": f"{M}x{Cin}->{Cout}"}
    Xs, dYs = copies(X), copies(dY)
    ref = C.gemm_nt(X, W, True, None, False, tiles[0])
    refd = C.gemm_nt(dY, W, False, None, True, tiles[0])[0]
    for t in tiles:
        o = C.gemm_nt(X, W, True, None, False, t)
        r[f"fwd_t{t}"] = timeit_rot(lambda xx: C.gemm_nt(xx, W, True, None, False, t), [(c,) for c in Xs])
        r[f"fwd_t{t}_err"] = round(rel(o[0], ref[0]), 5)
        od = C.gemm_nt(dY, W, False, None, True, t)[0]
        r[f"dgrad_t{t}"] = timeit_rot(lambda d: C.gemm_nt(d, W, False, None, True, t), [(c,) for c in dYs])
        r[f"dgrad_t{t}_err"] = round(rel(od, refd), 5)
    print(json.dumps(r), flush=True)
