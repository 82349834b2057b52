"""Micro-benchmark: native MFMA GEMMs vs torch (hipBLASLt) and MIOpen 1x1 conv on ResNet-50 shapes.

Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); random operands.
"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True


def timeit(fn, iters=20):
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


# (M = N*H*W at batch 256, Cin, Cout) for the ResNet-50 1x1 convs
shapes = [(802816, 64, 64), (802816, 64, 256), (802816, 256, 64), (200704, 512, 128), (200704, 128, 512),
          (50176, 1024, 256), (50176, 256, 1024), (12544, 2048, 512), (12544, 512, 2048)]
rows = []
for M, Cin, Cout in shapes:
    X = torch.randn(M, Cin, device=dev).to(torch.bfloat16)
    W = torch.randn(Cout, Cin, device=dev).to(torch.bfloat16) * 0.05
    dY = torch.randn(M, Cout, device=dev).to(torch.bfloat16)
    Wt = W.t().contiguous()
    n, h = M // 256, int((M // 256) ** 0.5)
    x4 = X.view(256, h, h, Cin).permute(0, 3, 1, 2)
    w4 = W.view(Cout, Cin, 1, 1).contiguous(memory_format=torch.channels_last)
    byts = lambda *ts: sum(t.numel() * t.element_size() for t in ts)  # noqa: E731
    r = {"M": M, "Cin": Cin, "Cout": Cout}
    r["fwd_native_ms"] = timeit(lambda: C.gemm_nt(X, W, False))
    r["fwd_native_stats_ms"] = timeit(lambda: C.gemm_nt(X, W, True))
    r["fwd_torch_mm_ms"] = timeit(lambda: X @ W.t())
    r["fwd_miopen_conv_ms"] = timeit(lambda: torch.nn.functional.conv2d(x4, w4))
    r["dgrad_native_ms"] = timeit(lambda: C.gemm_nt(dY, Wt, False))
    r["dgrad_native_kmajor_ms"] = timeit(lambda: C.gemm_nt(dY, W, False, None, True))
    # dgrad whose output is a fused BN's dy: + the BN backward-reduction partials in the epilogue
    xbn = torch.randn(M, Cin, device=dev).to(torch.bfloat16)
    wsb = torch.randn(7 * Cin, device=dev)
    mk = torch.randint(0, 255, ((M * Cin + 7) // 8,), device=dev, dtype=torch.uint8)
    r["dgrad_bn1_ms"] = timeit(lambda: C.gemm_nt_bn(dY, W, None, True, xbn, wsb, None, 1))
    r["dgrad_bn2_ms"] = timeit(lambda: C.gemm_nt_bn(dY, W, None, True, xbn, wsb, mk, 2))
    x4b = xbn.view(256, h, h, Cin).permute(0, 3, 1, 2)
    ws7 = torch.ones(7 * Cin, device=dev)
    r["bn_bwd_sep_ms"] = timeit(lambda: C.bn_act_bwd(x4b, None, mk, x4b, ws7, None, 2, True))
    for pipe in (0, 2, 3):
        C.set_mfma_pipeline(pipe)
        r[f"fwd_p{pipe}"] = timeit(lambda: C.gemm_nt(X, W, True))
        r[f"dgrad_p{pipe}"] = timeit(lambda: C.gemm_nt(dY, W, False, None, True))
        r[f"wgrad_p{pipe}"] = timeit(lambda: C.gemm_tn(dY, X, torch.float32, 1.0))
    C.set_mfma_pipeline(-1)
    r["dgrad_torch_mm_ms"] = timeit(lambda: dY @ W)
    r["wgrad_native_ms"] = timeit(lambda: C.gemm_tn(dY, X, torch.float32, 1.0))
    r["wgrad_torch_mm_ms"] = timeit(lambda: dY.t() @ X)
    fwd_bytes = byts(X, W) + M * Cout * 2
    r["fwd_native_TBps"] = fwd_bytes / r["fwd_native_ms"] / 1e9
    r["flops_fwd_TF"] = 2 * M * Cin * Cout / r["fwd_native_ms"] / 1e9
    rows.append(r)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
