"""Tile-config sweep of the native conv / GEMM forward at the compute-bound ResNet-50 bs512 shapes."""
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")


def timeit(fn, iters=10):
    for _ in range(2):
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


B = 512
for (H, Cin, Cout, s) in [(28, 128, 128, 1), (14, 256, 256, 1), (7, 512, 512, 1), (56, 64, 64, 1)]:
    x = torch.randn(B, Cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    fl = 2.0 * B * H * H * 9 * Cin * Cout
    r = {"conv3x3": [H, Cin, Cout]}
    for t in (1, 4):
        for pipe in ((2, 6) if t == 1 else (3, 7)):
            try:
                C.set_mfma_pipeline(pipe)
                ms = timeit(lambda: C.conv3x3_fwd(x, w, s, True, t))
                r[f"t{t}p{pipe}"] = round(fl / ms / 1e9)
            except Exception as e:  # noqa: BLE001
                r[f"t{t}p{pipe}"] = str(e)[:40]
    C.set_mfma_pipeline(2)
    ref = C.conv3x3_fwd(x, w, s, True, 1)[0]
    C.set_mfma_pipeline(7)
    r["eq_t4p7"] = bool(torch.equal(ref, C.conv3x3_fwd(x, w, s, True, 4)[0]))
    C.set_mfma_pipeline(2)
    ref = C.conv3x3_fwd(x, w, s, True, 1)[0]
    C.set_mfma_pipeline(7)
    r["eq_t4p7"] = bool(torch.equal(ref, C.conv3x3_fwd(x, w, s, True, 4)[0]))
    C.set_mfma_pipeline(-1)
    print(json.dumps(r), flush=True)
for (M, K, N) in [(100352, 1024, 256), (25088, 2048, 512), (25088, 512, 2048), (100352, 256, 1024), (401408, 256, 512)]:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    fl = 2.0 * M * K * N
    r = {"gemm": [M, K, N]}
    for t in (1, 4):
        for pipe in ((2, 6) if t == 1 else (3, 7)):
            try:
                C.set_mfma_pipeline(pipe)
                ms = timeit(lambda: C.gemm_nt(A, W, True, None, False, t))
                r[f"t{t}p{pipe}"] = round(fl / ms / 1e9)
            except Exception as e:  # noqa: BLE001
                r[f"t{t}p{pipe}"] = str(e)[:40]
    C.set_mfma_pipeline(2)
    ref = C.gemm_nt(A, W, True, None, False, 1)[0]
    C.set_mfma_pipeline(7)
    r["eq_t4p7"] = bool(torch.equal(ref, C.gemm_nt(A, W, True, None, False, 4)[0]))
    C.set_mfma_pipeline(-1)
    print(json.dumps(r), flush=True)
