"""Time the Cout-128 3x3 weight gradients (ResNet-50 stage 2 at bs1280) on the 128x128 vs 128x256 tiles."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
CL = torch.channels_last


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


for (N, H, stride) in [(1280, 28, 1), (1280, 56, 2)]:
    x = torch.randn(N, 128, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    oh = (H - 1) // stride + 1
    dy = torch.randn(N, 128, oh, oh, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    flops = 2 * N * oh * oh * 128 * 128 * 9
    r = {"N": N, "H": H, "stride": stride}
    for rep in range(2):
        for m in (0, 1):
            C.set_wgrad_w4(m)
            t = timeit(lambda: C.conv3x3_wgrad(dy, x, stride, torch.bfloat16))
            r.setdefault(f"w4_{m}_ms", []).append(t)
    C.set_wgrad_w4(-1)
    r["tflops_w4_0"] = round(flops / min(r["w4_0_ms"]) / 1e9, 1)
    r["tflops_w4_1"] = round(flops / min(r["w4_1_ms"]) / 1e9, 1)
    print(json.dumps(r), flush=True)
