"""Microbenchmark: native implicit-GEMM 3x3 convs vs MIOpen (via torch) at the ResNet-50 bs256 shapes."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd.ops import _ext  # noqa: E402

C = _ext.require()
dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
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


for (N, Cin, H, Cout, stride) in [(256, 64, 56, 64, 1), (256, 128, 56, 128, 2), (256, 128, 28, 128, 1),
                                  (256, 256, 28, 256, 2), (256, 256, 14, 256, 1), (256, 512, 14, 512, 2),
                                  (256, 512, 7, 512, 1)]:
    x = torch.randn(N, Cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    OH = (H - 1) // stride + 1
    dy = torch.randn(N, Cout, OH, OH, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    flops = 2 * N * OH * OH * Cout * Cin * 9
    r = {"N": N, "Cin": Cin, "H": H, "Cout": Cout, "stride": stride}
    r["fwd_native"] = timeit(lambda: C.conv3x3_fwd(x, w, stride, False))
    r["fwd_native_stats"] = timeit(lambda: C.conv3x3_fwd(x, w, stride, True))
    r["fwd_miopen"] = timeit(lambda: F.conv2d(x, w, None, stride, 1))
    for pipe in (0, 2, 3):
        C.set_mfma_pipeline(pipe)
        r[f"fwd_p{pipe}"] = timeit(lambda: C.conv3x3_fwd(x, w, stride, True))
        if stride == 1:
            r[f"dgrad_p{pipe}"] = timeit(lambda: C.conv3x3_dgrad(dy, w))
        r[f"wgrad_p{pipe}"] = timeit(lambda: C.conv3x3_wgrad(dy, x, stride, torch.bfloat16))
    C.set_mfma_pipeline(-1)
    if stride == 1:
        r["dgrad_native"] = timeit(lambda: C.conv3x3_dgrad(dy, w))
    else:
        r["dgrad_native"] = timeit(lambda: C.conv3x3s2_dgrad(dy, w, H, H))
    r["dgrad_miopen"] = timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, [stride, stride], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
    r["wgrad_native"] = timeit(lambda: C.conv3x3_wgrad(dy, x, stride, torch.bfloat16))
    r["wgrad_miopen"] = timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, w, None, [stride, stride], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
    r["fwd_native_TFs"] = round(flops / r["fwd_native"] / 1e9, 1)
    r["wgrad_native_TFs"] = round(flops / r["wgrad_native"] / 1e9, 1)
    print(json.dumps(r), flush=True)
