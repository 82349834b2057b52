"""Where does the fp32 (reference-precision) GoogLeNet bs128 step spend its time on MI355X?

The CLI's fp32 run measured 963 ms of backward per batch (gpurun_out/g08b). Times the torch-backend
step (fp32 params, fp32 activations, NCHW) under MIOpen immediate mode, MIOpen with find
(benchmark=True) and with MIOpen disabled (PyTorch's im2col + BLAS convolutions), and prints the
top ops of the slowest configuration from torch.profiler.

    python scripts/runs/probes/fp32_googlenet_probe.py [--batch 128] [--configs immediate,nomiopen,find]
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from distributed_learning_amd.models import get_spec  # noqa: E402
from distributed_learning_amd.ops import nn as dnn  # noqa: E402
from distributed_learning_amd.ops.loss import cross_entropy  # noqa: E402


def step(model, x, y):
    out = model(x)
    loss = cross_entropy(out, y)
    loss.backward()
    return loss


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--configs", default="immediate,nomiopen,find")
    ap.add_argument("--profile", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dnn.set_backend("torch")
    dnn.set_native_conv(False)
    torch.manual_seed(0)
    model = get_spec("googlenet").build().to(dev).train()
    x = torch.randn(a.batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    for cfg in a.configs.split(","):
        torch.backends.cudnn.enabled = cfg != "nomiopen"
        torch.backends.cudnn.benchmark = cfg == "find"
        t0 = time.time()
        step(model, x, y)
        torch.cuda.synchronize()
        first = time.time() - t0
        ts = []
        for _ in range(a.iters):
            model.zero_grad(set_to_none=True)
            t0 = time.time()
            step(model, x, y)
            torch.cuda.synchronize()
            ts.append(time.time() - t0)
        ms = sorted(ts)[len(ts) // 2] * 1e3
        print(json.dumps({"config": cfg, "first_s": round(first, 2), "ms_per_step": round(ms, 2),
                          "img_s": round(a.batch / ms * 1e3, 1)}), flush=True)
        if cfg == a.profile:
            from torch.profiler import ProfilerActivity, profile
            with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
                step(model, x, y)
                torch.cuda.synchronize()
            print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25), flush=True)


if __name__ == "__main__":
    main()
