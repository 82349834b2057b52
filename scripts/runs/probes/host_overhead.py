"""Host-side cost of one eager training step (GoogLeNet / ResNet): wall time per step with the GPU
work small (tiny batch) so the host is the bottleneck, fused Inception on vs off, plus a cProfile of
the fused step's Python hot spots. Diagnostics only.

    python scripts/host_overhead.py [--model googlenet] [--batch 8] [--steps 20]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("LOCAL_RANK", "0")

import torch  # noqa: E402

from distributed_learning_amd.data import SyntheticBatches  # noqa: E402
from distributed_learning_amd.models import get_spec  # noqa: E402
from distributed_learning_amd.ops import inception as ninc  # noqa: E402
from distributed_learning_amd.ops import nn as dnn  # noqa: E402
from distributed_learning_amd.ops.loss import cross_entropy  # noqa: E402
from distributed_learning_amd.ops.optim import FusedSGD  # noqa: E402
from distributed_learning_amd.parallel import PipelinedFusedDP, make_reducer  # noqa: E402
from distributed_learning_amd.parallel import context as ctxmod  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="googlenet")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    c = ctxmod.init(backend="nccl")
    dev = c.device
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    spec = get_spec(a.model)
    model = spec.build().to(dev).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    model = PipelinedFusedDP(model, make_reducer("immediate", "builtin", native=True), 8 << 20, dev)
    opt = FusedSGD(model.module.parameters(), lr=0.01, momentum=0.5, master_weights=True)
    data = SyntheticBatches(a.batch, spec.input_shape, spec.num_classes, dev, dtype=torch.bfloat16,
                            channels_last=True)

    def step():
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(model(x), y)
        loss.backward()
        model.sync_gradients()
        opt.step()

    orig = ninc.supported
    for label, fused in (("fused", True), ("unfused", False)):
        ninc.supported = orig if fused else (lambda *args: False)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        t1 = time.perf_counter()  # host issue time (GPU may still run)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{label}: host issue {1e3 * (t1 - t0) / a.steps:.2f} ms/step, wall {1e3 * (t2 - t0) / a.steps:.2f} ms/step",
              flush=True)
    ninc.supported = orig
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
