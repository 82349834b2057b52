"""Uninitialised-memory probe: run training steps with every torch.empty / at::empty filled with NaN
(torch.use_deterministic_algorithms(warn_only) + fill_uninitialized_memory) and compare with a normal
run: a kernel whose result depends on memory it never wrote shows up as non-finite or different
tensors (diagnosis helper, round 3 g25).

    python scripts/uninit_probe.py [--model resnet18] [--steps 2] [--batch 16]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(model_name, steps, batch, fill):
    from distributed_learning_amd.data import SyntheticBatches
    from distributed_learning_amd.models import get_spec
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.optim import FusedSGD

    torch.use_deterministic_algorithms(fill, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = fill
    dev = torch.device("cuda:0")
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    spec = get_spec(model_name)
    torch.manual_seed(0)
    model = spec.build().to(dev).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, master_weights=True)
    data = SyntheticBatches(batch, spec.input_shape, spec.num_classes, dev, dtype=torch.bfloat16, seed=3,
                            channels_last=True)
    grads = []
    for _ in range(steps):
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        cross_entropy(model(x), y).backward()
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None})
        opt.step()
    torch.cuda.synchronize()
    torch.use_deterministic_algorithms(False)
    return grads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    ref = run(a.model, a.steps, a.batch, False)
    got = run(a.model, a.steps, a.batch, True)
    clean = True
    for s, (gr, gg) in enumerate(zip(ref, got)):
        nonfinite = [n for n, t in gg.items() if not torch.isfinite(t).all()]
        differ = [n for n in gr if not torch.equal(gr[n], gg[n])]
        print(f"step {s}: {len(nonfinite)} non-finite grads {nonfinite[:6]}; {len(differ)} differ {differ[:6]}", flush=True)
        clean = clean and not nonfinite and not differ
    print("RESULT", "clean" if clean else "UNINIT-DEPENDENT", flush=True)


if __name__ == "__main__":
    main()
