#!/usr/bin/env python3
"""Deterministic replay for race detection.

Runs a few data-parallel training steps of a model on the native kernels with the full multi-rank
gradient path forced at world size 1 (autograd hooks -> comm-stream gather -> [all-reduce] ->
re-pointed gradients -> fused SGD), then saves every parameter and BN buffer. Every kernel on this
path is deterministic, so a run with the GPU serialised (``AMD_SERIALIZE_KERNEL=3``,
``HIP_LAUNCH_BLOCKING=1``) must produce bitwise the same tensors as a normal, concurrent run: any
difference is a missing stream/event dependency (a race between the compute and comm streams).

    python scripts/race_replay.py OUT.pt [--model resnet18] [--steps 3] [--batch 16]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--bucket_mb", type=float, default=1.0)
    ap.add_argument("--nodp", action="store_true", help="plain model, no DP wrapper / comm stream (diagnosis)")
    a = ap.parse_args()
    a.nodp = a.nodp or os.environ.get("RACE_NODP") == "1"
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    from distributed_learning_amd.data import SyntheticBatches
    from distributed_learning_amd.models import get_spec
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy
    from distributed_learning_amd.ops.optim import FusedSGD
    from distributed_learning_amd.parallel import PipelinedFusedDP, make_reducer
    from distributed_learning_amd.parallel import context as ctxmod
    from distributed_learning_amd.parallel.executor import NativeStreamExecutor

    c = ctxmod.init(backend="nccl")
    dev = c.device
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    spec = get_spec(a.model)
    torch.manual_seed(0)
    model = spec.build().to(dev).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    if a.nodp:
        w = model
        w.sync_gradients = lambda: None
        w.cleanup = lambda: None
    else:
        red = make_reducer("immediate", "builtin", native=True)
        w = PipelinedFusedDP(model, red, int(a.bucket_mb * 1024 * 1024), dev)
        w.sync.executor = NativeStreamExecutor(red.engine, "builtin", passthrough=False)
        w.sync.passthrough = False
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, master_weights=True)
    data = SyntheticBatches(a.batch, spec.input_shape, spec.num_classes, dev, dtype=torch.bfloat16, seed=3,
                            channels_last=True)
    losses = []
    for _ in range(a.steps):
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(w(x), y)
        loss.backward()
        if os.environ.get("RACE_JOIN") == "1":  # diagnosis: explicit join of the conv side stream
            from distributed_learning_amd.ops import conv as _conv

            for st in _conv._SIDE_STREAMS.values():
                torch.cuda.current_stream().wait_stream(st)
        if os.environ.get("RACE_SYNC") == "1":  # diagnosis: drain the device after backward
            torch.cuda.synchronize()
        w.sync_gradients()
        opt.step()
        losses.append(loss.detach())
    torch.cuda.synchronize()
    state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    state["__losses__"] = torch.stack(losses).float().cpu()
    torch.save(state, a.out)
    w.cleanup()
    ctxmod.shutdown()
    print(f"saved {len(state)} tensors, losses {[round(float(v), 5) for v in state['__losses__']]}")


if __name__ == "__main__":
    main()
