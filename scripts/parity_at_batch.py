#!/usr/bin/env python3
"""Teacher-forced parity (utils/parity.py) of the native training step at a given model and batch,
judged on chosen segments, as one JSON line -- the large-batch companion of a bench record.

The native step runs whole (every fusion and hand-off in the graph); the listed segments are then
re-run alone in fp32 PyTorch on the native path's own inputs and output gradients, with activation
and gradient storage rounded to bf16 like the native path (``bf16_grads``, needed at large batch:
tests/test_gpu_bench_batch.py explains the sqrt(rows) storage noise). Bounds are the bench-batch
test's: outputs 2e-2, input gradients 3e-2, weight gradients 5e-2.

usage: python scripts/parity_at_batch.py --model resnet152 --batch 1280 --segments stem,layer1.0,layer1.1,layer1.2
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--model", default="resnet152")
    ap.add_argument("--batch", type=int, default=1280)
    ap.add_argument("--segments", default="stem,layer1.0,layer1.1,layer1.2")
    ap.add_argument("--seed", type=int, default=11)
    a = ap.parse_args()
    import torch

    from distributed_learning_amd.models import get_spec
    from distributed_learning_amd.ops import _ext
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.utils.parity import teacher_forced, worst

    _ext.require()
    dev = torch.device("cuda:0")
    spec = get_spec(a.model)
    torch.manual_seed(1234)
    m = spec.build().to(dev).to(memory_format=torch.channels_last)
    dnn.bf16_weights(m)
    g = torch.Generator().manual_seed(a.seed)
    x = torch.rand(a.batch, *spec.input_shape, generator=g).to(dev, torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, spec.num_classes, (a.batch,), generator=g).to(dev)
    only = set(a.segments.split(","))
    rows = teacher_forced(m, x, y, only=only, bf16_grads=True)
    w, where = worst(rows)
    ok = all(r["out"] <= 2e-2 and (r["dx"] is None or r["dx"] <= 3e-2) and r["dw"] <= 5e-2 for r in rows)
    print(json.dumps({"model": a.model, "batch": a.batch, "segments": rows, "worst": w, "worst_at": where,
                      "bounds": {"out": 2e-2, "dx": 3e-2, "dw": 5e-2}, "ok": ok,
                      "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
