#!/usr/bin/env python3
"""Run-to-run determinism of the native forward / backward inside ONE process (race diagnosis).

Repeats forward (+ backward) of a model on one fixed batch ``--reps`` times and compares every
block output and every parameter gradient bitwise with the first repetition; prints the first
modules whose outputs differ. A difference here is an intra-kernel race (missing barrier / LDS
reuse), an uninitialised read, or a nondeterministic library kernel — not a stream-ordering bug.

    python scripts/fwd_determinism.py [--model resnet18] [--batch 16] [--reps 12]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--stem", action="store_true", help="also record the stem conv / stats / pooled output")
    ap.add_argument("--all", action="store_true", help="hook every module (convs and BNs run fused, so few fire)")
    a = ap.parse_args()
    from distributed_learning_amd.data import SyntheticBatches
    from distributed_learning_amd.models import get_spec
    from distributed_learning_amd.ops import nn as dnn
    from distributed_learning_amd.ops.loss import cross_entropy

    dev = torch.device("cuda:0")
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    spec = get_spec(a.model)
    torch.manual_seed(0)
    model = spec.build().to(dev).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    x, y = SyntheticBatches(a.batch, spec.input_shape, spec.num_classes, dev, dtype=torch.bfloat16, seed=3,
                            channels_last=True).next()
    names = [n for n, m in model.named_modules() if n and (a.all or n.count(".") <= 1)]  # layers, blocks, head
    mods = dict(model.named_modules())
    rec = {}

    def hook(name):
        def f(_m, _i, out):
            t = out[0] if isinstance(out, (tuple, list)) else out
            rec[name] = t.detach().clone()
        return f

    for n in names:
        mods[n].register_forward_hook(hook(n))
    ref = None
    bad = {}
    for rep in range(a.reps):
        rec.clear()
        for p in model.parameters():
            p.grad = None
        if a.stem:  # the stem pieces one by one (they run as fused ops, not module forwards)
            from distributed_learning_amd.ops import conv as nconv

            ys, st = nconv.stem_conv(x, model.conv1, want_stats=True)
            rec["stem_conv"] = ys.detach().clone()
            rec["stem_stats"] = st.detach().clone()
            rec["stem_pool"] = dnn.conv_bn_act_maxpool(x, model.conv1, model.bn1, model.maxpool).detach().clone()
        loss = cross_entropy(model(x), y)
        loss.backward()
        torch.cuda.synchronize()
        cur = {f"out:{k}": v for k, v in rec.items()}
        cur.update({f"grad:{k}": p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None})
        cur["loss"] = loss.detach().clone()
        if ref is None:
            ref = cur
            continue
        for k, v in cur.items():
            if not torch.equal(v, ref[k]):
                bad.setdefault(k, []).append(rep)
    order = list(ref)
    first = [k for k in order if k in bad]
    print(f"{a.model}: {len(first)} of {len(order)} recorded tensors differ in some repetition")
    for k in first[:25]:
        print(f"  {k}: reps {bad[k][:10]}")


if __name__ == "__main__":
    main()
