"""Localise an uninitialised-memory read to one block: every residual block of a model runs forward +
backward in isolation with and without NaN-filled allocations (see uninit_probe.py), and the block's
output, input gradient and parameter gradients are compared (diagnosis helper, round 3 g26).

    python scripts/uninit_blocks.py [--model resnet18] [--batch 16]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def block_run(blk, x, g, fill):
    torch.use_deterministic_algorithms(fill, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = fill
    xi = x.clone().requires_grad_(True)
    for p in blk.parameters():
        p.grad = None
    y = blk(xi)
    y.backward(g)
    torch.cuda.synchronize()
    torch.use_deterministic_algorithms(False)
    out = {"y": y.detach().float().clone(), "dx": xi.grad.detach().float().clone()}
    out.update({n: p.grad.detach().float().clone() for n, p in blk.named_parameters() if p.grad is not None})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    from distributed_learning_amd.models import get_spec
    from distributed_learning_amd.ops import nn as dnn

    dev = torch.device("cuda:0")
    dnn.set_backend("native")
    dnn.set_native_conv(True)
    torch.manual_seed(0)
    model = get_spec(a.model).build().to(dev).to(memory_format=torch.channels_last)
    dnn.bf16_weights(model)
    x = torch.rand(a.batch, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        h = dnn.conv_bn_act_maxpool(x, model.conv1, model.bn1, model.maxpool)
    for lname in ("layer1", "layer2", "layer3", "layer4"):
        for i, blk in enumerate(getattr(model, lname)):
            inp = h.detach().contiguous(memory_format=torch.channels_last)
            with torch.no_grad():
                yshape = blk(inp).shape
            g = torch.randn(yshape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            r0 = block_run(blk, inp, g, False)
            r1 = block_run(blk, inp, g, True)
            bad = [k for k in r0 if not torch.equal(r0[k], r1[k])]
            nonfin = [k for k in r1 if not torch.isfinite(r1[k]).all()]
            print(f"{lname}.{i}: {len(bad)} differ {bad[:8]}; non-finite {nonfin[:8]}", flush=True)
            with torch.no_grad():
                h = blk(inp)


if __name__ == "__main__":
    main()
