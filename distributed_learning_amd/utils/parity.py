"""Teacher-forced, segment-by-segment comparison of the native training step with fp32 PyTorch.

A whole-model bf16-vs-fp32 comparison at random init is chaotic: relative errors compound over 50
layers, so the early layers' gradients differ by O(1) (the round-2 smoke printed ``conv1.grad rel
1.34`` for both the native path and torch autocast), and a bound that passes that checks nothing.
Here the native path runs the whole model once, exactly as in training (autograd connects the
segments, so every cross-segment fusion — the dgrad-epilogue BN partials handed to the producer's
BatchNorm, the residual-gradient handoff into the next block's fork — is in the graph), and every
segment boundary's activation and gradient is captured. Then each segment is re-run alone in fp32
PyTorch (MIOpen convs, torch BN, the same bf16-valued weights held in fp32) on the native path's
own input, and back-propagated from the native path's own output gradient. Errors cannot compound:
each segment is judged on its own inputs. Per segment the check covers the output, the input
gradient and every parameter gradient (relative L2 error).

Storage precision is the framework's policy, not a kernel property: the native path keeps every
activation (conv outputs, ReLU outputs) in bf16. An fp32 reference that keeps them in fp32 makes a
different ReLU decision for every pre-activation within bf16 rounding of zero, and each such flip
moves one full gradient element — with ~0.3 % of elements near zero that alone is a ~5 % relative
L2 difference in every input gradient, whatever the kernels do. So the reference rounds what the
native path stores (conv inputs and outputs, linear inputs and outputs, max-pool inputs) to bf16 in its forward
(straight-through in its backward) and computes everything else — convolutions, BatchNorm
statistics and normalisation, ReLU, pooling, the whole backward — in fp32. What remains is the
kernels' arithmetic error: fp32 accumulation order and the bf16 rounding of gradient tensors.

Segments: ResNet — stem (conv+BN+ReLU+max-pool), every residual block, head (global average pool +
FC); GoogLeNet — the two fused stem stages, conv2, every Inception block and max-pool, head.
The head excludes dropout (random masks) and GoogLeNet's aux heads (outside the loss, reference
network.py:41).
"""
from __future__ import annotations

import copy
from typing import Callable, Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

Segment = Tuple[str, Callable, List[nn.Module]]


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def segments(model: nn.Module) -> List[Segment]:
    from ..models.googlenet import GoogLeNet
    from ..models.resnet import ResNet
    from ..ops import nn as dnn
    from ..ops.pool import global_avg_pool

    segs: List[Segment] = []
    if isinstance(model, ResNet):
        segs.append(("stem", lambda m, x: dnn.conv_bn_act_maxpool(x, m.conv1, m.bn1, m.maxpool), ["conv1", "bn1"]))
        for li in range(1, 5):
            for bi in range(len(getattr(model, f"layer{li}"))):
                name = f"layer{li}.{bi}"
                segs.append((name, (lambda li, bi: lambda m, x: getattr(m, f"layer{li}")[bi](x))(li, bi), [name]))
        segs.append(("head", lambda m, x: dnn.linear(global_avg_pool(x), m.fc), ["fc"]))
        return segs
    if isinstance(model, GoogLeNet):
        segs.append(("stem1", lambda m, x: dnn.conv_bn_act_maxpool(x, m.conv1.conv, m.conv1.bn, m.maxpool1), ["conv1"]))
        segs.append(("conv2", lambda m, x: m.conv2(x), ["conv2"]))
        segs.append(("stem3", lambda m, x: dnn.conv_bn_act_maxpool(x, m.conv3.conv, m.conv3.bn, m.maxpool2), ["conv3"]))
        for name in ["inception3a", "inception3b", "maxpool3", "inception4a", "inception4b", "inception4c",
                     "inception4d", "inception4e", "maxpool4", "inception5a", "inception5b"]:
            segs.append((name, (lambda n: lambda m, x: getattr(m, n)(x))(name), [name]))
        segs.append(("head", lambda m, x: dnn.linear(global_avg_pool(x), m.fc), ["fc"]))
        return segs
    raise TypeError(f"no segment map for {type(model).__name__}")


def _bf16_ste(t: torch.Tensor) -> torch.Tensor:
    """Round to bf16 in the forward, identity in the backward."""
    return t + (t.to(torch.bfloat16).to(t.dtype) - t).detach()


class _Bf16Both(torch.autograd.Function):
    """Round to bf16 in the forward AND round the gradient to bf16 in the backward: the storage
    precision of the native path's gradient tensors (conv data gradients, BN-backward outputs)."""

    @staticmethod
    def forward(ctx, t):
        return t.to(torch.bfloat16).to(t.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def bf16_storage_hooks(model: nn.Module, grads: bool = False) -> list:
    """Round the inputs and outputs of every Conv2d / Linear of ``model`` to bf16 (straight-through),
    i.e. the activation storage precision of the native path. ``grads``: round the gradients that
    cross those points too (the native path stores every activation gradient in bf16). Returns the
    hook handles."""
    rnd = _Bf16Both.apply if grads else _bf16_ste
    handles = []
    for m in model.modules():
        if isinstance(m, nn.MaxPool2d):  # the native pools take the max of the stored (bf16) activations
            handles.append(m.register_forward_pre_hook(lambda mod, args: tuple(
                rnd(a) if torch.is_tensor(a) and a.is_floating_point() else a for a in args)))
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            handles.append(m.register_forward_pre_hook(lambda mod, args: tuple(
                rnd(a) if torch.is_tensor(a) and a.is_floating_point() else a for a in args)))
            handles.append(m.register_forward_hook(lambda mod, args, out: rnd(out)))
    return handles


def _params(model: nn.Module, names: List[str]) -> Dict[str, nn.Parameter]:
    out = {}
    for n in names:
        mod = model.get_submodule(n)
        for pn, p in mod.named_parameters():
            out[f"{n}.{pn}"] = p
    return out


def teacher_forced(model: nn.Module, x: torch.Tensor, y: torch.Tensor,
                   bf16_storage: bool = True, only=None, bf16_grads: bool = False) -> List[Dict[str, float]]:
    """Run the native step on ``model`` (bf16 weights, channels_last, on the GPU) and compare every
    segment with fp32 PyTorch. Returns one row per segment: ``out`` (output rel. error), ``dx``
    (input-gradient rel. error; None for the first segment) and ``dw`` (max over the segment's
    parameter gradients, with ``dw_worst`` naming it); the head row also has ``dlogits`` (the fused
    cross-entropy's gradient vs torch's on the same logits). ``bf16_storage``: the reference rounds
    stored activations to bf16 like the native path (module docstring); False compares against pure
    fp32 activations (then ReLU-decision flips dominate the gradient errors). ``only``: names of the
    segments to compare (the native step still runs whole; e.g. the early segments at the benchmark
    batch, where the largest tensors and indices live). ``bf16_grads``: the reference also rounds the
    activation gradients to bf16 where the native path stores them. Needed at large batch: a weight
    gradient or BN-bias gradient whose true value nearly cancels over N*H*W rows (BN-backward outputs
    sum to zero per channel) picks up the per-element bf16 rounding of the stored gradients as
    ~2^-9 sqrt(N*H*W) relative noise, which is storage policy, not kernel error."""
    from ..ops import nn as dnn
    from ..ops.loss import cross_entropy

    segs = segments(model)
    ref = copy.deepcopy(model)
    for p in ref.parameters():
        p.data = p.data.float()
    prev_backend, prev_conv = dnn.get_backend(), dnn.native_conv()
    rows: List[Dict[str, float]] = []
    try:
        # ---- native run: the segments chained under autograd, boundaries retained ------------
        dnn.set_backend("native")
        dnn.set_native_conv(True)
        model.zero_grad(set_to_none=True)
        acts = [x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)]
        for _, fn, _ in segs:
            a = fn(model, acts[-1])
            a.retain_grad()
            acts.append(a)
        logits = acts[-1]
        loss = cross_entropy(logits, y)
        loss.backward()
        torch.cuda.synchronize()
        # ---- fp32 reference, one segment at a time on the native path's own tensors ----------
        dnn.set_backend("torch")
        dnn.set_native_conv(False)
        hooks = bf16_storage_hooks(ref, grads=bf16_grads) if bf16_storage else []
        for k, (name, fn, mods) in enumerate(segs):
            if only is not None and name not in only:
                continue
            ref.zero_grad(set_to_none=True)
            xin = acts[k].detach().float().contiguous(memory_format=torch.channels_last)
            xin.requires_grad_(k > 0)
            out = fn(ref, xin)
            gout = acts[k + 1].grad
            row: Dict[str, float] = {"segment": name, "out": _rel(acts[k + 1].detach().float(), out.detach())}
            out.backward(gout.float())
            row["dx"] = _rel(acts[k].grad.float(), xin.grad) if k > 0 else None
            worst, wname = 0.0, ""
            nat_p, ref_p = _params(model, mods), _params(ref, mods)
            for pn, rp in ref_p.items():
                if rp.grad is None:
                    continue
                e = _rel(nat_p[pn].grad.float(), rp.grad)
                if e > worst:
                    worst, wname = e, pn
            row["dw"], row["dw_worst"] = worst, wname
            if name == "head":
                lg = logits.detach().float()
                dl = (F.softmax(lg, 1) - F.one_hot(y, lg.shape[1]).float()) / lg.shape[0]
                row["dlogits"] = _rel(gout.float(), dl)
            rows.append(row)
        for h in hooks:
            h.remove()
    finally:
        dnn.set_backend(prev_backend)
        dnn.set_native_conv(prev_conv)
    return rows


def worst(rows: List[Dict[str, float]]) -> Tuple[float, str]:
    """Largest error over all segments and checks, and where it occurred."""
    w, where = 0.0, ""
    for r in rows:
        for k in ("out", "dx", "dw", "dlogits"):
            v = r.get(k)
            if v is not None and v > w:
                w, where = v, f"{r['segment']}.{k}" + (f" ({r['dw_worst']})" if k == "dw" else "")
    return w, where
