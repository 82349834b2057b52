"""FusedSGD: ``torch.optim.SGD`` semantics in ONE multi-tensor HIP launch per step.

Reference: ``optim.SGD(model.parameters(), lr=0.01, momentum=0.5)`` (/root/reference/src/main.py:36)
stepped once per batch (main.py:91) — a for-each over 187 (GoogLeNet) / 161 (ResNet-50) tensors.
On MI355X the update is HBM-bound (fp32: read p, g, m; write p, m = 20 B/param; ResNet-50 ≈ 0.5 GB
≈ 0.1 ms), so the win is launch count: one launch over a device-resident tensor table
(csrc/kernels/multi_tensor.hip) instead of one or several per tensor.

Extras over torch.optim.SGD: ``grad_scale`` (fold 1/N or loss-scale into the update) and an
optional bf16 shadow copy of each parameter written in the same pass.
On CPU (or without the extension) it falls back to the exact ``torch.optim.SGD`` math.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from . import _ext


class FusedSGD(torch.optim.Optimizer):
    """SGD(momentum, dampening, nesterov, weight_decay) as one native launch per (grad dtype) group.

    ``master_weights=True``: low-precision (bf16) parameters get an fp32 master copy in the
    optimizer state; the kernel reads the bf16 gradient, updates master + momentum in fp32 and
    writes the rounded bf16 parameter back in the same pass (no separate cast kernels, and no
    autocast weight casts in the forward). fp32 parameters (e.g. BatchNorm) are updated in place.
    """

    def __init__(self, params, lr: float = 0.01, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, grad_scale: float = 1.0,
                 master_weights: bool = False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, grad_scale=grad_scale)
        super().__init__(params, defaults)
        self.master_weights = master_weights
        self._tables = {}

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict casts floating-point state to each parameter's dtype
        (through a policy it calls by class name); the fp32 master copies and momentum buffers of
        bf16 parameters must stay fp32 for a bit-exact resume, so they are re-installed afterwards."""
        keep = {}
        for idx, st in state_dict.get("state", {}).items():
            for k in ("master", "momentum_buffer"):
                if k in st and torch.is_tensor(st[k]) and st[k].dtype == torch.float32:
                    keep[(idx, k)] = st[k]
        super().load_state_dict(state_dict)
        params = [p for g in self.param_groups for p in g["params"]]
        for (idx, k), v in keep.items():
            p = params[idx]
            self.state[p][k] = v.to(device=p.device, copy=True)
        self._tables = {}

    def _master(self, p):
        if p.dtype == torch.float32 or not self.master_weights:
            return None
        st = self.state[p]
        if "master" not in st:
            st["master"] = torch.empty_like(p, dtype=torch.float32).copy_(p)
        return st["master"]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        from . import conv as _conv

        _conv.join_all_devices()  # late weight gradients of a backward that raised before its own join
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            mom = group["momentum"]
            # partition by (grad dtype, first-step) so every launch has uniform semantics
            parts = {}
            for p in ps:
                st = self.state[p]
                first = mom != 0 and "momentum_buffer" not in st
                if mom != 0 and first:
                    st["momentum_buffer"] = torch.zeros_like(p, dtype=torch.float32)
                parts.setdefault((p.grad.dtype, first), []).append(p)
            for (gdt, first), plist in parts.items():
                self._step_part(gi, group, plist, first)
        return loss

    def _step_part(self, gi, group, ps, first):
        mom = group["momentum"]
        gs = [p.grad for p in ps]
        masters = [self._master(p) for p in ps]
        bufs = [self.state[p].get("momentum_buffer") for p in ps]
        native = ps[0].is_cuda and _ext.available() and all(
            (m is not None) or p.dtype == torch.float32 for p, m in zip(ps, masters))
        if ps[0].is_cuda and not native and _ext.gpu_required() and not _ext.available():
            _ext.require()
        if not native:
            targets = [m if m is not None else p for p, m in zip(ps, masters)]
            self._reference_step(targets, [g.float() for g in gs], bufs, group, first)
            for p, m in zip(ps, masters):
                if m is not None:
                    p.copy_(m)
            return
        fp = [m if m is not None else p for p, m in zip(ps, masters)]
        shadows = [p for p, m in zip(ps, masters) if m is not None]
        if shadows and len(shadows) != len(ps):  # mixed within a part cannot happen: grads share dtype
            raise RuntimeError("FusedSGD: mixed master/non-master parameters in one launch group")
        # By-value tensor lists in the kernel arguments (<= 32 tensors per launch): no device table,
        # so gradients may live anywhere and move every step (autograd-owned, set_to_none, views).
        _ext.require().sgd_step_list(fp, gs, bufs if mom != 0 else [], shadows, group["lr"], mom,
                                     group["dampening"], group["weight_decay"], group["nesterov"],
                                     group["grad_scale"], first)

    @staticmethod
    def _reference_step(ps, gs, bufs, group, first):
        lr, mom, damp, wd, nest, gsc = (group["lr"], group["momentum"], group["dampening"], group["weight_decay"],
                                        group["nesterov"], group["grad_scale"])
        for p, g, b in zip(ps, gs, bufs):
            d = g * gsc if gsc != 1.0 else g
            if wd != 0:
                d = d.add(p, alpha=wd)
            if mom != 0:
                if first:
                    b.copy_(d)
                else:
                    b.mul_(mom).add_(d, alpha=1 - damp)
                d = d.add(b, alpha=mom) if nest else b
            p.add_(d, alpha=-lr)
