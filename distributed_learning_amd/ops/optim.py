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
    def __init__(self, params, lr: float = 0.01, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, grad_scale: float = 1.0):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, grad_scale=grad_scale)
        super().__init__(params, defaults)
        self._tables = {}

    def _group_tensors(self, group):
        ps = [p for p in group["params"] if p.grad is not None]
        return ps, [p.grad for p in ps]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            ps, gs = self._group_tensors(group)
            if not ps:
                continue
            mom = group["momentum"]
            native = ps[0].is_cuda and ps[0].dtype == torch.float32 and _ext.available()
            if ps[0].is_cuda and not native and _ext.gpu_required():
                _ext.require()
            first = False
            bufs: List[Optional[torch.Tensor]] = []
            for p in ps:
                st = self.state[p]
                if mom != 0 and "momentum_buffer" not in st:
                    st["momentum_buffer"] = torch.zeros_like(p)
                    first = True
                bufs.append(st.get("momentum_buffer"))
            if native:
                key = (gi, tuple(p.data_ptr() for p in ps), tuple(g.data_ptr() for g in gs))
                tab = self._tables.get(gi)
                if tab is None or tab[0] != key:
                    C = _ext.require()
                    tab = (key, C.SgdTable(ps, gs, bufs if mom != 0 else [], []))
                    self._tables[gi] = tab
                tab[1].step(group["lr"], mom, group["dampening"], group["weight_decay"], group["nesterov"],
                            group["grad_scale"], first)
            else:
                self._reference_step(ps, gs, bufs, group, first)
        return loss

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
