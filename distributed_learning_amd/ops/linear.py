"""Fully connected layers on the framework's own MFMA GEMMs (csrc/kernels/gemm.hip).

``y = x W^T + b`` for bf16 activations [B, in] and weights [out, in]:

* forward: ``gemm_nt(x, W)``. The bias enters as the epilogue addend, read as a stride-0 row
  (``bias.expand(B, out)``), so there is no separate broadcast-add kernel;
* dx = dy W: ``gemm_nt`` with W read k-major as stored;
* dW = dy^T x: ``gemm_tn``, split-K over the batch rows;
* db = dy^T 1: the same ``gemm_tn`` against a cached [B, 8] ones block (column 0). It is a
  fixed-order reduction, deterministic like the other weight gradients.

It replaces the hipBLASLt ``Cijk_*`` kernels and the bias kernels of the ResNet / GoogLeNet heads,
which were the last library kernels of the native bf16 step. In the reference these layers are
``torch.nn.Linear`` (its hub GoogLeNet and torchvision-style ResNets).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext

_ONES: dict = {}


def _ones(rows: int, device) -> torch.Tensor:
    key = (rows, device)
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(rows, 8, dtype=torch.bfloat16, device=device)
    return t


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        C = _ext.require()
        w = weight.to(torch.bfloat16).contiguous()
        add = None
        if bias is not None:
            add = bias.to(torch.bfloat16).expand(x.shape[0], w.shape[0])
        y, _ = C.gemm_nt(x, w, False, add)
        ctx.save_for_backward(x, w)
        ctx.wdtype = weight.dtype
        ctx.bdtype = bias.dtype if bias is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx, _ = C.gemm_nt(dy, w, False, None, True)
        if ctx.needs_input_grad[1]:
            odt = ctx.wdtype if ctx.wdtype in (torch.float32, torch.bfloat16) else torch.float32
            dw = C.gemm_tn(dy, x, odt, 1.0).to(ctx.wdtype)
        if ctx.bdtype is not None and ctx.needs_input_grad[2]:
            db = C.gemm_tn(dy, _ones(dy.shape[0], dy.device), torch.float32, 1.0)[:, 0].to(ctx.bdtype).contiguous()
        return dx, dw, db


def supported(x: torch.Tensor, fc: nn.Linear) -> bool:
    return (x.is_cuda and x.dim() == 2 and x.dtype == torch.bfloat16 and x.is_contiguous()
            and x.data_ptr() % 16 == 0 and fc.in_features % 8 == 0 and fc.out_features % 8 == 0)


def linear(x: torch.Tensor, fc: nn.Linear) -> torch.Tensor:
    """``fc(x)`` on the native GEMMs when they apply, else ``F.linear``."""
    if supported(x, fc):
        return _Linear.apply(x, fc.weight, fc.bias)
    return F.linear(x, fc.weight, fc.bias)
