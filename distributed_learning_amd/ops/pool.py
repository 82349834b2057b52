"""NHWC max pooling on the native kernels (csrc/kernels/pool.hip).

:class:`MaxPool2d` is a drop-in ``nn.MaxPool2d`` (same constructor, same state) used by the model
zoo; with the ``native`` ops backend and a supported input (channels_last, C % 8 == 0, bf16/fp32,
no dilation / indices) it runs the fused forward that also records the 1-byte argmax window
position, and a gather-form backward (no zero-fill, no atomics). Everything else takes
``F.max_pool2d``. Reference usage: the GoogLeNet/ResNet stems (SURVEY.md §2.5 hot-path ops).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext


def _pair_same(v) -> int | None:
    if isinstance(v, (tuple, list)):
        return int(v[0]) if len(v) == 2 and v[0] == v[1] else None
    return int(v)


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil_mode):
        C = _ext.require()
        y, pos = C.maxpool_fwd(x, k, s, p, ceil_mode, x.requires_grad)
        ctx.geom = (x.shape[2], x.shape[3], k, s, p)
        ctx.save_for_backward(pos)
        return y

    @staticmethod
    def backward(ctx, dy):
        (pos,) = ctx.saved_tensors
        H, W, k, s, p = ctx.geom
        return _ext.require().maxpool_bwd(dy, pos, H, W, k, s, p), None, None, None, None


def supported(x: torch.Tensor, k, s, p, dilation, return_indices) -> bool:
    if return_indices or _pair_same(dilation) != 1:
        return False
    k, s, p = _pair_same(k), _pair_same(s if s is not None else k), _pair_same(p)
    if None in (k, s, p) or not (1 <= k <= 15 and 2 * p <= k):
        return False
    return (x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


def max_pool2d(x, kernel_size, stride=None, padding=0, dilation=1, ceil_mode=False):
    from .nn import get_backend

    if get_backend() == "native" and supported(x, kernel_size, stride, padding, dilation, False):
        k = _pair_same(kernel_size)
        s = _pair_same(stride if stride is not None else kernel_size)
        return _MaxPool.apply(x, k, s, _pair_same(padding), bool(ceil_mode))
    return F.max_pool2d(x, kernel_size, stride, padding, dilation, ceil_mode)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        if self.return_indices:
            return super().forward(x)
        return max_pool2d(x, self.kernel_size, self.stride, self.padding, self.dilation, self.ceil_mode)


class _GlobalAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return _ext.require().gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return _ext.require().gap_bwd(dy, *ctx.hw)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``flatten(adaptive_avg_pool2d(x, 1), 1)`` -> [N, C]. Native path (channels_last bf16/fp32,
    C % 8 == 0): one reduction kernel forward, and a backward that writes dy / HW straight into the
    channels_last layout (torch's expand makes the last block's BN backward copy a strided tensor)."""
    from .nn import get_backend

    if get_backend() == "native" and x.dim() == 4 and x.is_cuda and x.shape[1] % 8 == 0 and \
            x.dtype in (torch.bfloat16, torch.float32) and x.is_contiguous(memory_format=torch.channels_last) and \
            x.data_ptr() % 16 == 0:
        return _GlobalAvgPool.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
