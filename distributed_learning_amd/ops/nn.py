"""Model hot-path ops with a selectable backend.

``bn_act(x, bn, relu, residual)`` computes ``act(BN(x) [+ residual])`` — the Conv->BN->ReLU(->add)
tail of every ResNet/GoogLeNet block. Backends:

* ``"torch"``  — stock PyTorch ops (MIOpen BN, elementwise ReLU/add): the reference behaviour.
* ``"native"`` — the fused HIP kernel (csrc/kernels/bn_act.hip): one pass to compute the batch
  statistics, one fused normalise+affine+add+ReLU pass, and a two-pass fused backward; bf16
  NHWC activations, fp32 statistics.

The backend is process-global (``set_backend``) so a model definition does not change between
the parity path and the MI355X path.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

_BACKEND = "torch"


def set_backend(name: str) -> None:
    global _BACKEND
    if name not in ("torch", "native"):
        raise ValueError(f"unknown ops backend {name!r} (expected 'torch' or 'native')")
    if name == "native":
        from . import _ext

        _ext.require()
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


def bf16_weights(model: nn.Module) -> nn.Module:
    """Mixed-precision layout: conv/linear weights in bf16, normalisation params/stats in fp32.

    Used with ``FusedSGD(master_weights=True)`` (fp32 masters live in the optimizer), so the
    forward runs natively in bf16 with no autocast weight casts and gradients leave backward in
    bf16 (half the all-reduce bytes)."""
    norm_types = (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.LayerNorm, nn.GroupNorm)
    for m in model.modules():
        if isinstance(m, norm_types):
            continue
        for name, p in list(m.named_parameters(recurse=False)):
            p.data = p.data.to(torch.bfloat16)
    return model


def _torch_bn_act(x, bn: nn.BatchNorm2d, relu: bool, residual):
    y = bn(x)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y, inplace=residual is not None)
    return y


def bn_act(x: torch.Tensor, bn: nn.BatchNorm2d, relu: bool = True, residual: torch.Tensor | None = None):
    if _BACKEND == "native" and x.is_cuda:
        from .bn_act import fused_bn_act

        return fused_bn_act(x, bn, relu, residual)
    return _torch_bn_act(x, bn, relu, residual)


# 1x1 convolutions on the native MFMA GEMMs (ops/conv.py) — separately switchable so the conv path
# can be A/B'd against MIOpen while the fused BN stays on.
_NATIVE_CONV = False


def set_native_conv(on: bool) -> None:
    global _NATIVE_CONV
    if on:
        from . import _ext

        _ext.require()
    _NATIVE_CONV = bool(on)


def native_conv() -> bool:
    return _NATIVE_CONV


# fp32 convolutions on the fp32 matrix-core kernels (ops/conv_f32.py) -- the --precision fp32 path
_NATIVE_F32 = False


def set_native_conv_f32(on: bool) -> None:
    global _NATIVE_F32
    if on:
        from . import _ext

        _ext.require()
    _NATIVE_F32 = bool(on)


def native_conv_f32() -> bool:
    return _NATIVE_F32


def _conv(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """``conv(x)``: fp32 inputs on the native fp32 MFMA kernels when switched on and supported."""
    if _NATIVE_F32 and _BACKEND == "native" and x.is_cuda and x.dtype == torch.float32:
        from . import conv_f32

        if conv_f32.supported(x, conv):
            return conv_f32.conv(x, conv)
    return conv(x)


def linear(x: torch.Tensor, fc: nn.Linear) -> torch.Tensor:
    """``fc(x)``; with the native backend and native convs, on the MFMA GEMMs (ops/linear.py)."""
    if _BACKEND == "native" and _NATIVE_CONV and x.is_cuda:
        from .linear import linear as native_linear

        return native_linear(x, fc)
    return fc(x)


def conv_bn_act(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d, relu: bool = True,
                residual: torch.Tensor | None = None, presubsampled: bool = False, defer: bool = False):
    """``act(BN(conv(x)) [+ residual])``. With the native backend and native convs, a 1x1 conv runs as
    an MFMA GEMM whose epilogue also produces BN's batch statistics (one pass over the conv output
    saved). ``presubsampled``: ``x`` is already the stride-2 subsample a strided 1x1 ``conv`` would
    take (conv_bn_act_fork(..., subsample=True)), so the conv runs with stride 1. ``defer``: the result
    feeds only the next bottleneck's conv_bn_act_fork, which may write it itself (ops/bn_act.py PendingApply)."""
    from .bn_act import ensure

    if _BACKEND == "native" and _NATIVE_CONV and x.is_cuda:
        from . import conv as nconv
        from .bn_act import fused_bn_act, supported as bn_supported

        if nconv.supported(x, conv):
            stride = 1 if presubsampled else None
            y, stats = nconv.conv1x1(x, conv, want_stats=bn.training, stride=stride)
            if stats is not None and not bn_supported(y, bn, residual):
                stats = None
            return fused_bn_act(y, bn, relu, residual, stats, defer=defer)
        ensure(x)  # a deferred BN output is written by a 1x1 consumer's GEMM only
        if nconv.supported3x3(x, conv):
            want = bn.training and nconv.CONV3_POLICY["fwd"] == "native"
            y, stats = nconv.conv3x3(x, conv, want_stats=want)
            if stats is not None and not bn_supported(y, bn, residual):
                stats = None
            return fused_bn_act(y, bn, relu, residual, stats, defer=defer)
    ensure(x)
    if presubsampled:
        y = F.conv2d(x, conv.weight, conv.bias, 1, conv.padding, conv.dilation, conv.groups)
        return bn_act(y, bn, relu, residual)
    return bn_act(_conv(x, conv), bn, relu, residual)


def _native_conv_stats(x: torch.Tensor, conv: nn.Conv2d, want_stats: bool, presubsampled: bool = False):
    """(y, stats-or-None) from a native 1x1 / 3x3 conv, or None when neither applies."""
    from . import conv as nconv
    from .bn_act import ensure

    if nconv.supported(x, conv):
        return nconv.conv1x1(x, conv, want_stats=want_stats, stride=1 if presubsampled else None)
    ensure(x)
    if not presubsampled and nconv.supported3x3(x, conv):
        want = want_stats and nconv.CONV3_POLICY["fwd"] == "native"
        return nconv.conv3x3(x, conv, want_stats=want)
    return None


# act(BN(conv(x)) + BN_d(conv_d(xd))) in one apply pass (bench A/B switch)
DUAL_RESIDUAL = True

def conv_bn_add_conv_bn_act(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d, xd: torch.Tensor,
                            conv_d: nn.Conv2d, bn_d: nn.BatchNorm2d, relu: bool = True,
                            presubsampled: bool = False, defer: bool = False) -> torch.Tensor:
    """``act(BN(conv(x)) + BN_d(conv_d(xd)))`` — a residual block's last conv plus its downsample
    shortcut. Native path: both convs emit their BN statistics and one apply pass reads both conv
    outputs (the shortcut BN's output is never written). ``presubsampled``: ``xd`` is already the
    stride-2 subsample the strided ``conv_d`` would take. (Issuing the shortcut conv on a second stream
    measured slower: 73.42-73.62 vs 72.46-72.53 ms/step, profiles/r3/g21_branch_stream_ab.txt.)"""
    if _BACKEND == "native" and _NATIVE_CONV and DUAL_RESIDUAL and x.is_cuda and bn.training and bn_d.training:
        from .bn_act import dual_supported, fused_bn_add_bn_act

        a = _native_conv_stats(x, conv, True)
        b = _native_conv_stats(xd, conv_d, True, presubsampled) if a is not None else None
        if a is not None and b is not None and dual_supported(a[0], bn, b[0], bn_d):
            return fused_bn_add_bn_act(a[0], bn, b[0], bn_d, relu, a[1], b[1], defer=defer)
        if a is not None and b is not None:  # convs done; BN the plain way
            from .bn_act import fused_bn_act

            ident = fused_bn_act(b[0], bn_d, False, None, b[1])
            return fused_bn_act(a[0], bn, relu, ident, a[1])
    ident = conv_bn_act(xd, conv_d, bn_d, relu=False, presubsampled=presubsampled)
    return conv_bn_act(x, conv, bn, relu=relu, residual=ident)


def conv_bn_act_maxpool(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d, pool: nn.Module):
    """``pool(relu(BN(conv(x))))`` — the ResNet / GoogLeNet stem. Native path: the BN+ReLU+max-pool runs as one
    fused op (the 112x112 activation and its gradient are never written)."""
    if _BACKEND == "native" and x.is_cuda and isinstance(pool, nn.MaxPool2d):
        from .bn_act import fused_bn_relu_maxpool

        if _NATIVE_CONV and not x.requires_grad:
            from . import conv as nconv

            if nconv.supported_stem(x, conv):  # 7x7/s2 MFMA conv whose epilogue emits BN's statistics
                y, stats = nconv.stem_conv(x, conv, want_stats=bn.training)
                return fused_bn_relu_maxpool(y, bn, pool, stats)
        if _NATIVE_CONV:  # a 1x1 / 3x3 conv before the pool (GoogLeNet's conv3 -> maxpool2)
            r = _native_conv_stats(x, conv, bn.training)
            if r is not None:
                return fused_bn_relu_maxpool(r[0], bn, pool, r[1])
        return fused_bn_relu_maxpool(_conv(x, conv), bn, pool)
    return pool(conv_bn_act(x, conv, bn, relu=True))


# conv_bn_act_fork(..., subsample=True) may return the stride-2 subsample (see there); tests flip it
FORK_SUBSAMPLE = True


def conv_bn_act_fork(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d, relu: bool = True,
                     subsample: bool = False):
    """``(act(BN(conv(x))), identity[, x_sub])`` for a residual block whose identity branch starts
    at ``x`` itself.

    On the native path the returned identity is an alias of ``x`` produced by the same autograd
    node as the conv, so the block-input gradient (conv dgrad + identity gradient) is summed in
    the dgrad GEMM epilogue (ops/conv.py::_Conv1x1Fork). With ``subsample`` a third output is
    ``x[:, :, ::2, ::2]`` for a stride-2 downsample conv (``conv_bn_act(..., presubsampled=True)``),
    whose compact gradient the same epilogue adds at the even pixels; None when the native path
    does not apply (then subsample inside the downsample conv as usual)."""
    from .bn_act import ensure

    if _BACKEND == "native" and _NATIVE_CONV and x.is_cuda:
        from . import conv as nconv
        from .bn_act import fused_bn_act, supported as bn_supported

        sub_ok = subsample and FORK_SUBSAMPLE and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0
        if nconv.fork_supported(x, conv):  # writes a deferred x itself (or materialises it first)
            y, stats, ident, xs = nconv.conv1x1_fork(x, conv, want_stats=bn.training, sub=sub_ok)
            if stats is not None and not bn_supported(y, bn, None):
                stats = None
            out = fused_bn_act(y, bn, relu, None, stats)
            return (out, ident, xs if sub_ok else None) if subsample else (out, ident)
    ensure(x)
    out = conv_bn_act(x, conv, bn, relu)
    return (out, x, None) if subsample else (out, x)
