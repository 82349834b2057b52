"""Autograd wrapper for the fused BatchNorm(+residual)(+ReLU) HIP kernels (csrc/kernels/bn_act.hip).

Used by :func:`distributed_learning_amd.ops.nn.bn_act` when the ``native`` backend is selected.
Semantics match ``relu(batch_norm(x, training=bn.training) + residual)`` with PyTorch's running
statistics update (momentum, unbiased running variance). Inputs that the kernel does not cover
(channel counts not divisible by 8, non-channels_last layouts, cumulative-average momentum) take
the stock PyTorch path.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import knobs
from . import _ext
from . import limits as _limits


MASK_NONE, MASK_RECOMPUTE, MASK_BITS, MASK_Y = 0, 1, 2, 3


class BNLink:
    """Hand-off between a fused BN(+ReLU) and the native conv that consumes its output.

    The conv's data-gradient GEMM produces exactly this BN's dy, so its epilogue can also produce
    the BN backward's reduction partials (sum dy', sum dy'(x - mean)) while dy is still on chip
    (csrc/include/dla_mfma.h BnBwdEpi); the BN backward then skips its reduction pass over dy and x.
    The BN uses the partials only if the dy it receives is the very tensor that GEMM wrote — if the
    output had other consumers, autograd summed their gradients into a new tensor and the normal
    reduction runs."""

    __slots__ = ("x", "ws", "mask", "mode", "part", "dy_ptr")

    def __init__(self, x, ws, mask, mode):
        self.x, self.ws, self.mask, self.mode = x, ws, mask, mode
        self.part = None
        self.dy_ptr = None

    def publish(self, dy: torch.Tensor, part: torch.Tensor) -> None:
        self.part, self.dy_ptr = part, dy.data_ptr()

    def take(self, dy: torch.Tensor):
        part, ptr = self.part, self.dy_ptr
        self.part = self.dy_ptr = None
        return part if part is not None and ptr == dy.data_ptr() else None


class ResidualLink:
    """Hand-off from a fused BN(+residual)+ReLU to the conv that forked its identity input.

    The residual's gradient is dy * relu'(out) — dy masked by the forward's 1-bit mask. Instead of
    the BN backward writing it out (a full tensor write + read), it hands (dy, mask) to the forking
    conv (ops/conv.py::_Conv1x1Fork), whose dgrad epilogue adds dy where the mask bit is set. Valid
    only when the residual tensor is that fork's identity output (checked at forward time)."""

    __slots__ = ("dy", "mask")

    def __init__(self):
        self.dy = self.mask = None


class PendingApply:
    """A BN(+residual)+ReLU output whose apply pass was deferred to its consumer.

    The block-final BN of a bottleneck finalizes its statistics but does not write its output ``y``: the next
    block's conv1 GEMM (ops/conv.py::_Conv1x1Fork, csrc/kernels/gemm_apply.hip) reads the BN input ``x`` and the
    residual ``r`` itself, writes ``y`` and the ReLU mask while staging its operand, and multiplies -- the block
    output is never re-read. Any other consumer calls :func:`ensure` first (one apply pass, as without the
    deferral). Deferral only happens inside :func:`deferral_scope` (ResNet.forward), whose exit materialises
    whatever is still pending, so no code outside the model's own forward can see an unwritten output."""

    __slots__ = ("x", "r", "ws", "wsd", "y", "mask")

    def __init__(self, x, r, ws, wsd, y, mask):
        self.x, self.r, self.ws, self.wsd, self.y, self.mask = x, r, ws, wsd, y, mask

    def materialise(self) -> None:
        if self.y is not None:
            _ext.require().bn_apply_deferred(self.x, self.r, self.ws, self.wsd, self.y, self.mask)
            CALLS["materialised"] += 1
        self.clear()

    def clear(self) -> None:
        if self.y is not None:
            self.y._dla_pending = None
        self.x = self.r = self.ws = self.wsd = self.y = self.mask = None


CALLS = {"deferred": 0, "fused": 0, "materialised": 0}
_SCOPE: list = []  # open deferral scopes, each the list of the outputs it deferred


def pending_of(t):
    """The PendingApply of a deferred, not yet written BN output (None for any other tensor)."""
    p = getattr(t, "_dla_pending", None) if t is not None else None
    return p if p is not None and p.y is not None else None


def ensure(t):
    """Write a deferred BN output now (a no-op for every other tensor); returns ``t``."""
    p = pending_of(t)
    if p is not None:
        p.materialise()
    return t


class deferral_scope:
    """Context in which the bottleneck blocks may defer their final apply pass (DLA_DEFER_APPLY)."""

    def __enter__(self):
        _SCOPE.append([])
        return self

    def __exit__(self, *exc):
        for p in _SCOPE.pop():
            p.materialise()
        return False


def deferral_active() -> bool:
    return bool(_SCOPE) and knobs.flag("DEFER_APPLY")


def _defer_record(y, p) -> None:
    y._dla_pending = p
    _SCOPE[-1].append(p)
    CALLS["deferred"] += 1


_HANDOFF: list = [None]  # a deferring forward's PendingApply, picked up by its wrapper


def fork_link_of(t):
    return getattr(t, "_dla_fork", None) if t is not None else None


def bn_link_of(t: torch.Tensor):
    """The BNLink attached to a fused-BN output (None for any other tensor)."""
    return getattr(t, "_dla_bn", None)


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, training, momentum, eps, relu, stats,
                rlink=None, dlink=None, defer=False):
        C = _ext.require()
        y, ws, mask = C.bn_act_fwd(x, residual, weight, bias, running_mean, running_var, training, momentum, eps,
                                   relu, stats, None, 0, defer)
        if defer:  # y and mask are written by the consumer (PendingApply)
            _HANDOFF[0] = PendingApply(x, residual, ws, None, y, mask)
        ctx.has_res = residual is not None
        ctx.training = training
        ctx.rlink = rlink if (rlink is not None and residual is not None and training) else None
        # ReLU branch for backward: recomputed from x (ReLU right after BN) or the forward's 1-bit
        # mask (ReLU after the residual add) -- the output y is never re-read.
        ctx.mask_mode = MASK_NONE if not relu else (MASK_BITS if ctx.has_res else MASK_RECOMPUTE)
        m = mask if mask is not None and mask.numel() else None
        ctx.save_for_backward(x, ws, weight, m)
        ctx.link = BNLink(x, ws, m, ctx.mask_mode) if training and x.dtype == torch.bfloat16 else None
        # the producing 1x1 conv (the block's conv3) applies this BN's backward itself (ops/conv.py DualBNLink):
        # a bit-mask ReLU after the residual add, the residual gradient handed to the fork; bf16
        ok = (dlink is not None and x.dtype == torch.bfloat16 and ctx.mask_mode == MASK_BITS
              and ctx.rlink is not None and m is not None and dlink.claim())
        ctx.dlink = dlink if ok else None
        return y

    @staticmethod
    def backward(ctx, dy):
        if not ctx.training:
            raise RuntimeError("fused BN backward in eval mode is not supported; use the torch backend")
        x, ws, weight, mask = ctx.saved_tensors
        C = _ext.require()
        ext = ctx.link.take(dy) if ctx.link is not None else None
        rl = ctx.rlink
        if ctx.dlink is not None and ctx.dlink.can_park(x):
            # reduction + finalize only; the conv backward applies (dy, x, mask, ws) in its own kernel
            dy = dy.contiguous(memory_format=torch.channels_last)
            _, _, dg, db = C.bn_act_bwd(dy, None, mask, x, ws, weight, ctx.mask_mode, False, ext, False)
            dx = ctx.dlink.park(dy, x, ws, mask, weight, ctx.mask_mode)
            if rl is not None:
                rl.dy, rl.mask = dy, mask
            need = ctx.needs_input_grad
            return (dx, dg if need[1] else None, db if need[2] else None, None,
                    None, None, None, None, None, None, None, None, None, None)
        dx, dres, dg, db = C.bn_act_bwd(dy, None, mask, x, ws, weight, ctx.mask_mode, ctx.has_res and rl is None, ext)
        if rl is not None:  # the forking conv adds dy (masked) in its dgrad epilogue
            rl.dy = dy.contiguous(memory_format=torch.channels_last) if dy.dim() == 4 else dy.contiguous()
            rl.mask = mask if ctx.mask_mode == MASK_BITS else None
            dres = None
        need = ctx.needs_input_grad
        return (dx, dg if need[1] else None, db if need[2] else None, dres if ctx.has_res else None,
                None, None, None, None, None, None, None, None, None, None)


class _BNDualAct(torch.autograd.Function):
    """Training-mode ``act(BN(x) + BN_d(xd))``: a residual block's main branch plus its downsample
    shortcut. One apply pass reads both pre-BN tensors (the shortcut BN's output is never written);
    backward: one reduce and one apply pass read dy (+ the 1-bit ReLU mask) once for both BNs and
    write dx and dxd (no materialised residual gradient)."""

    @staticmethod
    def forward(ctx, x, weight, bias, xd, weight_d, bias_d, rm, rv, rmd, rvd, momentum, momentum_d, eps, eps_d,
                relu, stats, stats_d, dlink=None, dlink_d=None, defer=False):
        C = _ext.require()
        y, ws, wsd, mask = C.bn_dual_fwd(x, xd, weight, bias, rm, rv, weight_d, bias_d, rmd, rvd, momentum,
                                         momentum_d, eps, eps_d, relu, stats, stats_d, defer)
        if defer:
            _HANDOFF[0] = PendingApply(x, xd, ws, wsd, y, mask)
        ctx.relu = relu
        ctx.save_for_backward(x, ws, weight, xd, wsd, weight_d, mask if relu else None)
        # both inputs come from 1x1 convs that can apply their BN's backward themselves (ops/conv.py DualBNLink)
        ctx.dlinks = (dlink, dlink_d) if (dlink is not None and dlink_d is not None and relu and mask is not None
                                           and mask.numel() and x.dtype == torch.bfloat16
                                           and not dlink.claimed and not dlink_d.claimed
                                           and dlink.claim() and dlink_d.claim()) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, ws, weight, xd, wsd, weight_d, mask = ctx.saved_tensors
        need = ctx.needs_input_grad
        if ctx.dlinks is not None and ctx.dlinks[0].can_park(x) and ctx.dlinks[1].can_park(xd):
            dy = dy.contiguous(memory_format=torch.channels_last)
            _, dg, db, _, dgd, dbd = _ext.require().bn_dual_bwd(dy, mask, x, ws, weight, xd, wsd, weight_d, False)
            dx = ctx.dlinks[0].park(dy, x, ws, mask, weight, MASK_BITS)
            dxd = ctx.dlinks[1].park(dy, xd, wsd, mask, weight_d, MASK_BITS)
        else:
            dx, dg, db, dxd, dgd, dbd = _ext.require().bn_dual_bwd(dy, mask, x, ws, weight, xd, wsd, weight_d)
        return (dx, dg if need[1] else None, db if need[2] else None, dxd, dgd if need[4] else None,
                dbd if need[5] else None) + (None,) * 14


def dual_supported(x: torch.Tensor, bn: nn.BatchNorm2d, xd: torch.Tensor, bnd: nn.BatchNorm2d) -> bool:
    return (bn.training and bnd.training and x.dtype == xd.dtype and x.shape == xd.shape
            and supported(x, bn, None) and supported(xd, bnd, None)
            and bn.momentum is not None and bnd.momentum is not None)


def _can_defer(x, relu: bool, *others) -> bool:
    return (relu and x.dtype == torch.bfloat16 and deferral_active() and torch.is_grad_enabled()
            and any(t is not None and t.requires_grad for t in (x,) + others))


def _apply_deferred(fn, *args):
    """Run a deferring autograd Function and attach its PendingApply to the output."""
    _HANDOFF[0] = None
    y = fn.apply(*args)
    p, _HANDOFF[0] = _HANDOFF[0], None
    if p is not None:
        _defer_record(y, p)
        p.y = y
    return y


def fused_bn_add_bn_act(x: torch.Tensor, bn: nn.BatchNorm2d, xd: torch.Tensor, bnd: nn.BatchNorm2d,
                        relu: bool = True, stats=None, stats_d=None, defer: bool = False) -> torch.Tensor:
    """``act(bn(x) + bnd(xd))`` (training mode); falls back to the two-step form when unsupported.
    ``defer``: the output may be left for its consumer to write (PendingApply; inside a deferral_scope)."""
    if not dual_supported(x, bn, xd, bnd):
        return fused_bn_act(x, bn, relu, fused_bn_act(xd, bnd, False, None, stats_d), stats)
    running = []
    for b in (bn, bnd):
        running += [b.running_mean, b.running_var] if b.track_running_stats else [None, None]
        if b.track_running_stats:
            _PENDING_COUNTERS.append(b.num_batches_tracked)
    if len(_PENDING_COUNTERS) >= 1024:
        flush_bn_counters()
    defer = defer and _can_defer(x, relu, xd, bn.weight, bnd.weight)
    return _apply_deferred(_BNDualAct, x, bn.weight, bn.bias, xd, bnd.weight, bnd.bias, *running, float(bn.momentum),
                           float(bnd.momentum), float(bn.eps), float(bnd.eps), relu, stats, stats_d,
                           getattr(x, "_dla_dual", None), getattr(xd, "_dla_dual", None), defer)


# num_batches_tracked increments are batched into one multi-tensor launch per forward instead of
# 53 one-element kernels (ResNet-50); flushed by the DP wrappers after the model forward.
_PENDING_COUNTERS: list = []


def flush_bn_counters() -> None:
    if _PENDING_COUNTERS:
        torch._foreach_add_(_PENDING_COUNTERS, 1)
        _PENDING_COUNTERS.clear()


def supported(x: torch.Tensor, bn: nn.BatchNorm2d, residual) -> bool:
    if not (x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0):
        return False
    if x.dtype not in (torch.bfloat16, torch.float32):
        return False
    if not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
        return False
    if residual is not None and (residual.dtype != x.dtype or residual.shape != x.shape
                                 or not residual.is_contiguous(memory_format=torch.channels_last)):
        return False
    if bn.training and bn.momentum is None:  # cumulative moving average: torch path
        return False
    if bn.weight is not None and bn.weight.dtype != torch.float32:
        return False
    return True


def fused_bn_act(x: torch.Tensor, bn: nn.BatchNorm2d, relu: bool = True, residual: torch.Tensor | None = None,
                 stats: torch.Tensor | None = None, defer: bool = False):
    """``stats``: optional [row_blocks, C, 2] (sum, sumsq) partials of ``x`` produced by the conv GEMM
    epilogue (training mode only) — the statistics pass over ``x`` is then skipped. ``defer``: with ReLU (and
    optionally a residual), the output may be left for its consumer to write (PendingApply; inside a
    deferral_scope)."""
    if not supported(x, bn, residual):
        y = bn(x)
        if residual is not None:
            y = y + residual
        return torch.relu(y) if relu else y
    if bn.training:
        training = True
        rm, rv = (bn.running_mean, bn.running_var) if bn.track_running_stats else (None, None)
        if bn.track_running_stats:
            _PENDING_COUNTERS.append(bn.num_batches_tracked)
            if len(_PENDING_COUNTERS) >= 1024:  # used without a DP wrapper: flush periodically
                flush_bn_counters()
    elif bn.track_running_stats:
        training, rm, rv = False, bn.running_mean, bn.running_var
    else:
        training, rm, rv = True, None, None
    rlink = fork_link_of(residual)
    if rlink is not None and residual.dtype != torch.bfloat16:  # the epilogue addend is bf16
        rlink = None
    dlink = getattr(x, "_dla_dual", None) if training else None
    defer = (defer and training and (residual is None or residual.dtype == x.dtype)
             and _can_defer(x, relu, residual, bn.weight))
    y = _apply_deferred(_BNAct, x, bn.weight, bn.bias, residual, rm, rv, training, float(bn.momentum or 0.0),
                        float(bn.eps), relu, stats if training else None, rlink, dlink, defer)
    if y.grad_fn is not None:
        link = getattr(y.grad_fn, "link", None)
        if link is not None:
            y._dla_bn = link
    return y


class _BNReluPool(torch.autograd.Function):
    """Stem BN(train) + ReLU + max-pool in one op (csrc/kernels/bn_act.hip): the full-resolution
    activation and its gradient are never materialised."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, k, s, p, stats=None, ceil=False,
                slink=None):
        C = _ext.require()
        y, ws, pos = C.bn_relu_maxpool_fwd(x, weight, bias, running_mean, running_var, momentum, eps, k, s, p,
                                           stats, ceil)
        ctx.save_for_backward(x, ws, weight, pos)
        ctx.geom = (k, s, p)
        # the producing stem conv applies this op's backward inside its weight gradient (ops/conv.py StemBNLink)
        from .conv import stem_bn_fusable

        ok = slink is not None and stem_bn_fusable(x, y.shape, k, s, p) and slink.claim()
        ctx.slink = slink if ok else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, ws, weight, pos = ctx.saved_tensors
        k, s, p = ctx.geom
        need = ctx.needs_input_grad
        C = _ext.require()
        if ctx.slink is not None and ctx.slink.can_park(x):
            # reduction + finalize only (ws then holds the backward coefficients); the stem weight gradient applies
            dy = dy.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
            _, dg, db = C.bn_relu_maxpool_bwd(dy, pos, x, ws, weight, k, s, p, want_dx=False)
            dx = ctx.slink.park(dy, pos, x, ws, weight, ctx.geom)
        else:
            dx, dg, db = C.bn_relu_maxpool_bwd(dy, pos, x, ws, weight, k, s, p)
        return (dx, dg if need[1] else None, db if need[2] else None) + (None,) * 10


def fused_bn_relu_maxpool(x: torch.Tensor, bn: nn.BatchNorm2d, pool: nn.MaxPool2d, stats=None):
    """``pool(relu(bn(x)))`` with the fused kernels when they apply (training-mode BN with running
    stats or none, bf16 channels_last, square window, no dilation/indices; floor or ceil mode); otherwise the
    separate fused BN+ReLU and max-pool ops. ``stats``: the producing conv's [rows, C, 2] (sum, sumsq)
    partials of ``x`` (the statistics pass over x is skipped)."""
    from .pool import _pair_same, max_pool2d

    k, s, p = _pair_same(pool.kernel_size), _pair_same(pool.stride or pool.kernel_size), _pair_same(pool.padding)
    ok = (bn.training and bn.momentum is not None and x.dtype == torch.bfloat16 and supported(x, bn, None)
          and None not in (k, s, p) and _pair_same(pool.dilation) == 1
          and not pool.return_indices and 1 <= k <= 15 and 2 * p <= k
          and _limits.pixels_ok(x.numel() // x.shape[1], "stem BN+ReLU+max-pool"))
    if not ok:
        return max_pool2d(fused_bn_act(x, bn, True, None, stats), pool.kernel_size, pool.stride, pool.padding,
                          pool.dilation, pool.ceil_mode)
    rm, rv = (bn.running_mean, bn.running_var) if bn.track_running_stats else (None, None)
    if bn.track_running_stats:
        _PENDING_COUNTERS.append(bn.num_batches_tracked)
    return _BNReluPool.apply(x, bn.weight, bn.bias, rm, rv, float(bn.momentum), float(bn.eps), k, s, p, stats,
                             bool(pool.ceil_mode), getattr(x, "_dla_stem", None))
