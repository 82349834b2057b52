"""Native Inception block (GoogLeNet, torchvision v0.6 layout) without the concatenation copy and
without the autograd sum of the block input's four gradients.

A stock Inception block runs, besides its convolutions:

* ``torch.cat`` of the four branch outputs, which copies the whole block output once;
* in backward, ``cat``'s gradient slices, which each BN backward copies into a contiguous dy;
* three elementwise adds, which sum the gradients of the four consumers of the block input
  (autograd accumulation). In the round-2 GoogLeNet profile these were ``CatArrayBatchedCopy``,
  ``elementwise_kernel`` and ``CUDAFunctor_add`` (profiles/googlenet_bs128_r2k_ksum.md).

Here autograd nodes replace them:

* :class:`_InceptionFanIn` holds every consumer of ``x``: the three 1x1 convs (branch 1 and the
  branch 2/3 reductions, MFMA GEMMs with a BN-statistics epilogue) and branch 4's 3x3/s1 ceil-mode
  max-pool. Its backward starts from the max-pool gradient and adds each conv's data gradient to
  it through the dgrad GEMM's addend epilogue (``dX = dY_k W_k + dX``), so x's gradient is
  written once per consumer with no separate sum kernels.
* :class:`_InceptionFanInCat` (default) goes further: the three 1x1 convs are ONE GEMM over their
  stacked weights, whose output channels are the three branches side by side (read in place by the
  grouped BN kernels through their row stride). Its backward is one dgrad GEMM over
  K = C1 + C2r + C3r, which sums x's three conv gradients inside the reduction, and one
  weight-gradient GEMM; the BN backward passes write the three dy straight into the channel slices
  of one shared buffer (:class:`_FanInGrad`), so nothing is concatenated. GoogLeNet bs128 went from
  18.4k to 20.6k img/s with it (profiles/r3y).
* :class:`_BNReluConcat` applies the four branch BatchNorm+ReLU passes straight into channel slices
  of one preallocated NHWC block output (row stride = total channels). Its backward reads each
  branch's dy in place from the concatenated gradient (strided loads in the BN backward passes).
  The four branches run as one group per pass (``bn_concat_fwd`` / ``bn_concat_bwd``: one
  finalize + one apply launch forward, one reduce + finalize + apply backward, instead of one chain
  per branch), which matters at the 14x14 / 7x7 shapes where each pass is a few-microsecond launch.

Reference: the block structure of torchvision's GoogLeNet v0.6, which the reference loads through
torch.hub (/root/reference/src/network.py:33-54).
"""
from __future__ import annotations

from .. import knobs
import os

import torch
import torch.nn as nn

from . import _ext

CL = torch.channels_last


def _rows(t: torch.Tensor) -> torch.Tensor:
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


class _InceptionFanIn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, w2, w3, k: int, s: int, p: int, ceil: bool):
        C = _ext.require()
        ctx.set_materialize_grads(False)
        n, cin, h, w = x.shape
        xr = _rows(x)
        outs, w2ds = [], []
        for wt in (w1, w2, w3):
            cout = wt.shape[0]
            wm = wt.reshape(cout, cin).to(torch.bfloat16).contiguous()
            y2, st = C.gemm_nt(xr, wm, True)
            ctx.mark_non_differentiable(st)
            outs += [y2.view(n, h, w, cout).permute(0, 3, 1, 2), st]
            w2ds.append(wm)
        yp, pos = C.maxpool_fwd(x, k, s, p, ceil, True)
        ctx.save_for_backward(x, *w2ds, pos)
        ctx.pool = (h, w, k, s, p)
        ctx.wmeta = [(wt.dtype, wt.shape, wt.stride()) for wt in (w1, w2, w3)]
        return (*outs, yp)

    @staticmethod
    def backward(ctx, dy1, _s1, dy2, _s2, dy3, _s3, dyp):
        C = _ext.require()
        x, w1, w2, w3, pos = ctx.saved_tensors
        n, cin, h, w = x.shape
        xr = _rows(x)
        H, W, k, s, p = ctx.pool
        dx = None
        if ctx.needs_input_grad[0] and dyp is not None:
            dx = C.maxpool_bwd(dyp.contiguous(memory_format=CL), pos, H, W, k, s, p)
        dws = [None, None, None]
        # branch 3 first, then 2, then 1: each data gradient is accumulated into dx by the GEMM epilogue
        for i, (dy, wm) in reversed(list(enumerate(((dy1, w1), (dy2, w2), (dy3, w3))))):
            if dy is None:
                continue
            dy = dy.contiguous(memory_format=CL)
            if dy.dtype != torch.bfloat16:
                dy = dy.to(torch.bfloat16)
            d2 = _rows(dy)
            if ctx.needs_input_grad[1 + i]:
                dt, shape, stride = ctx.wmeta[i]
                odt = dt if dt in (torch.float32, torch.bfloat16) else torch.float32
                dws[i] = C.gemm_tn(d2, xr, odt, 1.0).to(dt).as_strided(shape, stride)
            if ctx.needs_input_grad[0]:
                add = None if dx is None else _rows(dx.contiguous(memory_format=CL))
                dx2, _ = C.gemm_nt(d2, wm, False, add, True)
                dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
        return dx, dws[0], dws[1], dws[2], None, None, None, None


class _FanInGrad:
    """The fused fan-in's gradient buffer [N, C1 + C2r + C3r, H, W]: the BN backward passes of
    branch 1 and of the two reductions write their dx straight into its channel slices, so the
    fan-in backward finds the three gradients already side by side (no concatenation)."""

    __slots__ = ("shape", "buf")

    def __init__(self, shape):
        self.shape = shape
        self.buf = None

    def slice(self, like: torch.Tensor, off: int, c: int) -> torch.Tensor:
        if self.buf is None:
            self.buf = torch.empty(self.shape, dtype=torch.bfloat16, device=like.device, memory_format=CL)
        return self.buf[:, off:off + c]

    def holds(self, dys) -> bool:
        """The gradients are this buffer's consecutive channel slices (as the BN passes wrote them)."""
        if self.buf is None or any(d is None for d in dys):
            return False
        off, base, es = 0, self.buf.data_ptr(), self.buf.element_size()
        for d in dys:
            if d.data_ptr() != base + off * es or d.stride() != self.buf.stride() or d.dtype != self.buf.dtype:
                return False
            off += d.shape[1]
        return off == self.shape[1]


class _InceptionFanInCat(torch.autograd.Function):
    """The three 1x1 convs of an Inception block on one input as ONE MFMA GEMM over their stacked
    weights [C1 + C2r + C3r, Cin] (BN statistics of all output channels in its epilogue), plus the
    branch-4 max-pool. The outputs are channel slices of the GEMM result, which the grouped BN
    kernels read with their row stride. Backward: one dgrad GEMM over K = C1 + C2r + C3r (the sum
    of x's three conv gradients falls out of the reduction; the max-pool gradient is its epilogue
    addend) and one split-K weight-gradient GEMM, sliced into the three weight gradients."""

    @staticmethod
    def forward(ctx, x, w1, w2, w3, k: int, s: int, p: int, ceil: bool, slot: _FanInGrad):
        C = _ext.require()
        ctx.set_materialize_grads(False)
        n, cin, h, w = x.shape
        cs = [wt.shape[0] for wt in (w1, w2, w3)]
        wcat = torch.cat([wt.reshape(c, cin) for wt, c in zip((w1, w2, w3), cs)]).to(torch.bfloat16)
        ycat, scat = C.gemm_nt(_rows(x), wcat, True)
        y4 = ycat.view(n, h, w, sum(cs)).permute(0, 3, 1, 2)
        ctx.mark_non_differentiable(scat)
        outs, off = [], 0
        for c in cs:
            outs += [y4[:, off:off + c], scat[:, off:off + c]]
            off += c
        yp, pos = C.maxpool_fwd(x, k, s, p, ceil, True)
        ctx.save_for_backward(x, wcat, pos)
        ctx.pool = (h, w, k, s, p)
        ctx.cs = cs
        ctx.slot = slot
        ctx.wmeta = [(wt.dtype, wt.shape, wt.stride()) for wt in (w1, w2, w3)]
        return (*outs, yp)

    @staticmethod
    def backward(ctx, dy1, _s1, dy2, _s2, dy3, _s3, dyp):
        C = _ext.require()
        x, wcat, pos = ctx.saved_tensors
        n, cin, h, w = x.shape
        H, W, k, s, p = ctx.pool
        dys = (dy1, dy2, dy3)
        dx = None
        if ctx.needs_input_grad[0] and dyp is not None:
            dx = C.maxpool_bwd(dyp.contiguous(memory_format=CL), pos, H, W, k, s, p)
        if ctx.slot.holds(dys):
            dcat = ctx.slot.buf
        else:
            dcat = torch.cat([d if d is not None else x.new_zeros((n, c, h, w), dtype=torch.bfloat16)
                              for d, c in zip(dys, ctx.cs)], dim=1).to(torch.bfloat16).contiguous(memory_format=CL)
        ctx.slot.buf = None
        d2 = _rows(dcat)
        dws = [None, None, None]
        if any(ctx.needs_input_grad[1:4]):
            odt = ctx.wmeta[0][0] if ctx.wmeta[0][0] in (torch.float32, torch.bfloat16) else torch.float32
            gcat = C.gemm_tn(d2, _rows(x), odt, 1.0)
            off = 0
            for i, c in enumerate(ctx.cs):
                dt, shape, stride = ctx.wmeta[i]
                if ctx.needs_input_grad[1 + i]:
                    dws[i] = gcat[off:off + c].to(dt).as_strided(shape, stride)
                off += c
        if ctx.needs_input_grad[0]:
            add = None if dx is None else _rows(dx.contiguous(memory_format=CL))
            dx2, _ = C.gemm_nt(d2, wcat, False, add, True)
            dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
        return dx, dws[0], dws[1], dws[2], None, None, None, None, None


class _BNReluConcat(torch.autograd.Function):
    """act(BN_b(y_b)) for every branch b, written into channel slices of one NHWC output."""

    @staticmethod
    def forward(ctx, metas, dsl, *tensors):
        C = _ext.require()
        ys, gs, bs = tensors[0::3], tensors[1::3], tensors[2::3]
        n, _, h, w = ys[0].shape
        ctx.dsl = dsl
        ctot = sum(y.shape[1] for y in ys)
        out = torch.empty((n, ctot, h, w), dtype=ys[0].dtype, device=ys[0].device, memory_format=CL)
        ctx.grouped = _grouped_ok(ys, gs, bs, metas)
        if ctx.grouped:
            # one finalize + one apply launch for all branches (bn_act.hip, grouped kernels)
            wss = C.bn_concat_fwd(list(ys), list(gs), list(bs), [m[0] for m in metas], [m[1] for m in metas],
                                  [m[2] for m in metas], [m[3] for m in metas], [m[4] for m in metas], out)
        else:
            wss, off = [], 0
            ys = tuple(y.contiguous(memory_format=CL) for y in ys)
            for y, g, b, (rm, rv, mom, eps, st) in zip(ys, gs, bs, metas):
                st = st.contiguous() if st is not None else None
                _, ws, _ = C.bn_act_fwd(y, None, g, b, rm, rv, True, mom, eps, True, st, out, off)
                wss.append(ws)
                off += y.shape[1]
        ctx.save_for_backward(*ys, *gs, *wss)
        ctx.nb = len(ys)
        return out

    @staticmethod
    def backward(ctx, dout):
        C = _ext.require()
        nb = ctx.nb
        saved = ctx.saved_tensors
        ys, gs, wss = saved[:nb], saved[nb:2 * nb], saved[2 * nb:]
        dout = dout.contiguous(memory_format=CL)
        if dout.dtype != ys[0].dtype:
            dout = dout.to(ys[0].dtype)
        if ctx.grouped:
            return (None, None, *C.bn_concat_bwd(dout, list(ys), list(gs), list(wss), _dx_out(ctx.dsl, ys)))
        grads, off = [None, None], 0
        for y, g, ws in zip(ys, gs, wss):
            c = y.shape[1]
            dx, _, dg, db = C.bn_act_bwd(dout[:, off:off + c], None, None, y, ws, g, 1, False, None)
            grads += [dx, dg, db]
            off += c
        return tuple(grads)


class _BNReluGroup(torch.autograd.Function):
    """act(BN_b(y_b)) for same-size tensors that each keep their own output (the 1x1 reductions of
    branches 2 and 3), one launch per pass. Each output carries a BNLink, so the 3x3 conv consuming
    it still produces this BN's backward partials in its dgrad epilogue; with all of them present
    the grouped backward is one finalize + one apply launch."""

    @staticmethod
    def forward(ctx, metas, dsl, *tensors):
        from .bn_act import BNLink, MASK_RECOMPUTE

        C = _ext.require()
        ys, gs, bs = tensors[0::3], tensors[1::3], tensors[2::3]
        n = len(ys)
        res = C.bn_group_fwd(list(ys), list(gs), list(bs), [m[0] for m in metas], [m[1] for m in metas],
                             [m[2] for m in metas], [m[3] for m in metas], [m[4] for m in metas])
        outs, wss = res[:n], res[n:]
        ctx.save_for_backward(*ys, *gs, *wss)
        ctx.nb = n
        ctx.dsl = dsl
        # the consumer conv's dgrad epilogue reads the BN input in place (a slice: its row stride)
        ctx.links = [BNLink(y, ws, None, MASK_RECOMPUTE) for y, ws in zip(ys, wss)]
        return tuple(outs)

    @staticmethod
    def backward(ctx, *douts):
        C = _ext.require()
        nb = ctx.nb
        saved = ctx.saved_tensors
        ys, gs, wss = saved[:nb], saved[nb:2 * nb], saved[2 * nb:]
        dys = []
        for d, y in zip(douts, ys):
            d = d.contiguous(memory_format=CL)
            dys.append(d if d.dtype == y.dtype else d.to(y.dtype))
        exts = [link.take(d) if link is not None else None for link, d in zip(ctx.links, dys)]
        if any(e is None for e in exts):
            exts = []
        return (None, None, *C.bn_group_bwd(dys, list(ys), list(gs), list(wss), exts, _dx_out(ctx.dsl, ys)))


def _dx_out(dsl, ys):
    """Per-branch dx destinations: a slice of the fan-in's gradient buffer where one is given."""
    if dsl is None or all(d is None for d in dsl):
        return []
    return [d[0].slice(y, d[1], y.shape[1]) if d is not None
            else torch.empty(y.shape, dtype=y.dtype, device=y.device, memory_format=CL) for d, y in zip(dsl, ys)]


# knobs BN_GROUPED=0 keeps one BN launch chain per branch; FANIN_CAT=0 keeps three fan-in GEMMs (A/B runs)
_GROUPED = knobs.get("BN_GROUPED") != "0"
_FANIN_CAT = knobs.get("FANIN_CAT") != "0"


def _grouped_ok(ys, gs, bs, metas) -> bool:
    """The grouped kernels take bf16 branches with epilogue statistics and fp32 BN parameters."""
    if not _GROUPED or not 1 <= len(ys) <= 4:
        return False
    for y, g, b, (rm, rv, _, _, st) in zip(ys, gs, bs, metas):
        if st is None or y.dtype != torch.bfloat16 or rm is None or rv is None:
            return False
        if not all(t.dtype == torch.float32 and t.is_contiguous() for t in (g, b, rm, rv)):
            return False
    return True


def _bn_ok(bn: nn.BatchNorm2d) -> bool:
    return (bn.training and bn.momentum is not None and bn.track_running_stats and bn.affine
            and bn.weight.dtype == torch.float32)


def supported(block, x: torch.Tensor) -> bool:
    """The fused path: training-mode BNs with running statistics, bf16 channels_last input, native
    1x1 / 3x3 convs for every branch conv, channel counts % 8."""
    from . import conv as nconv

    if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=CL)
            and x.shape[1] % 8 == 0 and x.data_ptr() % 16 == 0):
        return False
    pool = block.branch4[0]
    if not isinstance(pool, nn.MaxPool2d) or pool.return_indices or pool.dilation not in (1, (1, 1)):
        return False
    bcs = [block.branch1, block.branch2[0], block.branch2[1], block.branch3[0], block.branch3[1], block.branch4[1]]
    if not all(_bn_ok(b.bn) and b.conv.out_channels % 8 == 0 for b in bcs):
        return False
    return all(nconv.supported(x, b.conv) and b.conv.stride == (1, 1)
               for b in (block.branch1, block.branch2[0], block.branch3[0]))


def inception_forward(block, x: torch.Tensor) -> torch.Tensor:
    """The block's output on the fused path (:func:`supported` must hold)."""
    from . import bn_act
    from .conv import conv1x1, conv3x3, supported as sup1, supported3x3

    pool = block.branch4[0]

    def pair(v):
        return v[0] if isinstance(v, (tuple, list)) else v

    k, s, p = pair(pool.kernel_size), pair(pool.stride or pool.kernel_size), pair(pool.padding)
    ws3 = (block.branch1.conv.weight, block.branch2[0].conv.weight, block.branch3[0].conv.weight)
    slot = None
    if _FANIN_CAT and _GROUPED:
        cs = [wt.shape[0] for wt in ws3]
        slot = _FanInGrad((x.shape[0], sum(cs), x.shape[2], x.shape[3]))
        y1, s1, y2r, s2r, y3r, s3r, yp = _InceptionFanInCat.apply(x, *ws3, k, s, p, bool(pool.ceil_mode), slot)
        dsl1, dslr = (slot, 0), ((slot, cs[0]), (slot, cs[0] + cs[1]))
    else:
        y1, s1, y2r, s2r, y3r, s3r, yp = _InceptionFanIn.apply(x, *ws3, k, s, p, bool(pool.ceil_mode))
        dsl1, dslr = None, (None, None)
    outs = [(y1, block.branch1.bn, s1)]
    reds = ((y2r, s2r, block.branch2), (y3r, s3r, block.branch3))
    rbns = [cb[0].bn for _, _, cb in reds]
    rmetas = tuple((bn.running_mean, bn.running_var, float(bn.momentum), float(bn.eps), st)
                   for bn, (_, st, _) in zip(rbns, reds))
    rys = [r for r, _, _ in reds]
    if _grouped_ok(rys, [bn.weight for bn in rbns], [bn.bias for bn in rbns], rmetas):
        rt = []
        for y, bn in zip(rys, rbns):
            rt += [y, bn.weight, bn.bias]
            bn_act._PENDING_COUNTERS.append(bn.num_batches_tracked)
        acts = _BNReluGroup.apply(rmetas, dslr, *rt)
        for i, a in enumerate(acts):
            if a.grad_fn is not None and a.grad_fn.links[i] is not None:
                a._dla_bn = a.grad_fn.links[i]
    else:
        acts = [bn_act.fused_bn_act(red.contiguous(memory_format=CL), bn, True, None,
                                    stats.contiguous() if stats is not None else None)
                for (red, stats, _), bn in zip(reds, rbns)]
    for a, (_, _, conv_bn) in zip(acts, reds):
        c = conv_bn[1].conv
        if supported3x3(a, c):
            y, st = conv3x3(a, c, want_stats=True)
        elif sup1(a, c):
            y, st = conv1x1(a, c, want_stats=True)
        else:
            y, st = c(a), None
        outs.append((y, conv_bn[1].bn, st))
    c4 = block.branch4[1].conv
    y4, st4 = conv1x1(yp, c4, want_stats=True) if sup1(yp, c4) else (c4(yp), None)
    outs.append((y4, block.branch4[1].bn, st4))
    metas, tensors = [], []
    for i, (y, bn, st) in enumerate(outs):
        if y.dtype != torch.bfloat16 or (i > 0 and not y.is_contiguous(memory_format=CL)):
            y = y.contiguous(memory_format=CL).to(torch.bfloat16)
        metas.append((bn.running_mean, bn.running_var, float(bn.momentum), float(bn.eps), st))
        tensors += [y, bn.weight, bn.bias]
        bn_act._PENDING_COUNTERS.append(bn.num_batches_tracked)
    if len(bn_act._PENDING_COUNTERS) >= 1024:  # used without a DP wrapper: flush periodically
        bn_act.flush_bn_counters()
    return _BNReluConcat.apply(tuple(metas), (dsl1, None, None, None), *tensors)
