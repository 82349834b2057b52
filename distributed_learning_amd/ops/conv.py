"""1x1 convolutions as native bf16 MFMA GEMMs (csrc/kernels/gemm.hip) on channels_last activations.

For NHWC activations a 1x1 convolution is a GEMM over M = N*H*W rows, so ResNet-50's 36 pointwise
convs (plus their backward) run on the framework's own MFMA kernels instead of MIOpen:

* forward  ``Y = X W^T``   (``gemm_nt``, optionally emitting the BatchNorm column statistics of Y
  from the epilogue, so the following fused BN skips its statistics pass),
* dgrad    ``dX = dY W``   (``gemm_nt`` reading W k-major through transposing LDS reads),
* wgrad    ``dW = dY^T X`` (``gemm_tn``, split-K over the N*H*W rows).

Stride-2 1x1 convs (ResNet downsample) subsample the input first. Anything else (non-bf16 inputs,
odd channel counts, grouped/dilated/padded convs) uses ``F.conv2d``.
"""
from __future__ import annotations

from .. import knobs
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext
from . import limits as _limits
from .bn_act import ResidualLink
from .bn_act import pending_of
from .bn_act import bn_link_of as _bn_link_of

# Fuse the backward reduction of a producing BatchNorm into this conv's dgrad epilogue (BNLink).
# "0" (default) off, "1" every dgrad, "stream" only the short-K 1x1 data gradients the persistent
# streaming kernel serves (gemm_stream.hip kBM variants: the epilogue's x loads overlap the next tile's
# rows in flight). Measured on MI355X: round 2, reading the BN input in the tile kernels' epilogue cost
# about what the standalone reduction pass saves (+0.3 ms/step at bs512); round 4 at bs1280 "1" is
# 3.8 % slower (92.0 vs 88.5 ms/step, profiles/r4/g02/).
BN_EPILOGUE = knobs.get("BN_EPILOGUE")


def _epi_ok(M: int, N: int, K: int, add: bool) -> bool:
    """Use the BN-epilogue data gradient for this k-major 1x1 dgrad (output [M, N], K = its input channels)."""
    if BN_EPILOGUE == "1":
        return True
    if BN_EPILOGUE != "stream":
        return False
    return _ext.require().gemm_stream_rows(M, N, K, K, N, True, add, True) > 0

# Native conv dispatches by kind ("1x1", "1x1_fork", "3x3", "stem"): lets a test assert that a step
# (e.g. the reference-compatible CLI's) ran the framework's kernels rather than MIOpen.
import collections as _collections  # noqa: E402

CALLS = _collections.Counter()


def bn_link_of(x):
    return _bn_link_of(x) if BN_EPILOGUE != "0" else None


def supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and conv.kernel_size == (1, 1)
            and conv.padding in ((0, 0), 0) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.stride in ((1, 1), (2, 2)) and conv.in_channels % 8 == 0 and conv.out_channels % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and _limits.span_ok(max(x.numel(), x.numel() // x.shape[1] // conv.stride[0] ** 2 * conv.out_channels)
                                * x.element_size(), "conv1x1 operand"))


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> [N*H*W, C] view."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _as_param_layout(dw2: torch.Tensor, shape, stride) -> torch.Tensor:
    """[Cout, Cin] weight gradient viewed with the parameter's own strides: a 1x1 conv weight is the
    same memory in contiguous and channels_last form, but a stride mismatch would make autograd /
    the DP gradient gathering copy it."""
    return dw2.as_strided(shape, stride)


# Weight gradients of launches that under-fill the chip (ResNet-50 stages 2-4: M = N*H*W <= 200704
# rows gives <= 1568 128x128 tiles, 1-3 waves of 2 blocks on 256 CUs with a ragged last wave) can run
# on a side stream, concurrently with the data gradient of the same conv; the compute stream joins
# the side stream before the next op (event wait, also inside HIP-graph capture). 0 disables.
# Off by default: measured on MI355X (scripts/wgrad_overlap_sweep.sh, ResNet-50 bs256) the step took
# 22.75 ms without, 23.36 / 23.51 / 23.33 ms with the overlap up to 50176 / 200704 / 802816 rows —
# the concurrent GEMMs contend for the same L2 / Infinity Cache and CUs rather than filling gaps.
WGRAD_OVERLAP_MAX_ROWS = 0
_SIDE_STREAMS: dict = {}


class _SideWork:
    """``fn()`` on the device's side stream (after the current stream's pending work) when
    ``rows`` is small enough, else inline; ``result()`` joins and returns its tensor."""

    def __init__(self, fn, rows: int, device: torch.device):
        self.side = None
        if WGRAD_OVERLAP_MAX_ROWS and rows <= WGRAD_OVERLAP_MAX_ROWS:
            cur = torch.cuda.current_stream(device)
            side = _SIDE_STREAMS.get(device)
            if side is None:
                side = _SIDE_STREAMS[device] = torch.cuda.Stream(device=device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self.out = fn()
            self.side, self.cur = side, cur
        else:
            self.out = fn()

    def result(self):
        if self.side is not None:
            self.cur.wait_stream(self.side)
            if self.out is not None:
                self.out.record_stream(self.cur)  # allocated on the side stream, used on the current one
        return self.out


# Late-joined weight gradients (DLA_WGRAD_DEFER = "3x3" | "auto" | "all" | "0"): a conv's weight gradient is issued
# on the side stream right AFTER its data gradient, so it runs alongside the memory-bound BatchNorm-backward
# passes and the next data gradients of the compute stream instead of between them. The compute stream
# joins the side stream at the end of the backward pass (autograd queue_callback; DLA_WGRAD_JOIN=end) or
# already at the next conv backward (=conv). Collective executors make their stream wait for it (join_into) before
# they read a gradient. Only for parameters without an existing .grad: AccumulateGrad would add into one
# on the compute stream before the join. Default "3x3": ResNet-50 bs1024 on one MI355X, same box,
# interleaved (profiles/r3/g18_g19_wgrad_defer.md): 72.58-72.77 ms/step vs 73.67-73.80 inline; deferring
# the 1x1 weight gradients too ("all") gains nothing (they stream like the BN passes they would overlap),
# and at bs1280 it stalls: p50 89.7 ms but single steps of 1.4-6.9 s (profiles/r3/g47_defer_batch_ab.md),
# from the caching allocator's cross-stream frees (record_stream) forcing synchronising retries near the
# memory ceiling. Keep "all" for tests and small batches.
#
# Who may see a deferred gradient before the join: AccumulateGrad stores it (no read), the end-of-backward
# callback joins before backward() returns, GradSync's executors join it into their stream before they read,
# FusedSGD.step joins as a safety net. Consumers that read gradients INSIDE backward without joining
# (torch DDP's reducer hooks) must call block_deferral() for their lifetime: TorchDDP does.
WGRAD_DEFER = knobs.get("WGRAD_DEFER")
WGRAD_JOIN = knobs.get("WGRAD_JOIN")
_DEFER_PENDING: dict = {}  # device -> the side stream holds work the compute stream has not joined yet
_DEFERRED_W: dict = {}  # device -> ids of the weights deferred in the running backward (each at most once)
_DEFER_BLOCKS = [0]  # > 0: some live consumer reads gradients inside backward without joining


def block_deferral() -> None:
    _DEFER_BLOCKS[0] += 1


def unblock_deferral() -> None:
    _DEFER_BLOCKS[0] = max(0, _DEFER_BLOCKS[0] - 1)


def _side_stream(device: torch.device) -> torch.cuda.Stream:
    side = _SIDE_STREAMS.get(device)
    if side is None:
        side = _SIDE_STREAMS[device] = torch.cuda.Stream(device=device)
    return side


def side_pending(device: torch.device) -> bool:
    return bool(_DEFER_PENDING.get(device))


def join_into(stream, device: torch.device) -> None:
    """Make ``stream`` wait for the deferred weight gradients issued so far on ``device``."""
    if _DEFER_PENDING.get(device):
        stream.wait_stream(_SIDE_STREAMS[device])


def join_compute(device: torch.device) -> None:
    if _DEFER_PENDING.get(device):
        torch.cuda.current_stream(device).wait_stream(_SIDE_STREAMS[device])
        _DEFER_PENDING[device] = False
    _DEFERRED_W.pop(device, None)


def join_all_devices() -> None:
    """Safety net for optimizers: join every device's pending late weight gradients (a backward that
    raised drops its end-of-backward callback)."""
    for dev, pending in list(_DEFER_PENDING.items()):
        if pending:
            join_compute(dev)


# "auto": the 3x3 weight gradients plus the 1x1 ones whose arithmetic intensity Cin*Cout/(Cin+Cout)
# (FLOP per byte of the two streamed operands) is at least WGRAD_DEFER_MIN_AI: those are the MFMA-bound
# ones that complement the memory-bound passes they overlap; the short-channel 1x1 ones stream operands
# like the BatchNorm passes and only contend with them.
WGRAD_DEFER_MIN_AI = float(knobs.get("WGRAD_DEFER_MIN_AI"))


def _wants_defer(kind: str, ctx, cin: int = 0, cout: int = 0) -> bool:
    if not ctx.needs_input_grad[1]:
        return False
    if WGRAD_DEFER == "auto":
        return kind == "3x3" or cin * cout >= WGRAD_DEFER_MIN_AI * (cin + cout)
    return WGRAD_DEFER in ("all", kind)


def _wgrad_after_dgrad(fn, ctx, keep, device: torch.device):
    """The weight gradient issued after the data gradient: on the side stream (after everything the
    compute stream has issued so far) when the parameter has no .grad yet, else inline."""
    weight = getattr(ctx, "weight_leaf", None)
    # inside HIP-graph capture (GoogLeNet bs128 --graph on: 19.8k vs 20.7k img/s with the fork / join
    # nodes, profiles/r3/g38_other_models_ab.txt) the weight gradient stays on the captured stream
    if (weight is None or weight.grad is not None or _DEFER_BLOCKS[0] or
            torch.cuda.is_current_stream_capturing()):
        return fn()
    seen = _DEFERRED_W.setdefault(device, set())
    if id(weight) in seen:
        # a weight used twice in one graph: autograd sums its two gradients on the compute stream before any
        # join, so the first (deferred) one must be complete first and this one runs inline
        join_compute(device)
        return fn()
    seen.add(id(weight))
    cur = torch.cuda.current_stream(device)
    side = _side_stream(device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        out = fn()
    for t in keep:  # inputs the compute stream may free before the side stream has read them
        t.record_stream(side)
    out.record_stream(cur)
    _DEFER_PENDING[device] = True
    # the end-of-backward join (also after the last conv in "conv" mode), queued on THIS graph task by every
    # deferral: a backward that raises drops its callbacks with it instead of leaving a sticky "queued" flag
    # that would skip the join of every later backward; the extra callbacks find nothing pending
    torch.autograd.Variable._execution_engine.queue_callback(lambda: join_compute(device))
    return out


# Both gradients of the stride-1 1x1 convs whose shape gemm_dual.hip serves (stage 1: 64 -> 256 channels) in
# one pass over dy instead of a data-gradient GEMM and a weight-gradient GEMM that each stream it from HBM.
DUAL_1X1 = True
DUAL_1X1_MAX_COUT = 512  # A/B: 256 keeps it to stage 1
# ... and, where its output feeds a BN(+residual)+ReLU with a bit mask (the block's last BN), that BN's
# backward apply inside the same kernel: the BN backward stops after its reduction and hands (dy, y, mask,
# coefficients) over; dY never reaches HBM (gemm_dual.hip kBN).
DUAL_BN = True
# (The block's first BN(+ReLU) inside its conv1 (fork) backward was built and measured slower -- 32-row tiles of
# 64-128 channels: 88.1 vs 84.2 ms/step, profiles/r4/g11; 64-row tiles: 87.2 vs 84.5, g12 -- and removed.)


class DualBNLink:
    """Hand-off from the BN(+residual)+ReLU consuming a 1x1 conv's output to that conv's backward.

    The BN backward returns a zero-stride placeholder as its input gradient and parks its incoming gradient,
    input, mask and finalized coefficients here; the conv backward recognises the placeholder and runs the
    one-pass kernel with the BN apply fused. If autograd summed the placeholder with other gradients of the
    conv output (more consumers), the conv backward materialises the BN's gradient and adds it.

    Guards: one link serves ONE BN -- the first BN to claim() it in its forward; a second BN on
    the same conv output runs the normal path, so no parked gradient can be overwritten. And park()
    is refused (can_park False: the BN computes its input gradient itself) when anything else observes the
    conv output's gradient -- a tensor hook or retain_grad() on it -- since that observer would see the
    placeholder's zeros. Not detectable from inside the backward: ``torch.autograd.grad(..., inputs=[y])``
    with the conv output itself as an input (the engine captures the placeholder; its introspection,
    ``torch._C._will_engine_execute_node``, reports the producing node as executed either way). Code that
    differentiates with respect to a conv output turns the hand-offs off (``DUAL_BN`` / ``STEM_BN`` here,
    ``DLA_STEM_BN=0``) or registers a hook on it."""

    __slots__ = ("ph", "dout", "ybn", "ws", "mask", "weight", "mode", "claimed")

    def __init__(self):
        self.ph = self.dout = self.ybn = self.ws = self.mask = self.weight = self.mode = None
        self.claimed = False

    def claim(self) -> bool:
        if self.claimed:
            return False
        self.claimed = True
        return True

    @staticmethod
    def observed(y) -> bool:
        return bool(y.retains_grad or getattr(y, "_backward_hooks", None))

    def can_park(self, y) -> bool:
        return self.ph is None and not self.observed(y)

    def park(self, dout, ybn, ws, mask, weight, mode=2):
        assert self.can_park(ybn), "DualBNLink.park: check can_park first"
        self.dout, self.ybn, self.ws, self.mask, self.weight, self.mode = dout, ybn, ws, mask, weight, mode
        self.ph = torch.zeros((), dtype=ybn.dtype, device=ybn.device).expand(ybn.shape)
        return self.ph

    def take(self):
        out = (self.ph, self.dout, self.ybn, self.ws, self.mask, self.weight, self.mode)
        self.ph = self.dout = self.ybn = self.ws = self.mask = self.weight = self.mode = None
        return out

    def materialise(self, C, dy, parked):
        """The BN's input gradient from the parked operands, added to what autograd delivered."""
        ph, dout, ybn, ws, mask, weight, mode = parked
        dbn = C.bn_act_bwd(dout, None, mask, ybn, ws, weight, mode, False, None)[0]
        is_ph = dy is not None and dy.data_ptr() == ph.data_ptr() and dy.stride() == ph.stride()
        return dbn if (dy is None or is_ph) else dy + dbn


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride: int, want_stats: bool, pending=None):
        C = _ext.require()
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        ctx.wstride = weight.stride()
        ctx.link = bn_link_of(x) if stride == 1 else None
        if stride != 1:
            x = x[:, :, ::stride, ::stride].contiguous(memory_format=torch.channels_last)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        w2 = weight.reshape(cout, cin).to(torch.bfloat16).contiguous()
        if pending is not None:
            # x is a deferred BN+ReLU output: the streaming GEMM applies it to its operand chunks in LDS, writes x
            # and multiplies (gemm_stream.hip kAp)
            y2, stats = C.gemm_nt_stream_apply(_rows(pending.x), pending.ws, w2, _rows(x))
            pending.clear()
            CALLS["1x1_stream_apply"] += 1
        else:
            y2, stats = C.gemm_nt(_rows(x), w2, want_stats)
        y = y2.view(n, h, w, cout).permute(0, 3, 1, 2)
        ctx.save_for_backward(x, w2)
        ctx.dlink = DualBNLink() if (DUAL_1X1 and DUAL_BN and stride == 1 and x.dtype == torch.bfloat16
                                     and cout <= DUAL_1X1_MAX_COUT
                                     and C.conv1x1_dual_bn_ok(n * h * w, cin, cout)) else None
        ctx.stride = stride
        ctx.in_hw = None
        ctx.wdtype = weight.dtype
        ctx.wshape = weight.shape
        ctx.weight_leaf = weight if weight.is_leaf else None
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        C = _ext.require()
        x, w2 = ctx.saved_tensors
        odt = ctx.wdtype if ctx.wdtype in (torch.float32, torch.bfloat16) else torch.float32
        dl = ctx.dlink
        if dl is not None and dl.ph is not None:
            parked = dl.take()
            ph, dout, ybn, ws, mask, weight, _ = parked
            if (dy is not None and dy.data_ptr() == ph.data_ptr() and dy.stride() == ph.stride()
                    and ctx.needs_input_grad[0] and ctx.needs_input_grad[1]
                    and not _wants_defer("1x1", ctx, x.shape[1], ybn.shape[1])):
                out = C.conv1x1_dual(_rows(dout), _rows(x), w2, odt, _rows(ybn), ws, mask)
                if out:  # BN apply + data gradient + weight gradient, one pass over the BN's gradient
                    CALLS["1x1_dual_bn"] += 1
                    n, cin, h, w = x.shape
                    dx = out[0].view(n, h, w, cin).permute(0, 3, 1, 2)
                    return dx, _as_param_layout(out[1].to(ctx.wdtype), ctx.wshape, ctx.wstride), None, None, None
            # materialise the BN's input gradient (its reduction is re-run: ws is recomputed identically)
            dy = dl.materialise(C, dy, parked)
        if dy is None:
            return None, None, None, None, None
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        dy2 = _rows(dy)
        dx = dw = None
        wg = None
        if WGRAD_JOIN == "conv":
            join_compute(dy.device)

        def wgrad():
            return _as_param_layout(C.gemm_tn(dy2, _rows(x), odt, 1.0).to(ctx.wdtype), ctx.wshape, ctx.wstride)

        defer = _wants_defer("1x1", ctx, x.shape[1], dy.shape[1])
        if (DUAL_1X1 and dy.shape[1] <= DUAL_1X1_MAX_COUT and ctx.stride == 1 and ctx.needs_input_grad[0]
                and ctx.needs_input_grad[1] and not defer
                and ctx.link is None and x.dtype == torch.bfloat16
                and C.conv1x1_dual_blocks(dy2.shape[0], x.shape[1], dy.shape[1]) > 0):
            out = C.conv1x1_dual(dy2, _rows(x), w2, odt)
            if out:  # one pass over dy for both gradients (gemm_dual.hip)
                CALLS["1x1_dual"] += 1
                n, cin, h, w = x.shape
                dx = out[0].view(n, h, w, cin).permute(0, 3, 1, 2)
                return dx, _as_param_layout(out[1].to(ctx.wdtype), ctx.wshape, ctx.wstride), None, None, None
        if ctx.needs_input_grad[1] and not defer:
            wg = _SideWork(wgrad, dy2.shape[0], dy.device)
        if ctx.needs_input_grad[0]:
            link = ctx.link
            if link is not None and not _epi_ok(dy2.shape[0], w2.shape[1], dy2.shape[1], False):
                link = None
            if link is not None:
                dx2, part = C.gemm_nt_bn(dy2, w2, None, True, _rows(link.x), link.ws, link.mask, link.mode)
                link.publish(dx2, part)
            else:
                dx2, _ = C.gemm_nt(dy2, w2, False, None, True)
            n, cin, h, w = x.shape
            dxs = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
            if ctx.stride != 1:
                H, W = h * ctx.stride, w * ctx.stride
                dx = torch.empty((n, cin, H, W), device=dy.device, dtype=dxs.dtype,
                                 memory_format=torch.channels_last).zero_()
                dx[:, :, ::ctx.stride, ::ctx.stride] = dxs
            else:
                dx = dxs
        if defer:
            dw = _wgrad_after_dgrad(wgrad, ctx, (dy, x), dy.device)
        if wg is not None:
            dw = wg.result()
        return dx, dw, None, None, None


class _Conv1x1Fork(torch.autograd.Function):
    """Stride-1 1x1 conv that also hands its input on as a second output (the block's identity
    branch). Both gradients of ``x`` then arrive in one backward call, and the identity gradient
    is added inside the dgrad GEMM's epilogue (``dX = dY W + d_identity``) instead of by a separate
    elementwise kernel over the block-input tensor (the autograd sum of the two uses of ``x``)."""

    @staticmethod
    def forward(ctx, x, weight, want_stats: bool, rlink, sub: bool = False, pending=None):
        C = _ext.require()
        ctx.set_materialize_grads(False)
        ctx.rlink = rlink
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        w2 = weight.reshape(cout, cin).to(torch.bfloat16).contiguous()
        # sub: also hand on the stride-2 subsample of x (the downsample conv's input); its compact
        # gradient is added at the even pixels inside the dgrad epilogue (no zero-filled scatter)
        xs = None
        if pending is not None:
            # x is a deferred BN(+residual)+ReLU output: this GEMM writes it (and its ReLU mask, and with sub its
            # stride-2 subsample) while staging its operand from the BN's input and the residual (gemm_apply.hip),
            # then multiplies
            p = pending
            if sub and knobs.flag("APPLY_SUBSAMPLE"):
                xs = torch.empty((n, cin, h // 2, w // 2), dtype=x.dtype, device=x.device,
                                 memory_format=torch.channels_last)
            y2, stats = C.gemm_nt_apply(_rows(p.x), _rows(p.r), p.ws, p.wsd, w2, want_stats, _rows(x), p.mask,
                                        xs, h if xs is not None else 0, w if xs is not None else 0)
            p.clear()
            CALLS["1x1_apply"] += 1
        else:
            y2, stats = C.gemm_nt(_rows(x), w2, want_stats)
        if sub and xs is None:
            xs = C.subsample2(x) if (x.dtype == torch.bfloat16 and cin % 8 == 0) else \
                x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)
        y = y2.view(n, h, w, cout).permute(0, 3, 1, 2)
        ctx.save_for_backward(x, w2)
        ctx.wdtype = weight.dtype
        ctx.wshape = weight.shape
        ctx.weight_leaf = weight if weight.is_leaf else None
        ctx.wstride = weight.stride()
        ctx.link = bn_link_of(x)
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        return y, stats, x, xs

    @staticmethod
    def backward(ctx, dy, _dstats, dident, dsub=None):
        C = _ext.require()
        x, w2 = ctx.saved_tensors
        n, cin, h, w = x.shape
        if dsub is not None:
            dsub = dsub.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
        rl = ctx.rlink
        amask = None
        if rl is not None and rl.dy is not None:
            # identity gradient handed over by the BN(+residual)+ReLU that consumed the identity:
            # dy where the forward's ReLU bit is set (added in the epilogue below)
            rdy, rmask = rl.dy, rl.mask
            rl.dy = rl.mask = None
            if dident is None:
                dident, amask = rdy, rmask
            else:  # the identity had other consumers too: materialise the masked gradient
                dident = dident + (rdy if rmask is None else rdy * _unpack_bits(rmask, rdy))
        if dident is not None:
            dident = dident.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
        if dy is None:
            if amask is not None:
                dident = dident * _unpack_bits(amask, dident)
            if dsub is not None:
                full = torch.zeros_like(x) if dident is None else dident.clone()
                full[:, :, ::2, ::2] += dsub
                dident = full
            return dident, None, None, None, None, None
        odt = ctx.wdtype if ctx.wdtype in (torch.float32, torch.bfloat16) else torch.float32
        dy = dy.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
        dy2 = _rows(dy)
        dx = dw = None
        wg = None
        if WGRAD_JOIN == "conv":
            join_compute(dy.device)

        def wgrad():
            return _as_param_layout(C.gemm_tn(dy2, _rows(x), odt, 1.0).to(ctx.wdtype), ctx.wshape, ctx.wstride)

        defer = _wants_defer("1x1", ctx, x.shape[1], dy.shape[1])
        if ctx.needs_input_grad[1] and not defer:
            wg = _SideWork(wgrad, dy2.shape[0], dy.device)
        if ctx.needs_input_grad[0]:
            add = None if dident is None else _rows(dident)
            link = ctx.link
            if link is not None and (dsub is not None or not _epi_ok(dy2.shape[0], w2.shape[1], dy2.shape[1],
                                                                     add is not None)) and BN_EPILOGUE != "1":
                link = None
            if link is not None:
                dx2, part = C.gemm_nt_bn(dy2, w2, add, True, _rows(link.x), link.ws, link.mask, link.mode, amask,
                                         dsub, h, w)
            else:
                dx2, _ = C.gemm_nt(dy2, w2, False, add, True, 0, amask, dsub, h, w)
            dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
            if link is not None:
                link.publish(dx, part)
        if defer:
            dw = _wgrad_after_dgrad(wgrad, ctx, (dy, x), dy.device)
        if wg is not None:
            dw = wg.result()
        return dx, dw, None, None, None, None


def _unpack_bits(mask: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    """Expand a 1-bit mask (element order of `like` in channels_last) to a 0/1 tensor like `like`."""
    bits = torch.stack([(mask >> j) & 1 for j in range(8)], 1).reshape(-1)[: like.numel()]
    n, c, h, w = like.shape
    return bits.view(n, h, w, c).permute(0, 3, 1, 2).to(like.dtype)


def fork_supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return supported(x, conv) and conv.stride in ((1, 1), 1)


# Hand the residual gradient of the block's final BN(+residual)+ReLU to the fork as (dy, mask)
# instead of a materialised tensor (ResidualLink).
RESIDUAL_HANDOFF = True


def conv1x1_fork(x: torch.Tensor, conv: nn.Conv2d, want_stats: bool = False, sub: bool = False):
    """Returns (y, stats-or-None, x_alias, x_sub-or-None); use ``x_alias`` as the residual identity
    and ``x_sub`` (= x[:, :, ::2, ::2], with sub) as a stride-2 downsample conv's input."""
    CALLS["1x1_fork"] += 1
    rlink = ResidualLink() if RESIDUAL_HANDOFF and x.requires_grad else None
    pending = pending_of(x)
    if pending is not None and not (pending.r is not None and x.is_contiguous(memory_format=torch.channels_last)
                                    and _ext.require().gemm_nt_apply_ok(x.numel() // x.shape[1], conv.out_channels,
                                                                        x.shape[1])):
        pending.materialise()
        pending = None
    y, stats, xa, xs = _Conv1x1Fork.apply(x, conv.weight, want_stats, rlink, sub, pending)
    if rlink is not None:
        xa._dla_fork = rlink
    return y, stats, xa, xs


def conv1x1(x: torch.Tensor, conv: nn.Conv2d, want_stats: bool = False, stride: int | None = None):
    """Returns (y, stats-or-None); stats are [row_blocks, Cout, 2] partial (sum, sumsq).
    ``stride`` overrides the module's (1 for an input that is already subsampled)."""
    CALLS["1x1"] += 1
    s = conv.stride[0] if stride is None else stride
    if x.shape[2] % s or x.shape[3] % s:
        # odd spatial size with stride 2 (output ceil) — keep F.conv2d semantics exactly
        return F.conv2d(x, conv.weight.to(x.dtype), None, s), None
    pending = pending_of(x)
    if pending is not None and not (pending.r is None and s == 1 and want_stats
                                    and x.is_contiguous(memory_format=torch.channels_last)
                                    and _ext.require().gemm_nt_stream_apply_ok(x.numel() // x.shape[1],
                                                                              conv.out_channels, x.shape[1])):
        pending.materialise()
        pending = None
    y, stats = _Conv1x1.apply(x, conv.weight, s, want_stats, pending)
    dl = getattr(y.grad_fn, "dlink", None) if y.grad_fn is not None else None
    if dl is not None:
        y._dla_dual = dl
    return y, stats


# ---------------------------------------------------------------------------------------------
# 3x3 convolutions (csrc/kernels/conv.hip): implicit GEMMs gathered straight from NHWC tensors.
# Per-pass engine choice from scripts/bench_conv.py at the ResNet-50 bs256 shapes on MI355X
# (profiles/mfma_kernels_vs_libraries.md), with the 2-stage LDS-DMA main loop: the native forward
# beats MIOpen on 5 of the 7 shapes (and its epilogue yields the BatchNorm statistics, saving a
# pass over the output), the stride-1 data gradient and the weight gradient win everywhere. The
# stride-2 data gradient runs as 4 parity-class GEMMs (conv3x3s2_dgrad); MIOpen only for odd sizes.
# ---------------------------------------------------------------------------------------------
CONV3_POLICY = {"fwd": "native", "dgrad_native_max_cin": 1 << 30, "wgrad": "native"}


def supported3x3(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and conv.kernel_size == (3, 3)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and _conv3_channels_ok(conv) and x.is_contiguous(memory_format=torch.channels_last)
            and _limits.pixels_ok(x.numel() // x.shape[1], "conv3x3")
            and _limits.span_ok(max(x.numel(), x.numel() // x.shape[1] // conv.stride[0] ** 2 * conv.out_channels)
                                * x.element_size(), "conv3x3 operand"))


def _conv3_channels_ok(conv: nn.Conv2d) -> bool:
    """Stride 1: any channel count % 8 (the any-C loaders decode the tap per 8-channel chunk, e.g.
    GoogLeNet's 16/24/48/96/112/144/160); stride 2: % 64 (the parity-class data gradient)."""
    ci, co = conv.in_channels, conv.out_channels
    if conv.stride == (1, 1):
        return ci % 8 == 0 and co % 8 == 0
    return conv.stride == (2, 2) and ci % 64 == 0 and co % 64 == 0


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride: int, want_stats: bool):
        C = _ext.require()
        ctx.set_materialize_grads(False)
        ctx.link = bn_link_of(x)
        w = weight.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        stats = None
        if CONV3_POLICY["fwd"] == "native" or want_stats:
            y, stats = C.conv3x3_fwd(x, w, stride, want_stats)
        else:
            y = F.conv2d(x, w, None, stride, 1)
        ctx.save_for_backward(x, w)
        ctx.stride = stride
        ctx.wdtype = weight.dtype
        ctx.weight_leaf = weight if weight.is_leaf else None
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        if dy is None:
            return None, None, None, None
        C = _ext.require()
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
        dx = dw = None
        wg = None
        if WGRAD_JOIN == "conv":
            join_compute(dy.device)
        defer = _wants_defer("3x3", ctx)
        if ctx.needs_input_grad[1]:
            odt = ctx.wdtype if ctx.wdtype in (torch.float32, torch.bfloat16) else torch.float32

            def wgrad():
                if CONV3_POLICY["wgrad"] == "native":
                    g = C.conv3x3_wgrad(dy, x, ctx.stride, odt)
                else:
                    g = torch.ops.aten.convolution_backward(dy, x, w, None, [ctx.stride] * 2, [1, 1], [1, 1], False,
                                                            [0, 0], 1, [False, True, False])[1]
                return g.to(ctx.wdtype)

            if not defer:
                wg = _SideWork(wgrad, dy.shape[0] * dy.shape[2] * dy.shape[3], dy.device)
        if ctx.needs_input_grad[0]:
            if ctx.stride == 1 and x.shape[1] <= CONV3_POLICY["dgrad_native_max_cin"]:
                link = ctx.link if BN_EPILOGUE == "1" else None
                if link is not None:
                    dx, part = C.conv3x3_dgrad_bn(dy, w, None, link.x, link.ws, link.mask, link.mode)
                    link.publish(dx, part)
                else:
                    dx = C.conv3x3_dgrad(dy, w)
            elif ctx.stride == 2 and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0:
                dx = C.conv3x3s2_dgrad(dy, w, x.shape[2], x.shape[3])
            else:
                dx = torch.ops.aten.convolution_backward(dy, x, w, None, [ctx.stride] * 2, [1, 1], [1, 1], False,
                                                         [0, 0], 1, [True, False, False])[0]
        if defer:
            dw = _wgrad_after_dgrad(wgrad, ctx, (dy, x, w), dy.device)  # w: the aten fallback reads it
        if wg is not None:
            dw = wg.result()
        return dx, dw, None, None


def conv3x3(x: torch.Tensor, conv: nn.Conv2d, want_stats: bool = False):
    """Returns (y, stats-or-None); stats are [row_blocks, Cout, 2] partial (sum, sumsq) when the
    native forward ran."""
    CALLS["3x3"] += 1
    return _Conv3x3.apply(x, conv.weight, conv.stride[0], want_stats)


# ---- ResNet stem: 7x7 / stride 2 / pad 3 conv on 3-channel images (csrc/kernels/stem.hip) ---------
# The image is folded space-to-depth (2x2 pixels -> 12 channels, padded to 16) and the conv runs as
# a stride-1 4x4 conv over the fold: K = 16 taps x 16 channels = 256, weight index
# k = (th * 4 + tw) * 16 + (ph * 2 + pw) * 3 + c  <->  W[co, c, 2 th + ph - 1, 2 tw + pw - 1].
STEM_K = 256


def supported_stem(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.shape[1] == 3
            and conv.kernel_size == (7, 7) and conv.stride == (2, 2) and conv.padding == (3, 3)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None and conv.out_channels % 64 == 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and _limits.pixels_ok(x.shape[0] * ((x.shape[2] + 1) // 2) * ((x.shape[3] + 1) // 2), "stem conv"))


def stem_pack_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, 3, 7, 7] -> packed bf16 [Cout, 256] of the folded 4x4 conv (zeros at kh or kw = -1)."""
    co = w.shape[0]
    wp = F.pad(w.to(torch.bfloat16), (1, 0, 1, 0))  # [co, 3, 8, 8]: index kh + 1 = 2 th + ph
    wp = wp.reshape(co, 3, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1).reshape(co, 16, 12)  # (th, tw), (ph, pw, c)
    return F.pad(wp, (0, 4)).reshape(co, STEM_K).contiguous()


def stem_unpack_grad(dwp: torch.Tensor) -> torch.Tensor:
    """Packed [Cout, 256] gradient -> [Cout, 3, 7, 7]."""
    co = dwp.shape[0]
    g = dwp.reshape(co, 4, 4, 16)[..., :12].reshape(co, 4, 4, 2, 2, 3)  # th, tw, ph, pw, c
    g = g.permute(0, 5, 1, 3, 2, 4).reshape(co, 3, 8, 8)  # c, (th, ph), (tw, pw)
    return g[:, :, 1:, 1:]


# The stem BN+ReLU+max-pool backward apply inside the stem weight gradient (stem.hip stem_wgrad_bn_kernel): the
# conv output's gradient (2 GB at batch 1280) is never written or read back.
STEM_BN = knobs.flag("STEM_BN")


class StemBNLink(DualBNLink):
    """Hand-off from the stem BN+ReLU+max-pool (ops/bn_act.py _BNReluPool) to the stem conv's backward.

    The pooled op's backward stops after its reduction + finalize, parks (pooled gradient, argmax positions,
    conv output, coefficients) here and returns a zero-stride placeholder; the stem weight gradient computes the
    conv output's gradient tile by tile from them. Same claim / observed guards as DualBNLink; a non-placeholder
    gradient (other consumers of the conv output) materialises the parked gradient and adds it."""

    __slots__ = ("pos", "geom")

    def park(self, dout, pos, ybn, ws, weight, geom):
        assert self.can_park(ybn), "StemBNLink.park: check can_park first"
        self.dout, self.pos, self.ybn, self.ws, self.weight, self.geom = dout, pos, ybn, ws, weight, geom
        self.ph = torch.zeros((), dtype=ybn.dtype, device=ybn.device).expand(ybn.shape)
        return self.ph

    def take(self):
        out = (self.ph, self.dout, self.pos, self.ybn, self.ws, self.weight, self.geom)
        self.ph = self.dout = self.pos = self.ybn = self.ws = self.weight = self.geom = None
        return out

    def materialise(self, C, dy, parked):
        ph, dout, pos, ybn, ws, weight, (k, s, p) = parked
        dbn = C.bn_relu_maxpool_bwd(dout, pos, ybn, ws, weight, k, s, p)[0]  # reduction re-run: same ws
        is_ph = dy is not None and dy.data_ptr() == ph.data_ptr() and dy.stride() == ph.stride()
        return dbn if (dy is None or is_ph) else dy + dbn


def stem_bn_fusable(x: torch.Tensor, y_shape, k: int, s: int, p: int) -> bool:
    """Whether the stem conv output ``x`` pooled 3x3 / s2 / p1 to ``y_shape`` is the quad form stem_wgrad_bn
    serves (64 channels, even size, pooled to exactly half; < 2^24 pixels)."""
    n, c, h, w = x.shape
    return (k == 3 and s == 2 and p == 1 and c == 64 and h % 2 == 0 and w % 2 == 0
            and tuple(y_shape[2:]) == (h // 2, w // 2) and n * h * w < (1 << 24))


class _StemConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, want_stats: bool):
        C = _ext.require()
        ctx.set_materialize_grads(False)
        y, stats, xs = C.stem_fwd(x, stem_pack_weight(weight), want_stats)
        ctx.save_for_backward(xs)
        ctx.slink = StemBNLink() if STEM_BN and y.dtype == torch.bfloat16 else None
        ctx.hw = (x.shape[2], x.shape[3])
        ctx.wdtype = weight.dtype
        ctx.wfmt = torch.channels_last if weight.is_contiguous(memory_format=torch.channels_last) and \
            not weight.is_contiguous() else torch.contiguous_format
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        if dy is None:
            return None, None, None
        if ctx.needs_input_grad[0]:
            raise RuntimeError("native stem conv: no input gradient (the stem input is the data batch)")
        (xs,) = ctx.saved_tensors
        dw = None
        sl = ctx.slink
        if sl is not None and sl.ph is not None:
            parked = sl.take()
            ph, dout, pos, ybn, ws = parked[:5]
            if not ctx.needs_input_grad[1]:
                return None, None, None
            if dy.data_ptr() == ph.data_ptr() and dy.stride() == ph.stride():
                odt = ctx.wdtype if ctx.wdtype in (torch.float32, torch.bfloat16) else torch.float32
                CALLS["stem_bn"] += 1
                dwp = _ext.require().stem_wgrad_bn(dout, pos, ybn, ws, xs, ctx.hw[0], ctx.hw[1], odt)
                dw = stem_unpack_grad(dwp).to(ctx.wdtype).contiguous(memory_format=ctx.wfmt)
                return None, dw, None
            dy = sl.materialise(_ext.require(), dy, parked)
        if ctx.needs_input_grad[1]:
            odt = ctx.wdtype if ctx.wdtype in (torch.float32, torch.bfloat16) else torch.float32
            dwp = _ext.require().stem_wgrad(dy.contiguous(memory_format=torch.channels_last).to(torch.bfloat16), xs,
                                            ctx.hw[0], ctx.hw[1], odt)
            dw = stem_unpack_grad(dwp).to(ctx.wdtype).contiguous(memory_format=ctx.wfmt)
        return None, dw, None


def stem_conv(x: torch.Tensor, conv: nn.Conv2d, want_stats: bool = False):
    """The ResNet stem conv on the native kernels. Returns (y, stats-or-None); stats are the
    [row_blocks, Cout, 2] (sum, sumsq) partials of y for the fused BatchNorm."""
    CALLS["stem"] += 1
    y, stats = _StemConv.apply(x, conv.weight, want_stats)
    sl = getattr(y.grad_fn, "slink", None) if y.grad_fn is not None else None
    if sl is not None:
        y._dla_stem = sl
    return y, stats

