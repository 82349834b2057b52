"""GoogLeNet Inception blocks on the fp32 path (``--precision fp32`` with native convs).

The reference's block (torchvision v0.6 Inception, /root/reference/src/network.py:33-54) runs four branches on the
same input: three of them start with a 1x1 conv of x (branch1, the 3x3-reduce of branch2, the "5x5"-reduce of
branch3). Here those three convs are ONE fp32 GEMM over x with their weights concatenated along Cout
(``torch.cat`` of the three weight tensors: their gradients split back through autograd), followed by ONE fused
BatchNorm+ReLU pass over the concatenated channels (the three BN modules' parameters concatenated; their running
statistics are views into one buffer, so the fused kernel updates all three in place). The reduce activations are
consumed as channel slices (the fp32 conv kernels read a slice in place: pixel stride = the concatenation's width),
and their gradients are written back into one buffer by :class:`_SplitChannels`.

Per block that replaces 3 small GEMMs (16-192 output channels, 10-50 TFLOP/s) by one of 176-464 channels in each of
forward, data gradient and weight gradient, 3 BN launches by 1 in each direction, and two of the three autograd
sums of x's four branch gradients (the data gradient of the concatenated conv already is their sum).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import conv_f32

CL = torch.channels_last


class _SplitChannels(torch.autograd.Function):
    """``a`` -> its channel slices (views); backward assembles the slices' gradients in one channels_last buffer."""

    @staticmethod
    def forward(ctx, a, sizes):
        ctx.sizes = tuple(sizes)
        ctx.meta = (a.shape, a.dtype, a.device)
        outs, off = [], 0
        for c in sizes:
            outs.append(a.narrow(1, off, c))
            off += c
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        shape, dtype, device = ctx.meta
        g = torch.empty(shape, dtype=dtype, device=device, memory_format=CL)
        off = 0
        for d, c in zip(grads, ctx.sizes):
            sl = g.narrow(1, off, c)
            if d is None:
                sl.zero_()
            else:
                sl.copy_(d)
            off += c
        return g, None


class _CatBN:
    """Duck-typed BatchNorm2d over the concatenated channels of several BN modules (what ops/bn_act.fused_bn_act
    reads): concatenated affine parameters (autograd-tracked), running statistics in one buffer of which the
    modules' own buffers are views."""

    def __init__(self, bns, rm, rv):
        self.training = bns[0].training
        self.track_running_stats = True
        self.affine = True
        self.momentum = bns[0].momentum
        self.eps = bns[0].eps
        self.weight = torch.cat([b.weight for b in bns])
        self.bias = torch.cat([b.bias for b in bns])
        self.running_mean, self.running_var = rm, rv
        self.num_batches_tracked = bns[0].num_batches_tracked


def _stat_views(block, bns):
    """The concatenated running-statistics buffers, (re)built when a module's buffers are not views of them
    (first call, or after .to() / load_state_dict replaced them)."""
    st = getattr(block, "_dla_f32_stats", None)
    if st is not None:
        rm, rv = st
        off, ok = 0, True
        for b in bns:
            c = b.num_features
            ok = ok and b.running_mean.data_ptr() == rm.data_ptr() + 4 * off \
                and b.running_var.data_ptr() == rv.data_ptr() + 4 * off and rm.device == b.running_mean.device
            off += c
        if ok:
            return rm, rv
    rm = torch.cat([b.running_mean for b in bns]).contiguous()
    rv = torch.cat([b.running_var for b in bns]).contiguous()
    off = 0
    for b in bns:
        c = b.num_features
        b.running_mean = rm[off:off + c]
        b.running_var = rv[off:off + c]
        off += c
    block._dla_f32_stats = (rm, rv)
    return rm, rv


def supported(block, x: torch.Tensor) -> bool:
    heads = (block.branch1, block.branch2[0], block.branch3[0])
    if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and x.is_contiguous(memory_format=CL)):
        return False
    for h in heads:
        c, bn = h.conv, h.bn
        if c.kernel_size != (1, 1) or c.stride != (1, 1) or c.padding != (0, 0) or not conv_f32.supported(x, c):
            return False
        if not (bn.affine and bn.track_running_stats and bn.momentum is not None and bn.weight.dtype == torch.float32):
            return False
        if bn.eps != heads[0].bn.eps or bn.momentum != heads[0].bn.momentum or bn.training != heads[0].bn.training:
            return False
        if c.out_channels % 8:
            return False
    return True


def forward(block, x: torch.Tensor) -> torch.Tensor:
    from . import bn_act

    heads = (block.branch1, block.branch2[0], block.branch3[0])
    bns = [h.bn for h in heads]
    sizes = [h.conv.out_channels for h in heads]
    w = torch.cat([h.conv.weight for h in heads])  # [c1 + c2r + c3r, cin, 1, 1]
    y = conv_f32.conv_w(x, w, 0, 1)
    rm, rv = _stat_views(block, bns)
    cat_bn = _CatBN(bns, rm, rv)
    a = bn_act.fused_bn_act(y, cat_bn, True, None)
    if cat_bn.training:  # fused_bn_act queued the first module's counter; the others advance with it
        for b in bns[1:]:
            bn_act._PENDING_COUNTERS.append(b.num_batches_tracked)
    a1, a2r, a3r = _SplitChannels.apply(a, sizes)
    y2 = block.branch2[1](a2r)
    y3 = block.branch3[1](a3r)
    y4 = block.branch4(x)
    return torch.cat([a1, y2, y3, y4], 1)
