"""fp32 convolutions on the native fp32 matrix-core kernels (csrc/kernels/conv_f32.hip).

The reference-precision path (``--precision fp32``: GoogLeNet in fp32, /root/reference/src/network.py:33-54,
main.py:36) ran its convolutions on MIOpen; here every 1x1 / 3x3 / 7x7 conv of that step is an implicit GEMM on
``v_mfma_f32_16x16x4_f32`` (exact fp32 products and fp32 accumulation, no reduced-precision xf32 form):

* forward   ``C.conv_f32_fwd(x, W_ohwi, pad, stride)``;
* dgrad     the forward kernel over ``dy`` with the weights flipped and transposed (``[Cin][R][S][Cout]``,
  padding ``R - 1 - pad``; stride 1 -- the only strided conv, the stem, has no input gradient);
* wgrad     ``C.conv_f32_wgrad``: the pixel reduction split over blocks, fp32 slabs summed by splitk_reduce.

Activations stay channels_last (NHWC) and fp32 end to end; a channels_last conv weight IS the OHWI layout the
kernels read, so the forward takes it without a copy, and its gradient is produced in the same layout. The stem's
3 input channels are padded to 4 with zeros (the kernels move 16-byte channel chunks).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext

CL = torch.channels_last

# The stem (3 input channels, 7x7 / stride 2) on these kernels. Generic form: 3 channels padded to 4, each 16-byte
# chunk a different tap, scattered loads (~1.2x MIOpen's time, profiles/r6/g07). Space-to-depth form (stem_s2d):
# the padded image regrouped into 2x2 pixel blocks of 12 channels makes the conv a 4x4 / stride-1 one over the
# block image, whose k-steps read 128 contiguous bytes; STEM_NATIVE routes the model's stem to it.
STEM_NATIVE = True


def supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """A conv this path runs: fp32 channels_last CUDA input, groups 1, no dilation, no bias, channels
    (after padding 3 -> 4) and Cout multiples of 4, stride 1 whenever the input needs a gradient."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and conv.weight.dtype == torch.float32):
        return False
    if conv.groups != 1 or conv.dilation != (1, 1) or conv.bias is not None:
        return False
    if conv.kernel_size[0] != conv.kernel_size[1] or conv.stride[0] != conv.stride[1] or conv.padding[0] != conv.padding[1]:
        return False
    cin, cout = x.shape[1], conv.out_channels
    if cin == 3 and STEM_NATIVE and stem_s2d_ok(x, conv):
        return True
    if cout % 4 or not (cin % 4 == 0 or (cin == 3 and STEM_NATIVE)):
        return False
    if conv.stride[0] != 1 and x.requires_grad:
        return False
    oh = (x.shape[2] + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1
    ow = (x.shape[3] + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1
    return x.shape[0] * oh * ow < (1 << 24) and x.numel() * 4 < (1 << 31)


def nhwc_view_ok(x: torch.Tensor) -> bool:
    """channels_last, or a 16-byte aligned channel slice of a channels_last tensor (what the kernels read in place)."""
    if x.is_contiguous(memory_format=CL):
        return True
    n, c, h, w = x.shape
    ldp = x.stride(3)
    return (x.stride(1) == 1 and ldp >= c and ldp % 4 == 0 and x.stride(2) == ldp * w and x.stride(0) == ldp * w * h
            and x.data_ptr() % 16 == 0)


def _ohwi(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, R, S] -> [Cout, R, S, Cin] contiguous (a view when w is channels_last)."""
    return w.permute(0, 2, 3, 1).contiguous()


def _pad_channels(x: torch.Tensor, c: int) -> torch.Tensor:
    n, c0, h, w = x.shape
    out = torch.empty((n, c, h, w), dtype=x.dtype, device=x.device, memory_format=CL).zero_()
    out[:, :c0] = x
    return out


class _ConvF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, pad: int, stride: int):
        C = _ext.require()
        cin = x.shape[1]
        xs = x if nhwc_view_ok(x) else x.contiguous(memory_format=CL)
        w = _ohwi(weight)
        if cin % 4:  # the stem: 3 channels -> 4, zero channel and zero weights
            xs = _pad_channels(xs, 4)
            w = F.pad(w, (0, 4 - cin))
        y = C.conv_f32_fwd(xs, w, pad, stride)
        ctx.save_for_backward(xs, weight)
        ctx.pad, ctx.stride, ctx.cin = pad, stride, cin
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        xs, weight = ctx.saved_tensors
        dy = dy.contiguous(memory_format=CL)
        if dy.dtype != torch.float32:
            dy = dy.float()
        r, s = weight.shape[2], weight.shape[3]
        dx = dw = None
        if ctx.needs_input_grad[0]:
            # dX = the forward of dY with W flipped in both taps and transposed to [Cin][R][S][Cout] (stride 1)
            wt = weight.flip(2, 3).permute(1, 2, 3, 0).contiguous()
            dx = C.conv_f32_fwd(dy, wt, r - 1 - ctx.pad, 1)
        if ctx.needs_input_grad[1]:
            g = C.conv_f32_wgrad(dy, xs, r, s, ctx.pad, ctx.stride)  # [Cout, R, S, Cin(+pad)]
            if g.shape[3] != ctx.cin:
                g = g[..., : ctx.cin]
            dw = g.permute(0, 3, 1, 2)  # [Cout, Cin, R, S] in channels_last memory
            if not dw.is_contiguous(memory_format=CL) or weight.stride() != dw.stride():
                dw = dw.contiguous(memory_format=CL) if weight.is_contiguous(memory_format=CL) else dw.contiguous()
        return dx, dw, None, None


def stem_s2d_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.shape[1] == 3 and conv.kernel_size == (7, 7) and conv.stride == (2, 2) and conv.padding == (3, 3)
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0 and not x.requires_grad and conv.out_channels % 4 == 0)


def _s2d_image(x: torch.Tensor) -> torch.Tensor:
    """[N, 3, H, W] -> the zero-padded (3 px) image as 2x2 pixel blocks: [N, 12, (H+6)/2, (W+6)/2] channels_last,
    channel (dh, dw, c)."""
    n, c, h, w = x.shape
    xp = F.pad(x, (3, 3, 3, 3))
    hb, wb = (h + 6) // 2, (w + 6) // 2
    img = xp.reshape(n, c, hb, 2, wb, 2).permute(0, 2, 4, 3, 5, 1).reshape(n, hb, wb, 4 * c)
    return img.permute(0, 3, 1, 2)  # channels_last view of the contiguous [N, hb, wb, 12] image


def _s2d_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, 3, 7, 7] -> [Cout, 4, 4, 12] (taps over 2x2 blocks, channel (dh, dw, c)); the 8th row / column are 0."""
    co, c = w.shape[0], w.shape[1]
    wp = F.pad(w, (0, 1, 0, 1))  # [co, c, 8, 8]
    return wp.reshape(co, c, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1).reshape(co, 4, 4, 4 * c).contiguous()


def _s2d_grad(g: torch.Tensor, c: int) -> torch.Tensor:
    """inverse of _s2d_weight for the gradient: [Cout, 4, 4, 12] -> [Cout, 3, 7, 7]"""
    co = g.shape[0]
    return g.reshape(co, 4, 4, 2, 2, c).permute(0, 5, 1, 3, 2, 4).reshape(co, c, 8, 8)[:, :, :7, :7]


class _StemS2D(torch.autograd.Function):
    """The 7x7 / stride-2 stem as a 4x4 / stride-1 conv over the space-to-depth image (no input gradient)."""

    @staticmethod
    def forward(ctx, x, weight):
        C = _ext.require()
        img = _s2d_image(x)
        y = C.conv_f32_fwd(img, _s2d_weight(weight), 0, 1)
        ctx.save_for_backward(img)
        ctx.cin = weight.shape[1]
        ctx.wlayout = weight.is_contiguous(memory_format=CL)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        (img,) = ctx.saved_tensors
        dy = dy.contiguous(memory_format=CL)
        dw = None
        if ctx.needs_input_grad[1]:
            dw = _s2d_grad(C.conv_f32_wgrad(dy, img, 4, 4, 0, 1), ctx.cin)
            dw = dw.contiguous(memory_format=CL) if ctx.wlayout else dw.contiguous()
        return None, dw


def conv(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """``conv(x)`` on the fp32 matrix-core kernels (caller checked :func:`supported`)."""
    if x.shape[1] == 3 and STEM_NATIVE and stem_s2d_ok(x, conv):
        return _StemS2D.apply(x, conv.weight)
    return _ConvF32.apply(x, conv.weight, conv.padding[0], conv.stride[0])


def conv_w(x: torch.Tensor, weight: torch.Tensor, pad: int = 0, stride: int = 1) -> torch.Tensor:
    """The same with an explicit weight tensor (e.g. several convs' weights concatenated along Cout)."""
    return _ConvF32.apply(x, weight, pad, stride)
