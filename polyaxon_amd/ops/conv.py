"""KxK convolutions (K = 1 or 3, pad K//2, stride 1 or 2) on NHWC bf16 as implicit MFMA GEMMs (csrc/conv_gemm.hip).

Every ResNet-50 convolution except the 3-channel stem goes through here or through the dense 1x1 path of
:mod:`polyaxon_amd.ops.conv1x1`.  Each pass reuses the GEMM kernels with a gathered operand: the reduction
index is (tap, channel), and the operand row for a tap is the pixel shifted by that tap, read straight from
the NHWC activation by the per-lane global->LDS copy (out-of-image taps read a zero page = the padding).  No
im2col buffer is ever materialised.

* forward      ``y[m][co] = Σ_tap,ci x[S·m + tap - p][ci] · W[co][tap][ci]``         (+ BN channel stats)
* data grad    stride 1: the same gather with flipped taps over dy; stride 2: one GEMM per (ih, iw) parity
               class of the input, over the taps of matching parity, rows scattered back (no wasted taps)
* weight grad  ``dW[co][tap][ci] = Σ_m dy[m][co] · x[S·m + tap - p][ci]`` (fp32, split over m, slab-reduced)

No pass needs a memset: this path is hipGraph-capturable end to end (MIOpen's strided data-gradient kernels
are not — their uncaptured output zeroing leaves garbage on replay, see polyflow.executor.capture(verify=)).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import ctypes

from polyaxon_amd.ops import _native, side_stream, wcache
from polyaxon_amd.ops.conv1x1 import (GradMailbox, _bf16_context, _num_cus, _stream, _zero_page, bn_link_of, nt_stats_rows,
                                      unpack_relu_mask)
from polyaxon_amd.ops.flat import direct_grad


def _out(h: int, k: int, s: int) -> int:
    return (h + 2 * (k // 2) - k) // s + 1


def weight_prep_k(w: torch.Tensor):
    """fp32 [Cout][Cin][K][K] (any strides) -> (bf16 Wf [Cout][K*K][Cin], bf16 Wd [Cin][K*K][Cout])."""
    cout, cin, k = w.shape[0], w.shape[1], w.shape[2]
    if w.dtype != torch.float32:
        w = w.float()
    wf = torch.empty(cout, k * k, cin, dtype=torch.bfloat16, device=w.device)
    wd = torch.empty(cin, k * k, cout, dtype=torch.bfloat16, device=w.device)
    st = w.stride()
    rc = _native.lib("plx_conv").plx_weight_prepk(w.data_ptr(), st[0], st[1], st[2], st[3], wf.data_ptr(),
                                                  wd.data_ptr(), cout, cin, k, _stream())
    _native.check(rc, "plx_weight_prepk")
    return wf, wd


class _ConvK(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stats, stride, box, link):
        lib = _native.lib("plx_conv")
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n, cin, h, w = x.shape
        cout, k = weight.shape[0], weight.shape[2]
        ho, wo = _out(h, k, stride), _out(w, k, stride)
        wf, wd = wcache.lookup(weight) or weight_prep_k(weight)
        y = torch.empty((n, cout, ho, wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        rc = lib.plx_conv_fwd(x.data_ptr(), wf.data_ptr(), y.data_ptr(), n, h, w, cin, cout, k, stride,
                              _zero_page(x.device).data_ptr(), stats.data_ptr() if stats is not None else None,
                              _stream())
        _native.check(rc, "plx_conv_fwd")
        ctx.save_for_backward(x, wd)
        ctx.wshape = weight.shape
        ctx.stride = stride
        ctx.box = box
        # a strided 1x1 dgrad never writes the odd pixels: it only finishes a split link (BnLink.request_split)
        ctx.s2k1 = stride == 2 and k == 1
        ctx.link = link
        g = direct_grad(weight)
        ctx.wgrad = g if (g is not None and g.stride() == (k * k * cin, 1, k * cin, cin)) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.lib("plx_conv")
        x, wd = ctx.saved_tensors
        n, cin, h, w = x.shape
        cout, k = ctx.wshape[0], ctx.wshape[2]
        s = ctx.stride
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        zero = _zero_page(x.device).data_ptr()
        dx = dw = None
        extra, extra_mask = ctx.box.take() if ctx.box is not None else (None, None)
        if extra is not None and extra_mask is not None:
            extra = unpack_relu_mask(extra, extra_mask)
        if ctx.needs_input_grad[0]:
            add = None
            if extra is not None:
                extra = extra.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                if s == 2 and k == 1:
                    dx = add = extra  # in place: the even pixels get += dgrad, the rest keep the deferred gradient
                else:
                    add = extra
            if dx is None:
                # a strided 1x1 only reaches the even-even pixels: the rest of dx is zero
                dx = (torch.zeros_like if (s == 2 and k == 1) else torch.empty_like)(x, memory_format=torch.channels_last)
            bnr = None
            if ctx.link is not None and ctx.s2k1:
                if extra is not None and ctx.link.split and ctx.link.part is not None:
                    bnr = ctx.link.request_rest()
            elif ctx.link is not None and (ctx.box is None or extra is not None):
                nblk = _native.size("plx_conv", "plx_conv_dgrad_blocks", n, h, w, cin, cout, k, s)
                bnr = ctx.link.request(nblk)
            rc = lib.plx_conv_dgrad(dy.data_ptr(), wd.data_ptr(), dx.data_ptr(), n, h, w, cin, cout, k, s, zero,
                                    add.data_ptr() if add is not None else None,
                                    ctypes.addressof(bnr) if bnr is not None else None, _stream())
            _native.check(rc, "plx_conv_dgrad")
        if ctx.needs_input_grad[1]:
            cus = _num_cus(x.device)
            direct = ctx.wgrad is not None
            g = ctx.wgrad if direct else torch.empty(cout, k, k, cin, dtype=torch.float32, device=x.device)

            def wgrad():
                ws = torch.empty(_native.size("plx_conv", "plx_conv_wgrad_workspace", n, h, w, cin, cout, k, s, cus),
                                 dtype=torch.float32, device=x.device)
                rc = lib.plx_conv_wgrad(dy.data_ptr(), x.data_ptr(), g.data_ptr(), ws.data_ptr(), n, h, w, cin, cout,
                                        k, s, zero, cus, int(direct), _stream())
                _native.check(rc, "plx_conv_wgrad")
            if direct:  # only the optimizer reads the flat slot: overlap with the data-gradient chain
                side_stream.run(wgrad, (dy, x), x.device)
            else:
                wgrad()
            if not direct:
                dw = g.permute(0, 3, 1, 2)  # [co][ci][kh][kw] view with channels_last strides
        return dx, dw, None, None, None, None


def supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    k = conv.kernel_size[0]
    return (x.is_cuda and x.dim() == 4 and _bf16_context(x) and conv.kernel_size in ((1, 1), (3, 3))
            and conv.stride[0] == conv.stride[1] and conv.stride[0] in (1, 2) and conv.padding == (k // 2, k // 2)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0 and x.numel() > 0)


def conv_k(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, with_stats: bool = False,
           grad_box: GradMailbox = None, bn_link: bool = False) -> torch.Tensor:
    """``grad_box``: add the box's deferred gradient into dx (see ops.conv1x1.GradMailbox); ``bn_link``: dx is the
    complete gradient of ``x`` — serve the producing BatchNorm its backward partials (ops.conv1x1.BnLink)."""
    stats = None
    if with_stats:
        n, _, h, w = x.shape
        k = weight.shape[2]
        m, cout = n * _out(h, k, stride) * _out(w, k, stride), weight.shape[0]
        nblk = -(-m // nt_stats_rows(cout))
        stats = torch.empty(2 * nblk * cout, dtype=torch.float32, device=x.device)
    if grad_box is not None:
        grad_box.armed = True
        grad_box.s2k1 = stride == 2 and weight.shape[2] == 1
    y = _ConvK.apply(x, weight, stats, stride, grad_box, bn_link_of(x, bn_link))
    if stats is not None:
        y._plx_channel_stats = (stats, nblk)
    return y


class ConvKxK(nn.Conv2d):
    """``nn.Conv2d(in, out, k, stride, padding=k//2, bias=False)`` whose GPU path is the implicit-GEMM op above
    (1x1/3x3, stride 1/2); ``F.conv2d`` on CPU or for unsupported shapes."""

    def __init__(self, in_ch: int, out_ch: int, k: int = 3, stride: int = 1, native: bool = True,
                 bn_stats: bool = True):
        super().__init__(in_ch, out_ch, k, stride=stride, padding=k // 2, bias=False)
        self.native = native
        self.bn_stats = bn_stats

    def forward(self, x: torch.Tensor, grad_box: GradMailbox = None, bn_link: bool = False) -> torch.Tensor:
        if self.native and supported(x, self):
            return conv_k(x, self.weight, self.stride[0], with_stats=self.bn_stats and self.training,
                          grad_box=grad_box, bn_link=bn_link)
        return F.conv2d(x, self.weight, None, self.stride, self.padding)


def Conv3x3(in_ch: int, out_ch: int, stride: int = 1, native: bool = True, bn_stats: bool = True) -> ConvKxK:
    return ConvKxK(in_ch, out_ch, 3, stride, native, bn_stats)
