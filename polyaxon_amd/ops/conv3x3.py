"""3x3 / stride-1 / pad-1 convolution on NHWC bf16 as implicit MFMA GEMMs (csrc/conv_gemm.hip).

13 of ResNet-50's 16 3x3 convolutions are stride 1.  Each pass reuses the 1x1-conv GEMM kernels with a
gathered operand: the reduction index is (tap, channel), and the operand row for a tap is the pixel shifted by
that tap, read straight from the NHWC activation by the per-lane global->LDS copy (out-of-image taps read a
zero page = the zero padding).  No im2col buffer is ever materialised.

* forward      ``y[m][co]  = Σ_tap,ci x[m+tap][ci]·W[co][tap][ci]``          (+ BN channel stats)
* data grad    ``dx[m][ci] = Σ_tap,co dy[m-tap][co]·W[co][tap][ci]``
* weight grad  ``dW[co][tap][ci] = Σ_m dy[m][co]·x[m+tap][ci]``  (fp32, split over m, slab-reduced)
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from polyaxon_amd.ops import _native
from polyaxon_amd.ops.conv1x1 import _bf16_context, _num_cus, _stream, _zero_page, nt_stats_rows


def weight_prep3(w: torch.Tensor):
    """fp32 [Cout][Cin][3][3] (any strides) -> (bf16 Wf [Cout][9][Cin], bf16 Wd [Cin][9][Cout])."""
    cout, cin = w.shape[0], w.shape[1]
    if w.dtype != torch.float32:
        w = w.float()
    wf = torch.empty(cout, 9, cin, dtype=torch.bfloat16, device=w.device)
    wd = torch.empty(cin, 9, cout, dtype=torch.bfloat16, device=w.device)
    st = w.stride()
    rc = _native.lib("plx_conv").plx_weight_prep3(w.data_ptr(), st[0], st[1], st[2], st[3], wf.data_ptr(),
                                                  wd.data_ptr(), cout, cin, _stream())
    _native.check(rc, "plx_weight_prep3")
    return wf, wd


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stats):
        lib = _native.lib("plx_conv")
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        wf, wd = weight_prep3(weight)
        y = torch.empty((n, cout, h, w), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        rc = lib.plx_conv3x3_fwd(x.data_ptr(), wf.data_ptr(), y.data_ptr(), n, h, w, cin, cout,
                                 _zero_page(x.device).data_ptr(), stats.data_ptr() if stats is not None else None,
                                 _stream())
        _native.check(rc, "plx_conv3x3_fwd")
        ctx.save_for_backward(x, wd)
        ctx.wshape = weight.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.lib("plx_conv")
        x, wd = ctx.saved_tensors
        n, cin, h, w = x.shape
        cout = ctx.wshape[0]
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        zero = _zero_page(x.device).data_ptr()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            rc = lib.plx_conv3x3_dgrad(dy.data_ptr(), wd.data_ptr(), dx.data_ptr(), n, h, w, cin, cout, zero,
                                       _stream())
            _native.check(rc, "plx_conv3x3_dgrad")
        if ctx.needs_input_grad[1]:
            cus = _num_cus(x.device)
            ws = torch.empty(int(lib.plx_conv3x3_wgrad_workspace(n, h, w, cin, cout, cus)), dtype=torch.float32,
                             device=x.device)
            g = torch.empty(cout, 3, 3, cin, dtype=torch.float32, device=x.device)  # [co][kh][kw][ci]
            rc = lib.plx_conv3x3_wgrad(dy.data_ptr(), x.data_ptr(), g.data_ptr(), ws.data_ptr(), n, h, w, cin, cout,
                                       zero, cus, 0, _stream())
            _native.check(rc, "plx_conv3x3_wgrad")
            dw = g.permute(0, 3, 1, 2)  # [co][ci][kh][kw] view with channels_last strides
        return dx, dw, None


def supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and _bf16_context(x) and conv.kernel_size == (3, 3)
            and conv.stride == (1, 1) and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.bias is None and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0 and x.numel() > 0)


def conv3x3(x: torch.Tensor, weight: torch.Tensor, with_stats: bool = False) -> torch.Tensor:
    stats = None
    if with_stats:
        n, _, h, w = x.shape
        m, cout = n * h * w, weight.shape[0]
        nblk = -(-m // nt_stats_rows(cout))
        stats = torch.empty(2 * nblk * cout, dtype=torch.float32, device=x.device)
    y = _Conv3x3.apply(x, weight, stats)
    if stats is not None:
        y._plx_channel_stats = (stats, nblk)
    return y


class Conv3x3(nn.Conv2d):
    """``nn.Conv2d(in, out, 3, stride, padding=1, bias=False)``; stride-1 instances on the GPU run the
    implicit-GEMM kernels above (strided ones stay on MIOpen)."""

    def __init__(self, in_ch: int, out_ch: int, stride: int = 1, native: bool = True, bn_stats: bool = True):
        super().__init__(in_ch, out_ch, 3, stride=stride, padding=1, bias=False)
        self.native = native
        self.bn_stats = bn_stats

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.native and supported(x, self):
            return conv3x3(x, self.weight, with_stats=self.bn_stats and self.training)
        return F.conv2d(x, self.weight, None, self.stride, self.padding)
