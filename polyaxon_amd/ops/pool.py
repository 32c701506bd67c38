"""3x3/stride-2/pad-1 max pool on NHWC bf16 (the ResNet stem pool) — csrc/pool_kernels.hip.

The forward keeps a 1-byte window position per element instead of PyTorch's int64 index; the backward is a
gather (each input pixel sums the dy of the <= 4 windows whose argmax it is), so it needs no zero-fill pass.
"""
from __future__ import annotations


import torch
import torch.nn as nn
import torch.nn.functional as F

from polyaxon_amd.ops import _native


def _stream() -> int:
    return _native.current_stream()


class _MaxPool3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous(memory_format=torch.channels_last)
        n, c, h, w = x.shape
        oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        y = torch.empty((n, c, oh, ow), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty(n * oh * ow * c, dtype=torch.uint8, device=x.device)
        rc = _native.lib("plx_pool").plx_maxpool3s2_forward(x.data_ptr(), y.data_ptr(), idx.data_ptr(), n, h, w, c,
                                                            _stream())
        _native.check(rc, "plx_maxpool3s2_forward")
        ctx.save_for_backward(idx)
        ctx.shape = (n, c, h, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        n, c, h, w = ctx.shape
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty((n, c, h, w), dtype=torch.bfloat16, device=dy.device, memory_format=torch.channels_last)
        rc = _native.lib("plx_pool").plx_maxpool3s2_backward(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), n, h, w, c,
                                                             _stream())
        _native.check(rc, "plx_maxpool3s2_backward")
        return dx


def supported(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0 and x.numel() > 0


class MaxPool3s2(nn.MaxPool2d):
    """``nn.MaxPool2d(3, 2, 1)`` with the HIP NHWC bf16 path on the GPU."""

    def __init__(self, native: bool = True):
        super().__init__(3, stride=2, padding=1)
        self.native = native

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.native and supported(x):
            return _MaxPool3s2.apply(x)
        return F.max_pool2d(x, 3, 2, 1)


class _GlobalAvgPoolNHWC(torch.autograd.Function):
    """Mean over H x W of a channels_last [N, C, H, W] tensor -> [N, C], with the backward written straight in the
    input's NHWC layout.  Autograd's own x.mean((2, 3)) backward expanded the gradient into an NCHW-strided tensor,
    which the BatchNorm backward then had to transpose into channels_last: a generic strided-copy kernel of ~80 us
    plus the division pass, ~100 us per ResNet-50 step at the forward -> backward hand-off (scripts/trace_window.py).
    bf16 on the GPU: one HIP kernel each way (csrc/pool_kernels.hip plx_gap_forward / plx_gap_backward: 16-byte
    rows, fp32 sums); otherwise torch ops on the NHWC view."""

    @staticmethod
    def forward(ctx, x):
        n, c, h, w = x.shape
        ctx.shape = (n, c, h, w)
        if x.is_cuda and x.dtype == torch.bfloat16 and c % 8 == 0 and x.data_ptr() % 16 == 0:
            y = torch.empty((n, c), dtype=x.dtype, device=x.device)
            _native.check(_native.lib("plx_pool").plx_gap_forward(x.data_ptr(), y.data_ptr(), n, h * w, c, _stream()),
                          "plx_gap_forward")
            return y
        return x.permute(0, 2, 3, 1).reshape(n, h * w, c).mean(1)  # a contiguous NHWC view: column means

    @staticmethod
    def backward(ctx, g):
        n, c, h, w = ctx.shape
        if g.is_cuda and g.dtype == torch.bfloat16 and c % 8 == 0:
            g = g.contiguous()
            dx = torch.empty((n, c, h, w), dtype=g.dtype, device=g.device, memory_format=torch.channels_last)
            _native.check(_native.lib("plx_pool").plx_gap_backward(g.data_ptr(), dx.data_ptr(), n, h * w, c,
                                                                   _stream()), "plx_gap_backward")
            return dx
        dx = (g / (h * w)).unsqueeze(1).expand(n, h * w, c).contiguous()  # one broadcast write, NHWC
        return dx.view(n, h, w, c).permute(0, 3, 1, 2)  # channels_last [N, C, H, W], no copy


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """x.mean((2, 3)) for a 4-D tensor; the NHWC-native autograd function when x is channels_last (and not NCHW
    contiguous, i.e. C > 1 and H * W > 1)."""
    if x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last):
        return _GlobalAvgPoolNHWC.apply(x)
    return x.mean((2, 3))
