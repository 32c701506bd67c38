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
