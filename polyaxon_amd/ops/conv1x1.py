"""Stride-1 1x1 convolution on NHWC bf16 activations as three MFMA GEMMs (csrc/conv_gemm.hip).

ResNet-50's bottleneck conv1/conv3 are 33 of its 53 convolutions.  On channels_last activations each pass is
a plain GEMM over the M = N·H·W pixel rows, so instead of MIOpen's implicit-GEMM convolutions (which zero
their output with an extra SubTensorOp launch before every call and accumulate the weight gradient in a
fp32 workspace that is then cast to bf16 and added into the fp32 master gradient) the op runs:

* forward     ``y = x · Wᵀ``            — ``plx_gemm_nt`` (bf16 out)
* data grad   ``dx = dy · W``           — ``plx_gemm_nt`` against the pre-transposed bf16 ``Wᵀ``
* weight grad ``dW = dyᵀ · x``           — ``plx_gemm_tn`` split over M, accumulated in fp32 directly

The fp32 master weight is cast to bf16 (and transposed) once per forward by ``plx_weight_prep``; the weight
gradient comes back in fp32, so autocast's bf16 weight copy and its backward cast disappear too.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn as nn
import torch.nn.functional as F

from polyaxon_amd.ops import _native

_ZERO: Dict[int, torch.Tensor] = {}
_CUS: Dict[int, int] = {}


def _zero_page(dev: torch.device) -> torch.Tensor:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    z = _ZERO.get(idx)
    if z is None:
        z = _ZERO[idx] = torch.zeros(256, dtype=torch.bfloat16, device=dev)
    return z


def _num_cus(dev: torch.device) -> int:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _CUS:
        _CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _CUS[idx]


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """out[M][N] = a[M][K] · b[N][K]ᵀ, bf16 (rows may be strided, K contiguous)."""
    m, k = a.shape
    n = b.shape[0]
    if out is None:
        out = torch.empty(m, n, dtype=torch.bfloat16, device=a.device)
    assert a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1 and b.shape[1] == k
    assert a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and out.data_ptr() % 8 == 0
    rc = _native.lib("plx_conv").plx_gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0),
                                             b.stride(0), out.stride(0), _zero_page(a.device).data_ptr(), _stream())
    _native.check(rc, "plx_gemm_nt")
    return out


def gemm_tn(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None, accumulate: bool = False) -> torch.Tensor:
    """out[N1][N2] (fp32) = a[M][N1]ᵀ · b[M][N2]  (``+=`` with ``accumulate``)."""
    m, n1 = a.shape
    n2 = b.shape[1]
    if out is None:
        out = torch.empty(n1, n2, dtype=torch.float32, device=a.device)
        accumulate = False
    assert a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1 and b.shape[0] == m
    assert a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0
    lib = _native.lib("plx_conv")
    cus = _num_cus(a.device)
    ws = torch.empty(int(lib.plx_gemm_tn_workspace(m, n1, n2, cus)), dtype=torch.float32, device=a.device)
    rc = lib.plx_gemm_tn(a.data_ptr(), b.data_ptr(), out.data_ptr(), ws.data_ptr(), m, n1, n2, a.stride(0),
                         b.stride(0), out.stride(0), _zero_page(a.device).data_ptr(), cus, int(accumulate),
                         _stream())
    _native.check(rc, "plx_gemm_tn")
    return out


def weight_prep(w: torch.Tensor):
    """fp32 [Cout][Cin] -> (bf16 W, bf16 Wᵀ)."""
    cout, cin = w.shape[0], w.shape[1]
    wb = torch.empty(cout, cin, dtype=torch.bfloat16, device=w.device)
    wt = torch.empty(cin, cout, dtype=torch.bfloat16, device=w.device)
    w32 = w.reshape(cout, cin)
    if w32.dtype != torch.float32 or not w32.is_contiguous():
        w32 = w32.float().contiguous()
    rc = _native.lib("plx_conv").plx_weight_prep(w32.data_ptr(), wb.data_ptr(), wt.data_ptr(), cout, cin, _stream())
    _native.check(rc, "plx_weight_prep")
    return wb, wt


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N,C,H,W] channels_last -> [N*H*W, C] view."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        wb, wt = weight_prep(weight)
        y = torch.empty((n, cout, h, w), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        gemm_nt(_rows(x), wb, _rows(y))
        ctx.save_for_backward(x, wt)
        ctx.wshape = weight.shape
        ctx.wdtype = weight.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            gemm_nt(_rows(dy), wt, _rows(dx))
        if ctx.needs_input_grad[1]:
            dw = gemm_tn(_rows(dy), _rows(x)).view(ctx.wshape).to(ctx.wdtype)
        return dx, dw


def supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.groups == 1 and conv.bias is None
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0 and x.numel() > 0)


def conv1x1(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    return _Conv1x1.apply(x, weight)


class Conv1x1(nn.Conv2d):
    """``nn.Conv2d(in, out, 1, bias=False)`` whose GPU path is the MFMA GEMM op above (same parameter, same
    init; falls back to ``F.conv2d`` on CPU or for unsupported channel counts)."""

    def __init__(self, in_ch: int, out_ch: int, stride: int = 1, native: bool = True):
        super().__init__(in_ch, out_ch, 1, stride=stride, bias=False)
        self.native = native

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.native and supported(x, self):
            return conv1x1(x, self.weight)
        return F.conv2d(x, self.weight, None, self.stride)
