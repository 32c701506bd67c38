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


def nt_stats_rows(n: int) -> int:
    """Rows per block of plx_gemm_nt for an N-wide output (the granularity of its BN-stats partials)."""
    return int(_native.lib("plx_conv").plx_gemm_nt_rows_per_block(n))


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None, stats: torch.Tensor = None,
            add: torch.Tensor = None) -> torch.Tensor:
    """out[M][N] = a[M][K] · b[N][K]ᵀ, bf16 (rows may be strided, K contiguous).  ``stats`` (fp32
    [2][ceil(M / nt_stats_rows(N))][N]) receives per-block channel sums and sums of squares of ``out``;
    ``add`` (bf16 [M][N]) is summed into the product in the epilogue."""
    m, k = a.shape
    n = b.shape[0]
    if out is None:
        out = torch.empty(m, n, dtype=torch.bfloat16, device=a.device)
    assert a.stride(1) == 1 and b.stride(1) == 1 and out.stride(1) == 1 and b.shape[1] == k
    assert a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0
    if stats is not None:
        nblk = -(-m // nt_stats_rows(n))
        assert stats.dtype == torch.float32 and stats.is_contiguous() and stats.numel() >= 2 * nblk * n
    if add is not None:
        assert add.shape == (m, n) and add.stride(1) == 1 and add.dtype == torch.bfloat16 and add.data_ptr() % 16 == 0
    rc = _native.lib("plx_conv").plx_gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0),
                                             b.stride(0), out.stride(0), _zero_page(a.device).data_ptr(),
                                             stats.data_ptr() if stats is not None else None,
                                             add.data_ptr() if add is not None else None,
                                             add.stride(0) if add is not None else 0, _stream())
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


class GradMailbox:
    """Hands a gradient from a later op's backward to an earlier op's backward that consumes the same tensor.

    In a ResNet identity block the block input feeds conv1 and the residual add of bn3; autograd would sum the
    two gradients with a separate bf16 add over the whole activation.  Instead bn3's backward ``put``s its
    residual gradient here and conv1's backward adds it in its data-gradient GEMM epilogue.  conv1 runs before
    bn3 in the forward, so it ``arm``s the box only when it took the native path that will consume it; bn3
    defers its gradient only into an armed box.  Reverse-topological backward order guarantees bn3's backward
    (later in the forward) runs before conv1's."""

    __slots__ = ("armed", "grad")

    def __init__(self):
        self.armed = False
        self.grad = None

    def put(self, g: torch.Tensor) -> None:
        self.grad = g if self.grad is None else self.grad + g

    def take(self):
        g, self.grad = self.grad, None
        return g


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N,C,H,W] channels_last -> [N*H*W, C] view."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stats, box):
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ctx.box = box
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        wb, wt = weight_prep(weight)
        y = torch.empty((n, cout, h, w), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        gemm_nt(_rows(x), wb, _rows(y), stats)
        ctx.save_for_backward(x, wt)
        ctx.wshape = weight.shape
        ctx.wdtype = weight.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        extra = ctx.box.take() if ctx.box is not None else None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            if extra is not None:
                extra = extra.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            gemm_nt(_rows(dy), wt, _rows(dx), add=_rows(extra) if extra is not None else None)
        if ctx.needs_input_grad[1]:
            dw = gemm_tn(_rows(dy), _rows(x)).view(ctx.wshape).to(ctx.wdtype)
        return dx, dw, None, None


def _bf16_context(x: torch.Tensor) -> bool:
    """bf16 activations, or fp32 ones inside a bf16 autocast region (an fp32 network keeps fp32 convs)."""
    if x.dtype == torch.bfloat16:
        return True
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


def supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and _bf16_context(x) and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.groups == 1 and conv.bias is None
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0 and x.numel() > 0)


def conv1x1(x: torch.Tensor, weight: torch.Tensor, with_stats: bool = False,
            grad_box: "GradMailbox" = None) -> torch.Tensor:
    """With ``with_stats`` the output carries ``_plx_channel_stats`` = (fp32 [2][nblk][Cout] per-block channel
    sums / sums of squares, nblk), which a following fused BatchNorm uses instead of its own stats pass."""
    stats = None
    if with_stats:
        n, _, h, w = x.shape
        m, cout = n * h * w, weight.shape[0]
        nblk = -(-m // nt_stats_rows(cout))
        stats = torch.empty(2 * nblk * cout, dtype=torch.float32, device=x.device)
    if grad_box is not None:
        grad_box.armed = True
    y = _Conv1x1.apply(x, weight, stats, grad_box)
    if stats is not None:
        y._plx_channel_stats = (stats, nblk)
    return y


class Conv1x1(nn.Conv2d):
    """``nn.Conv2d(in, out, 1, bias=False)`` whose GPU path is the MFMA GEMM op above (same parameter, same
    init; falls back to ``F.conv2d`` on CPU or for unsupported channel counts)."""

    def __init__(self, in_ch: int, out_ch: int, stride: int = 1, native: bool = True, bn_stats: bool = True):
        super().__init__(in_ch, out_ch, 1, stride=stride, bias=False)
        self.native = native
        self.bn_stats = bn_stats  # emit channel stats for the BatchNorm that follows (training only)

    def forward(self, x: torch.Tensor, grad_box: GradMailbox = None) -> torch.Tensor:
        if self.native and supported(x, self):
            return conv1x1(x, self.weight, with_stats=self.bn_stats and self.training, grad_box=grad_box)
        return F.conv2d(x, self.weight, None, self.stride)
