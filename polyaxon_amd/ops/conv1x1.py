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

import ctypes
from typing import Dict

import torch
import torch.nn as nn
import torch.nn.functional as F

from polyaxon_amd.ops import _native, side_stream, wcache
from polyaxon_amd.ops.flat import direct_grad

_ZERO: Dict[int, torch.Tensor] = {}
_CUS: Dict[int, int] = {}


def _zero_page(dev: torch.device) -> torch.Tensor:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    return _native.cached(_ZERO, idx, lambda: torch.zeros(256, dtype=torch.bfloat16, device=dev))


def _num_cus(dev: torch.device) -> int:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _CUS:
        _CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _CUS[idx]


def _stream() -> int:
    return _native.current_stream()


def nt_stats_rows(n: int) -> int:
    """Rows per block of plx_gemm_nt for an N-wide output (the granularity of its BN-stats partials)."""
    return _native.size("plx_conv", "plx_gemm_nt_rows_per_block", n)


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None, stats: torch.Tensor = None,
            add: torch.Tensor = None, bnr: "_native.BnBwdArgs" = None, add_mask: torch.Tensor = None) -> torch.Tensor:
    """out[M][N] = a[M][K] · b[N][K]ᵀ, bf16 (rows may be strided, K contiguous).  ``stats`` (fp32
    [2][ceil(M / nt_stats_rows(N))][N]) receives per-block channel sums and sums of squares of ``out``;
    ``add`` (bf16 [M][N]) is summed into the product in the epilogue, only where ``add_mask`` (a ReLU's 1-bit
    forward mask, uint8 [M*N/8]) is set when given; ``bnr`` (from :meth:`BnLink.request`) makes the epilogue
    emit the BatchNorm-backward partials of ``out``."""
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
    if add_mask is not None:
        assert add is not None and add.stride(0) == n and add_mask.dtype == torch.uint8 and add_mask.numel() == m * n // 8
    rc = _native.lib("plx_conv").plx_gemm_nt(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0),
                                             b.stride(0), out.stride(0), _zero_page(a.device).data_ptr(),
                                             stats.data_ptr() if stats is not None else None,
                                             add.data_ptr() if add is not None else None,
                                             add.stride(0) if add is not None else 0,
                                             add_mask.data_ptr() if add_mask is not None else None,
                                             ctypes.addressof(bnr) if bnr is not None else None, _stream())
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
    ws = torch.empty(_native.size("plx_conv", "plx_gemm_tn_workspace", m, n1, n2, cus), dtype=torch.float32,
                     device=a.device)
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
    residual gradient here and conv1's backward adds it in its data-gradient GEMM epilogue.  In a downsampling
    block the input feeds the downsample conv and conv1: conv1's backward ``put``s its data gradient and the
    downsample conv's dgrad adds it (in place, for the strided 1x1 whose GEMM only reaches the even pixels).
    The consumer runs first in the forward and ``arm``s the box only on the native path that will drain it;
    the producer defers only into an armed box and sets ``expect``.  Reverse-topological backward order (higher
    autograd sequence number first) runs the producer's backward before the consumer's; ``take`` fails loudly
    if that ever does not hold instead of silently dropping a gradient."""

    __slots__ = ("armed", "grad", "mask", "expect", "s2k1")

    def __init__(self):
        self.armed = False
        self.grad = None
        self.mask = None
        self.expect = False
        self.s2k1 = False  # the consumer is a stride-2 1x1 conv (its dgrad adds to the even-even pixels only)

    def put(self, g: torch.Tensor) -> None:
        if self.grad is not None:
            g = self._dense() + g
        self.grad, self.mask = g, None

    def put_masked(self, g: torch.Tensor, mask: torch.Tensor) -> None:
        """The gradient is ``g`` where the 1-bit ReLU ``mask`` (uint8, bit k of byte i = element 8i+k of the NHWC
        rows) is set, else 0: bn3's backward hands over its incoming gradient and forward mask instead of writing
        d_residual, and the consumer's dgrad epilogue applies the mask (``gemm_nt(add_mask=...)``)."""
        if self.grad is not None:
            self.put(unpack_relu_mask(g, mask))
            return
        self.grad, self.mask = g, mask

    def _dense(self) -> torch.Tensor:
        return self.grad if self.mask is None else unpack_relu_mask(self.grad, self.mask)

    def take(self):
        """(gradient, mask or None)."""
        g, m = self.grad, self.mask
        self.grad = self.mask = None
        if g is None and self.expect:
            raise RuntimeError("GradMailbox: the deferred gradient did not arrive before its consumer's backward")
        return g, m


def unpack_relu_mask(g: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """g * mask with the 1-bit mask expanded (channels_last NHWC element order)."""
    bits = (mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1
    n, c, h, w = g.shape
    keep = bits.view(n, h, w, c).permute(0, 3, 1, 2).to(g.dtype)
    return (g * keep).contiguous(memory_format=torch.channels_last)


class BnLink:
    """A fused BatchNorm(+ReLU)'s output → the convolution whose data gradient is that output's COMPLETE gradient.

    The BatchNorm forward attaches one to its output (``y._plx_bn_link``) holding what its backward reduction
    reads (x, ReLU mask, mean, invstd).  A consumer conv that the model marks as the sole gradient source
    (``bn_link=True``) ``request``s a partials buffer and its dgrad GEMM epilogue writes the per-block
    Σdz and Σdz·x̂ (csrc/conv_gemm.hip ``BnBwd``); the BatchNorm backward then skips its reduce pass."""

    __slots__ = ("x", "mask", "mean", "invstd", "part", "nblk", "_args", "affine", "split")

    def __init__(self, x=None, mask=None, mean=None, invstd=None):
        self.x, self.mask, self.mean, self.invstd = x, mask, mean, invstd
        self.affine = None  # deferred apply: fp32 [scale | bias] the consumer applies to the raw x
        self.part = None
        self.nblk = 0
        self._args = None
        self.split = 0  # > 0: the first of two GEMMs wrote rows [0, split); the strided 1x1 dgrad still owes the rest

    def _args_for(self, nblk_total: int, blk_off: int) -> "_native.BnBwdArgs":
        return _native.BnBwdArgs(self.x.data_ptr(), self.mask.data_ptr() if self.mask is not None else None,
                                 self.mean.data_ptr(), self.invstd.data_ptr(), self.part.data_ptr(), nblk_total,
                                 blk_off)

    def request(self, nblk: int) -> "_native.BnBwdArgs":
        c = self.x.shape[1]
        self.part = torch.empty(2 * nblk * c, dtype=torch.float32, device=self.x.device)
        self.nblk, self.split = nblk, 0
        self._args = self._args_for(nblk, 0)
        return self._args

    def request_split(self, nblk1: int, nblk2: int) -> "_native.BnBwdArgs":
        """ResNet downsampling block: x feeds conv1 (stride-1 1x1, dgrad deferred into the box) and the stride-2 1x1
        downsample conv (dgrad adds the box's gradient at the even-even pixels).  conv1's dgrad epilogue reduces
        the pixels the strided one never touches (rows [0, nblk1), even-even pixels skipped), and the strided
        dgrad the even-even ones with their final value (rows from nblk1, :meth:`request_rest`)."""
        n, c, h, w = self.x.shape
        self.part = torch.empty(2 * (nblk1 + nblk2) * c, dtype=torch.float32, device=self.x.device)
        self.nblk, self.split = nblk1 + nblk2, nblk1
        a = self._args_for(nblk1 + nblk2, 0)
        a.skip_h, a.skip_w = h, w
        self._args = a
        return a

    def request_rest(self) -> "_native.BnBwdArgs":
        a = self._args_for(self.nblk, self.split)
        self.split = 0
        self._args = a
        return a

    def take(self):
        part, nblk = self.part, self.nblk
        if self.split:  # the second GEMM never ran: the rows are incomplete, the BatchNorm reduces itself
            part, nblk = None, 0
        self.part, self._args, self.split = None, None, 0
        return part, nblk


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N,C,H,W] channels_last -> [N*H*W, C] view."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def bn_link_of(x: torch.Tensor, want: bool):
    link = getattr(x, "_plx_bn_link", None) if want else None
    return link if (link is not None and link.x is not None and link.x.shape == x.shape) else None


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stats, box, sink, link):
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ctx.box = box
        ctx.sink = sink if (sink is not None and sink.armed) else None
        if ctx.sink is not None:
            ctx.sink.expect = True
        # a sink nobody drains (its consumer is not on the native path) means x has another gradient source that
        # autograd adds: dx is then never x's whole gradient, so the link must not be served
        ctx.link = link if (sink is None or sink.armed) else None
        ctx.wgrad = direct_grad(weight)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        wb, wt = wcache.lookup(weight) or weight_prep(weight)
        y = torch.empty((n, cout, h, w), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        gemm_nt(_rows(x), wb, _rows(y), stats)
        ctx.save_for_backward(x, wt)
        ctx.wshape = weight.shape
        ctx.wdtype = weight.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        n, cin, h, w = x.shape
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        extra, extra_mask = ctx.box.take() if ctx.box is not None else (None, None)
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            if extra is not None and (extra.dtype != torch.bfloat16
                                      or not extra.is_contiguous(memory_format=torch.channels_last)):
                if extra_mask is not None:
                    extra, extra_mask = unpack_relu_mask(extra, extra_mask), None
                extra = extra.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            bnr = None
            # the link is only served when dx (+ the box's gradient) is the whole gradient of x: with a box, the
            # producer must actually have deferred into it; a sink means dx is only part of it -- except where the
            # sink's consumer is a strided 1x1, which only adds to the even-even pixels (BnLink.request_split)
            rows = nt_stats_rows(cin)
            if ctx.link is not None and ctx.sink is None and (ctx.box is None or extra is not None):
                bnr = ctx.link.request(-(-(n * h * w) // rows))
            elif ctx.link is not None and ctx.sink is not None and ctx.sink.s2k1 and extra is None:
                bnr = ctx.link.request_split(-(-(n * h * w) // rows), -(-(n * ((h + 1) // 2) * ((w + 1) // 2)) // rows))
            gemm_nt(_rows(dy), wt, _rows(dx), add=_rows(extra) if extra is not None else None, bnr=bnr,
                    add_mask=extra_mask)
            if ctx.sink is not None:  # the downsample conv's dgrad adds this gradient in its epilogue
                ctx.sink.put(dx)
                dx = None
        if ctx.needs_input_grad[1]:
            cout = ctx.wshape[0]
            if ctx.wgrad is not None:  # accumulate into the flat gradient slot, autograd sees no weight grad
                slot = ctx.wgrad.as_strided((cout, cin), (cin, 1))
                side_stream.run(lambda: gemm_tn(_rows(dy), _rows(x), out=slot, accumulate=True), (dy, x), x.device)
            else:
                dw = gemm_tn(_rows(dy), _rows(x)).view(ctx.wshape).to(ctx.wdtype)
        return dx, dw, None, None, None, None


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
            grad_box: "GradMailbox" = None, grad_sink: "GradMailbox" = None, bn_link: bool = False) -> torch.Tensor:
    """With ``with_stats`` the output carries ``_plx_channel_stats`` = (fp32 [2][nblk][Cout] per-block channel
    sums / sums of squares, nblk), which a following fused BatchNorm uses instead of its own stats pass.
    ``grad_box``: add the box's deferred gradient into dx; ``grad_sink``: defer dx into that (armed) box;
    ``bn_link``: dx (+ ``grad_box``'s gradient) is the complete gradient of ``x`` — serve the BatchNorm that
    produced ``x`` its backward partials (:class:`BnLink`)."""
    stats = None
    if with_stats:
        n, _, h, w = x.shape
        m, cout = n * h * w, weight.shape[0]
        nblk = -(-m // nt_stats_rows(cout))
        stats = torch.empty(2 * nblk * cout, dtype=torch.float32, device=x.device)
    if grad_box is not None:
        grad_box.armed = True
    y = _Conv1x1.apply(x, weight, stats, grad_box, grad_sink, bn_link_of(x, bn_link))
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

    def forward(self, x: torch.Tensor, grad_box: GradMailbox = None, grad_sink: GradMailbox = None,
                bn_link: bool = False) -> torch.Tensor:
        if self.native and supported(x, self):
            return conv1x1(x, self.weight, with_stats=self.bn_stats and self.training, grad_box=grad_box,
                           grad_sink=grad_sink, bn_link=bn_link)
        return F.conv2d(x, self.weight, None, self.stride)
