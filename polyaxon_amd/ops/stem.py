"""ResNet stem BatchNorm + ReLU + 3x3/s2/p1 max-pool as one op (csrc/bn_kernels.hip ``plx_stem_bn_pool_*``).

Unfused, the stem's 112x112x64 activation is the largest tensor of the step and it makes six HBM round trips
around the BatchNorm and the pool: stats read, apply read + write (+ ReLU mask), pool read, then in the backward
pool-bwd write, BN reduce read (dy, x, mask) and BN dx read (dy, x, mask) + write — ≈1.2 ms of a bs-256 step
(``profiles/r2_*``).  Fused:

* forward: statistics pass (as before) → one pass that applies scale/bias + ReLU while max-pooling, writing only the
  pooled tensor and a 1-byte window position per element;
* backward: two passes over x that gather the pooled gradient through the window positions, recompute the ReLU
  test, and reduce the BatchNorm partials (pass 1) / write dx (pass 2).

Same numerics as the unfused ops (the apply pass's bf16 value is what is pooled, ties keep the first maximum, the
gathered gradient is rounded to bf16 as the pool backward stores it); the GPU test compares the two paths.
"""
from __future__ import annotations

import torch

from polyaxon_amd.ops import _native
from polyaxon_amd.ops.bn_fused import _cl, _counters, _stream
from polyaxon_amd.ops.flat import direct_grad


class _StemBNReLUPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, ext=None):
        lib = _native.lib("plx_bn")
        x = _cl(x)
        n, c, h, w = x.shape
        oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        f32 = dict(dtype=torch.float32, device=x.device)
        stats = torch.empty(4 * c, **f32)  # mean | invstd | scale | bias
        if ext is not None:  # channel sums from the stem convolution's epilogue (StemConv): no statistics pass
            part, nblk = ext
            ws = torch.empty(_native.size("plx_bn", "plx_bn_l2_workspace", nblk, c), **f32)
        else:
            part, nblk = None, 0
            ws = torch.empty(_native.size("plx_bn", "plx_bn_workspace", n * h * w, c), **f32)
        y = torch.empty((n, c, oh, ow), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty(n * oh * ow * c, dtype=torch.uint8, device=x.device)
        rc = lib.plx_stem_bn_pool_forward(
            x.data_ptr(), y.data_ptr(), idx.data_ptr(), n, h, w, c, weight.data_ptr(), bias.data_ptr(), float(eps),
            float(momentum), running_mean.data_ptr(), running_var.data_ptr(), stats.data_ptr(),
            stats[c:].data_ptr(), stats[2 * c:].data_ptr(), ws.data_ptr(),
            part.data_ptr() if part is not None else None, int(nblk), _counters(x.device), _stream())
        _native.check(rc, "plx_stem_bn_pool_forward")
        ctx.save_for_backward(x, idx, weight, stats)
        gw, gb = direct_grad(weight), direct_grad(bias)
        ctx.direct = (gw, gb) if (gw is not None and gb is not None) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.lib("plx_bn")
        x, idx, weight, stats = ctx.saved_tensors
        n, c, h, w = x.shape
        dy = _cl(dy)
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        f32 = dict(dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        if ctx.direct is not None:
            dg_ptr, db_ptr, acc, dgb = ctx.direct[0].data_ptr(), ctx.direct[1].data_ptr(), 1, None
        else:
            dgb = torch.empty(2 * c, **f32)
            dg_ptr, db_ptr, acc = dgb.data_ptr(), dgb[c:].data_ptr(), 0
        coef = torch.empty(3 * c, **f32)
        ws = torch.empty(int(lib.plx_stem_bn_pool_bwd_workspace(n, h, w, c)), **f32)
        rc = lib.plx_stem_bn_pool_backward(
            dy.data_ptr(), idx.data_ptr(), x.data_ptr(), dx.data_ptr(), n, h, w, c, weight.data_ptr(),
            stats.data_ptr(), stats[c:].data_ptr(), stats[2 * c:].data_ptr(), dg_ptr, db_ptr, coef.data_ptr(),
            ws.data_ptr(), acc, _counters(x.device), _stream())
        _native.check(rc, "plx_stem_bn_pool_backward")
        dgamma = dgb[:c] if dgb is not None else None
        dbeta = dgb[c:] if dgb is not None else None
        return dx, dgamma, dbeta, None, None, None, None, None


def supported(x: torch.Tensor, bn, pool) -> bool:
    """Training-mode fused path: CUDA bf16 NHWC input, a fused ReLU BatchNorm with running stats, a native pool."""
    c = x.shape[1] if x.dim() == 4 else 0
    g = c // 8
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and c % 8 == 0 and 0 < g <= 256
            and 256 % g == 0 and bn.training and bn.fused and bn.act and not bn.residual
            and bn.running_mean is not None and getattr(pool, "native", False) and x.numel() > 0)


def stem_bn_relu_pool(x: torch.Tensor, bn, pool) -> torch.Tensor:
    """``pool(bn(x))`` for a ``BatchNormAct(act=True)`` and a ``MaxPool3s2``, fused when :func:`supported`."""
    if supported(x, bn, pool):
        ext = getattr(x, "_plx_channel_stats", None)
        return _StemBNReLUPool.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                                     ext)
    return pool(bn(x))


# ---------------------------------------------------------------------------------------------- stem convolution
class _StemConv(torch.autograd.Function):
    """7x7/s2/p3 3->64 convolution as an MFMA GEMM (csrc/conv_gemm.hip ``plx_stem_conv_fwd``): the input is packed
    into 16-byte super-pixels (2 pixels x 4 channels) and the epilogue emits the BatchNorm channel stats.  The weight
    gradient is the same window as a TN GEMM (``plx_stem_conv_wgrad``)."""

    @staticmethod
    def forward(ctx, x, weight, stats):
        conv = _native.lib("plx_conv")
        x = _cl(x.to(torch.bfloat16))
        n, _, h, w = x.shape
        cout = weight.shape[0]
        st = _stream()
        xp = torch.empty(n * h * (w // 2) * 8, dtype=torch.bfloat16, device=x.device)
        _native.check(conv.plx_stem_pack_input(x.data_ptr(), xp.data_ptr(), n, h, w, st), "plx_stem_pack_input")
        wp = torch.empty(cout, 256, dtype=torch.bfloat16, device=x.device)
        s = weight.stride()
        w32 = weight if weight.dtype == torch.float32 else weight.float()
        if w32 is not weight:
            s = w32.stride()
        _native.check(conv.plx_stem_pack_weight(w32.data_ptr(), s[0], s[1], s[2], s[3], wp.data_ptr(), cout, st),
                      "plx_stem_pack_weight")
        oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        y = torch.empty((n, cout, oh, ow), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        from polyaxon_amd.ops.conv1x1 import _zero_page
        rc = conv.plx_stem_conv_fwd(xp.data_ptr(), wp.data_ptr(), y.data_ptr(), n, h, w,
                                    _zero_page(x.device).data_ptr(),
                                    stats.data_ptr() if stats is not None else None, st)
        _native.check(rc, "plx_stem_conv_fwd")
        ctx.save_for_backward(xp, weight)
        ctx.shape = (n, h, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        """Weight gradient only (the input is data): the same super-pixel window as a TN GEMM over the output pixels
        (``plx_stem_conv_wgrad``), accumulated straight into the flat gradient slot when there is one.  It is the
        step's last backward op, so it runs on the main stream (nothing is left to overlap it with)."""
        xp, weight = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:
            return None, None, None
        conv = _native.lib("plx_conv")
        n, h, w = ctx.shape
        dy = _cl(dy.to(torch.bfloat16))
        from polyaxon_amd.ops.conv1x1 import _num_cus, _zero_page
        cus = _num_cus(dy.device)
        ws = torch.empty(int(conv.plx_stem_conv_wgrad_workspace(n, h, w, cus)), dtype=torch.float32, device=dy.device)
        slot = direct_grad(weight)
        out = slot if slot is not None else torch.empty_like(weight, dtype=torch.float32)
        st_ = out.stride()
        rc = conv.plx_stem_conv_wgrad(dy.data_ptr(), xp.data_ptr(), out.data_ptr(), st_[0], st_[1], st_[2], st_[3],
                                      ws.data_ptr(), n, h, w, _zero_page(dy.device).data_ptr(), cus,
                                      int(slot is not None), _stream())
        _native.check(rc, "plx_stem_conv_wgrad")
        return None, (None if slot is not None else out.to(weight.dtype)), None


def stem_conv_supported(x: torch.Tensor, conv) -> bool:
    from polyaxon_amd.ops.conv1x1 import _bf16_context

    return (x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and _bf16_context(x) and conv.out_channels == 64
            and conv.kernel_size == (7, 7) and conv.stride == (2, 2) and conv.padding == (3, 3)
            and conv.groups == 1 and conv.bias is None and x.shape[3] % 2 == 0 and x.numel() > 0)


class StemConv(torch.nn.Conv2d):
    """``nn.Conv2d(3, 64, 7, 2, 3, bias=False)`` whose GPU path is :class:`_StemConv`; in training its output carries
    ``_plx_channel_stats`` for the fused stem BatchNorm (``stem_bn_relu_pool``)."""

    def __init__(self, in_ch: int = 3, out_ch: int = 64, native: bool = True):
        super().__init__(in_ch, out_ch, 7, stride=2, padding=3, bias=False)
        self.native = native

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.native and stem_conv_supported(x, self):
            stats, nblk = None, 0
            if self.training:
                n, _, h, w = x.shape
                m = n * ((h - 1) // 2 + 1) * ((w - 1) // 2 + 1)
                nblk = -(-m // 256)
                stats = torch.empty(2 * nblk * self.out_channels, dtype=torch.float32, device=x.device)
            y = _StemConv.apply(x, self.weight, stats)
            if stats is not None:
                y._plx_channel_stats = (stats, nblk)
            return y
        return torch.nn.functional.conv2d(x, self.weight, None, self.stride, self.padding)
