"""Autograd wrapper for the fused NHWC bf16 BatchNorm(+add)(+ReLU) HIP kernels (csrc/bn_kernels.hip).

Forward (training): stats → finalize (mean/invstd/scale/bias + running-stat update) → apply.
Backward: reduce (Σdz, Σdz·x̂) → finalize (dγ, dβ, dx coefficients) → dx (+ d_residual) in one pass.
With ReLU the forward also writes a 1-bit-per-element mask (1/16 of ``y``); the backward reads it instead of
``y``, one fewer full activation stream in each of its two passes.
"""
from __future__ import annotations

import ctypes

from typing import Optional

import torch

from polyaxon_amd.ops import _native
from polyaxon_amd.ops.conv1x1 import BnLink
from polyaxon_amd.ops.flat import direct_grad


def _stream() -> int:
    return _native.current_stream()


_COUNTERS = {}


def _counters(dev: torch.device):
    """Zeroed ticket counters of the one-launch reduce + finalize (csrc/bn_kernels.hip ``reduce_l2_last``), one
    array per (device, stream): launches sharing it are stream-ordered and each leaves it zeroed again."""
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    # >= ceil(2048 / 64) groups
    return _native.cached(_COUNTERS, key, lambda: torch.zeros(64, dtype=torch.int32, device=dev)).data_ptr()


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


def supported(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dtype != torch.bfloat16 or x.dim() != 4:
        return False
    c = x.shape[1]
    g = c // 8
    return c % 8 == 0 and g > 0 and (g & (g - 1)) == 0 and x.numel() > 0


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, momentum, eps, relu, ext=None, box=None,
                link=None, rlink=None, defer=False):
        lib = _native.lib("plx_bn")
        x = _cl(x)
        n, c, h, w = x.shape
        m = n * h * w
        ws = _native.size("plx_bn", "plx_bn_workspace", m, c)
        if ws < 0:
            raise RuntimeError("unsupported channel count for fused BN")
        f32 = dict(dtype=torch.float32, device=x.device)
        # defer: no apply pass -- the output aliases x and its only consumer (the residual add of a fused
        # BatchNorm) applies scale/bias on the fly (link.affine); the backward is unchanged
        defer = bool(defer) and not relu and residual is None and link is not None
        y = None if defer else torch.empty_like(x, memory_format=torch.channels_last)
        yp = y.data_ptr() if y is not None else None
        stats = torch.empty(4 * c, **f32)  # mean | invstd | scale | bias
        res_sb = None
        if residual is not None:
            rl = getattr(residual, "_plx_bn_link", None)
            if rl is not None and rl.affine is not None and getattr(residual, "_plx_deferred", False):
                res_sb = rl.affine
        res = _cl(residual) if residual is not None else None
        rsp = res_sb.data_ptr() if res_sb is not None else None
        rm = running_mean.data_ptr() if running_mean is not None else None
        rv = running_var.data_ptr() if running_var is not None else None
        mask = torch.empty(m * c // 8, dtype=torch.uint8, device=x.device) if relu else None
        mp = mask.data_ptr() if mask is not None else None
        if ext is not None:
            # channel sums came from the producing conv's GEMM epilogue: no stats pass over x
            part, nblk = ext
            l2 = torch.empty(_native.size("plx_bn", "plx_bn_l2_workspace", nblk, c), **f32)
            rc = lib.plx_bn_forward_from_partials(
                x.data_ptr(), res.data_ptr() if res is not None else None, yp, m, c, weight.data_ptr(),
                bias.data_ptr(), float(eps), float(momentum), rm, rv, stats.data_ptr(), stats[c:].data_ptr(),
                stats[2 * c:].data_ptr(), part.data_ptr(), nblk, l2.data_ptr(), mp, int(relu), rsp,
                _counters(x.device), _stream())
            _native.check(rc, "plx_bn_forward_from_partials")
        else:
            partials = torch.empty(ws, **f32)
            rc = lib.plx_bn_forward(
                x.data_ptr(), res.data_ptr() if res is not None else None, yp, m, c,
                weight.data_ptr(), bias.data_ptr(), float(eps), float(momentum), rm, rv,
                stats.data_ptr(), stats[c:].data_ptr(), stats[2 * c:].data_ptr(), partials.data_ptr(), mp, int(relu),
                rsp, _counters(x.device), _stream())
            _native.check(rc, "plx_bn_forward")
        ctx.save_for_backward(x, mask, weight, stats)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.box = box if (box is not None and box.armed and residual is not None) else None
        if ctx.box is not None:
            ctx.box.expect = True
        ctx.ws = ws
        # direct gradients: dgamma / dbeta accumulate into the flat gradient slots (ops.flat.direct_grad)
        gw, gb = direct_grad(weight), direct_grad(bias)
        ctx.direct = (gw, gb) if (gw is not None and gb is not None) else None
        # the consumer conv may produce this BN's backward partials in its dgrad epilogue (ops.conv1x1.BnLink)
        ctx.link = link
        if link is not None:
            link.x, link.mask, link.mean, link.invstd = x, mask, stats[:c], stats[c:2 * c]
            if defer:
                link.affine = stats[2 * c:]
        # rlink: the residual came from a fused BatchNorm whose output nothing else consumes (a downsampling branch):
        # d_residual is that BatchNorm's whole gradient, so the dx pass below reduces its backward partials too
        ctx.rlink = rlink if (rlink is not None and residual is not None and rlink.x is not None
                              and rlink.x.shape == x.shape and ctx.box is None) else None
        if defer:
            return x.view_as(x)  # the raw input; bn_act marks it _plx_deferred
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.lib("plx_bn")
        x, mask, weight, stats = ctx.saved_tensors
        n, c, h, w = x.shape
        m = n * h * w
        dy = _cl(dy)
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        f32 = dict(dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        # identity block: the residual's gradient dz = dy * mask is not written here; dy and the mask ride into
        # conv1's dgrad epilogue (GradMailbox.put_masked), which adds them
        masked_box = ctx.box is not None and ctx.relu and mask is not None
        dres = (torch.empty_like(x, memory_format=torch.channels_last)
                if ctx.has_res and not masked_box else None)
        if ctx.direct is not None:
            dg_ptr, db_ptr, acc = ctx.direct[0].data_ptr(), ctx.direct[1].data_ptr(), 1
            dgb = None
        else:
            dgb = torch.empty(2 * c, **f32)
            dg_ptr, db_ptr, acc = dgb.data_ptr(), dgb[c:].data_ptr(), 0
        coef = torch.empty(3 * c, **f32)
        part, nblk = ctx.link.take() if ctx.link is not None else (None, 0)
        rb = None
        if ctx.rlink is not None and dres is not None:
            rl = ctx.rlink
            nblk2 = _native.size("plx_bn", "plx_bn_dx_blocks", m, c)
            rl.part = torch.empty(2 * nblk2 * c, **f32)
            rl.nblk = nblk2
            rb = _native.ResBnArgs(rl.x.data_ptr(), rl.mask.data_ptr() if rl.mask is not None else None,
                                   rl.mean.data_ptr(), rl.invstd.data_ptr(), rl.part.data_ptr())
        rbp = ctypes.addressof(rb) if rb is not None else None
        if part is not None:  # the consumer's dgrad epilogue already reduced dz and dz*xhat per block
            l2 = torch.empty(_native.size("plx_bn", "plx_bn_l2_workspace", nblk, c), **f32)
            rc = lib.plx_bn_backward_from_partials(
                x.data_ptr(), mask.data_ptr() if mask is not None else None, dy.data_ptr(), dx.data_ptr(),
                dres.data_ptr() if dres is not None else None, m, c, weight.data_ptr(), stats.data_ptr(),
                stats[c:].data_ptr(), dg_ptr, db_ptr, coef.data_ptr(), part.data_ptr(), nblk, l2.data_ptr(),
                int(ctx.relu), acc, rbp, _counters(x.device), _stream())
            _native.check(rc, "plx_bn_backward_from_partials")
        else:
            partials = torch.empty(ctx.ws, **f32)
            rc = lib.plx_bn_backward(
                x.data_ptr(), mask.data_ptr() if mask is not None else None, dy.data_ptr(), dx.data_ptr(),
                dres.data_ptr() if dres is not None else None, m, c, weight.data_ptr(), stats.data_ptr(),
                stats[c:].data_ptr(), dg_ptr, db_ptr, coef.data_ptr(), partials.data_ptr(), int(ctx.relu), acc,
                rbp, _counters(x.device), _stream())
            _native.check(rc, "plx_bn_backward")
        if ctx.box is not None:  # the residual's gradient rides into conv1's dgrad epilogue (ops.conv1x1)
            if masked_box:
                ctx.box.put_masked(dy, mask)
            else:
                ctx.box.put(dres)
            dres = None
        dgamma = dgb[:c] if dgb is not None else None
        dbeta = dgb[c:] if dgb is not None else None
        return dx, dgamma, dbeta, None, None, dres, None, None, None, None, None, None, None, None


class _Materialize(torch.autograd.Function):
    """A deferred BatchNorm output (the raw input plus its pending scale/bias) made real for a consumer that does
    not apply the affine itself; the gradient passes through unchanged (it is the BatchNorm output's gradient)."""

    @staticmethod
    def forward(ctx, t, sb):
        c = t.shape[1]
        return (t.float() * sb[:c].view(1, c, 1, 1) + sb[c:].view(1, c, 1, 1)).to(t.dtype).contiguous(
            memory_format=torch.channels_last)

    @staticmethod
    def backward(ctx, g):
        return g, None


def materialize(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """The real value of a possibly deferred BatchNorm output (:func:`bn_act` with ``defer_apply``)."""
    if t is None or not getattr(t, "_plx_deferred", False):
        return t
    return _Materialize.apply(t, t._plx_bn_link.affine)


def bn_act(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, running_mean: Optional[torch.Tensor],
           running_var: Optional[torch.Tensor], training: bool, momentum: float, eps: float,
           residual: Optional[torch.Tensor], act: bool, ext_stats=None, residual_grad_box=None,
           residual_link: bool = False, defer_apply: bool = False) -> torch.Tensor:
    """``ext_stats`` = (fp32 [2][nblk][C] channel sums / sums of squares of ``x``, nblk) from the op that
    produced ``x`` (the 1x1-conv GEMM epilogue); training mode then skips the stats pass.  ``residual_link``:
    ``residual`` is the output of a fused BatchNorm that nothing else consumes; its backward partials are then
    reduced by this op's dx pass.  ``defer_apply`` (training, no activation, no residual): skip the apply pass
    and return ``x`` itself marked ``_plx_deferred``; the fused BatchNorm that takes it as its residual applies
    the scale/bias while adding (a ResNet downsampling branch: ~0.3 ms of a bs-256 step), any other consumer
    must call :func:`materialize` first."""
    if residual is not None and residual.dtype != x.dtype:
        residual = residual.to(x.dtype)
    if training:
        link = BnLink()
        rlink = getattr(residual, "_plx_bn_link", None) if (residual_link and residual is not None) else None
        defer = bool(defer_apply) and not act and residual is None
        y = _BNAct.apply(x, weight, bias, running_mean, running_var, residual, momentum, eps, act, ext_stats,
                         residual_grad_box, link, rlink, defer)
        y._plx_bn_link = link
        if defer:
            y._plx_deferred = True
        return y
    residual = materialize(residual)
    # inference: fold running stats into scale/bias, one apply pass
    lib = _native.lib("plx_bn")
    x = _cl(x)
    n, c, h, w = x.shape
    inv = torch.rsqrt(running_var.float() + eps)
    scale = weight.float() * inv
    sb = torch.cat([scale, bias.float() - running_mean.float() * scale]).contiguous()
    y = torch.empty_like(x, memory_format=torch.channels_last)
    res = _cl(residual) if residual is not None else None
    rc = lib.plx_bn_apply(x.data_ptr(), res.data_ptr() if res is not None else None, y.data_ptr(), n * h * w, c,
                          sb.data_ptr(), int(act), _stream())
    _native.check(rc, "plx_bn_apply")
    return y
