"""RMSNorm and LayerNorm: fused HIP kernels (csrc/rmsnorm.hip) for bf16 CUDA tensors (bf16 in and out, fp32
statistics and parameters), PyTorch composition otherwise."""
from __future__ import annotations

import os

import torch

from polyaxon_amd.ops import _native, side_stream

# the norms' parameter-gradient reduction on the side stream (ops/side_stream.py) when every parameter has a
# first-written flat slot and the side stream is in use this backward: only the optimizer / FlatDDP read those, after
# side_stream.join / fence
# (PLX_LM_WGRAD_STREAM=0: inline, as ops/lm.py)
_SIDE = os.environ.get("PLX_LM_WGRAD_STREAM", "1") != "0"


def rms_norm_reference(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    return y.to(x.dtype)


def _stream() -> int:
    return _native.current_stream()


def _param_grads(parts, params, d: int):
    """Column sums of the backward kernel's fp32 [nb, d] partial matrices (one per parameter) in one launch
    (csrc/rmsnorm.hip plx_partial_colsum).  A parameter with a direct fp32 flat-gradient slot (ops/flat.py) gets its
    sum written -- or, for a slot already written this step, accumulated -- there and None is returned for it (no
    autograd ``grad += g`` kernel; FlatDDP still sees the parameter through its post-accumulate hook); otherwise the sum is
    returned in the parameter's dtype."""
    from polyaxon_amd.ops.flat import direct_grad

    lib = _native.lib("plx_rms")
    dev = parts[0].device
    nb = parts[0].shape[0]
    outs, accs, ret = [], [], []
    for p in params:
        slot = direct_grad(p)
        if (slot is not None and slot.dtype == torch.float32 and slot.is_contiguous() and slot.numel() == d
                and slot.device == dev):
            accs.append(int(p._plx_flat.mark_written(slot)))
            outs.append(slot)
            ret.append(None)
        else:
            t = torch.empty(d, dtype=torch.float32, device=dev)
            accs.append(0)
            outs.append(t)
            ret.append(t)
    nz = len(parts)

    def reduce():  # workspace and tickets of the stream it runs on
        l2 = torch.empty(int(lib.plx_partial_colsum_workspace(nb, d, nz)), dtype=torch.float32, device=dev)
        cnt = _native.counters(dev, f"plx_partial_colsum:{_stream()}")
        _native.check(lib.plx_partial_colsum(parts[0].data_ptr(), parts[-1].data_ptr(), nb, d, nz, l2.data_ptr(),
                                             cnt.data_ptr(), outs[0].data_ptr(), outs[-1].data_ptr(), accs[0],
                                             accs[-1], _stream()), "plx_partial_colsum")
    # only beside side-stream work this backward already queued (GPT-2's weight gradients: +0.4 %,
    # r6_lm_norm_side_ab.jsonl); alone on it (Llama-3 8B, whose weight gradients stay inline) it cost 0.8 %
    # (r6_lm_norm_side_llama_ab.jsonl)
    if _SIDE and side_stream.busy(dev) and all(r is None for r in ret) and not any(accs):
        side_stream.run(reduce, parts, dev)
    else:
        reduce()
    return [r if r is None else r.to(p.dtype) for r, p in zip(ret, params)]


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps):
        lib = _native.lib("plx_rms")
        x = x.contiguous()
        d = x.shape[-1]
        rows = x.numel() // d
        y = torch.empty_like(x)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        w = weight.float().contiguous()
        _native.check(lib.plx_rms_forward(x.data_ptr(), w.data_ptr(), y.data_ptr(), rstd.data_ptr(), rows, d,
                                          float(eps), _stream()), "plx_rms_forward")
        ctx.save_for_backward(x, w, rstd)
        ctx.param = weight
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.lib("plx_rms")
        x, w, rstd = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        d = x.shape[-1]
        rows = x.numel() // d
        dx = torch.empty_like(x)
        nb = lib.plx_rms_bwd_blocks(rows)
        part = torch.empty((nb, d), dtype=torch.float32, device=x.device)
        _native.check(lib.plx_rms_backward(x.data_ptr(), w.data_ptr(), dy.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                           part.data_ptr(), rows, d, _stream()), "plx_rms_backward")
        return dx, _param_grads([part], [ctx.param], d)[0], None


class _AddRMSNorm(torch.autograd.Function):
    """(s, y) = (x + res, RMSNorm(x + res)) in one pass (csrc/rmsnorm.hip plx_add_rms_forward); backward: the norm's
    dx plus the residual gradient ds in one pass, returned for both x and res."""

    @staticmethod
    def forward(ctx, x, res, weight, eps):
        ctx.set_materialize_grads(False)
        lib = _native.lib("plx_rms")
        d = x.shape[-1]
        rows = x.numel() // d
        s, y = torch.empty_like(x), torch.empty_like(x)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        w = weight.float().contiguous()
        _native.check(lib.plx_add_rms_forward(x.data_ptr(), res.data_ptr(), w.data_ptr(), s.data_ptr(), y.data_ptr(),
                                              rstd.data_ptr(), rows, d, float(eps), _stream()), "plx_add_rms_forward")
        ctx.save_for_backward(s, w, rstd)
        ctx.param = weight
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        lib = _native.lib("plx_rms")
        s, w, rstd = ctx.saved_tensors
        if dy is None:
            return ds, ds, None, None
        d = s.shape[-1]
        rows = s.numel() // d
        dy = dy.contiguous().to(s.dtype)
        dx = torch.empty_like(s)
        part = torch.empty((lib.plx_rms_bwd_blocks(rows), d), dtype=torch.float32, device=s.device)
        if ds is None:
            _native.check(lib.plx_rms_backward(s.data_ptr(), w.data_ptr(), dy.data_ptr(), rstd.data_ptr(), dx.data_ptr(),
                                               part.data_ptr(), rows, d, _stream()), "plx_rms_backward")
        else:
            ds = ds.contiguous().to(s.dtype)
            _native.check(lib.plx_add_rms_backward(s.data_ptr(), w.data_ptr(), dy.data_ptr(), rstd.data_ptr(),
                                                   ds.data_ptr(), dx.data_ptr(), part.data_ptr(), rows, d, _stream()),
                          "plx_add_rms_backward")
        return dx, dx, _param_grads([part], [ctx.param], d)[0], None


def add_rms_norm(x: torch.Tensor, res: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5):
    """(s, y) = (x + res, RMSNorm(s)): the pre-norm residual add fused into the next RMSNorm for bf16 GPU rows; the
    separate add and :func:`rms_norm` otherwise."""
    if supported(x) and res.dtype == x.dtype and res.shape == x.shape and x.is_contiguous() and res.is_contiguous():
        return _AddRMSNorm.apply(x, res, weight, eps)
    s = x + res
    return s, rms_norm(s, weight, eps)


def supported(x: torch.Tensor) -> bool:
    d = x.shape[-1]
    return x.is_cuda and x.dtype == torch.bfloat16 and d % 8 == 0 and d <= 8192


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if x.is_cuda and x.dtype != torch.bfloat16 and torch.is_autocast_enabled("cuda"):
        x = x.to(torch.bfloat16)
    if supported(x):
        return _RMSNorm.apply(x, weight, eps)
    return rms_norm_reference(x, weight, eps)


def layer_norm_reference(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float) -> torch.Tensor:
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), weight, bias, eps)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        lib = _native.lib("plx_rms")
        x = x.contiguous()
        d = x.shape[-1]
        rows = x.numel() // d
        y = torch.empty_like(x)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        w, b = weight.float().contiguous(), bias.float().contiguous()
        _native.check(lib.plx_ln_forward(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                         rstd.data_ptr(), rows, d, float(eps), _stream()), "plx_ln_forward")
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.lib("plx_rms")
        x, w, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        d = x.shape[-1]
        rows = x.numel() // d
        dx = torch.empty_like(x)
        nb = lib.plx_ln_bwd_blocks(rows, d)
        part = torch.empty((2, nb, d), dtype=torch.float32, device=x.device)
        _native.check(lib.plx_ln_backward(x.data_ptr(), w.data_ptr(), dy.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                          dx.data_ptr(), part[0].data_ptr(), part[1].data_ptr(), rows, d, _stream()),
                      "plx_ln_backward")
        dw, db = _param_grads([part[0], part[1]], list(ctx.params), d)
        return dx, dw, db, None


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """LayerNorm over the last dim.  Under bf16 autocast the input is taken as bf16 and the output stays bf16 (what
    the next GEMM reads); the fused kernels need d % 8 == 0 and d <= 8192."""
    if x.is_cuda and x.dtype != torch.bfloat16 and torch.is_autocast_enabled("cuda"):
        x = x.to(torch.bfloat16)
    if supported(x):
        return _LayerNorm.apply(x, weight, bias, eps)
    return layer_norm_reference(x, weight, bias, eps)


class _AddLayerNorm(torch.autograd.Function):
    """(s, y) = (x + res, LayerNorm(x + res)) in one pass (csrc/rmsnorm.hip plx_add_ln_forward); backward: the norm's
    dx plus the residual gradient ds in one pass, returned for both x and res."""

    @staticmethod
    def forward(ctx, x, res, weight, bias, eps):
        ctx.set_materialize_grads(False)
        lib = _native.lib("plx_rms")
        d = x.shape[-1]
        rows = x.numel() // d
        s, y = torch.empty_like(x), torch.empty_like(x)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        w, b = weight.float().contiguous(), bias.float().contiguous()
        _native.check(lib.plx_add_ln_forward(x.data_ptr(), res.data_ptr(), w.data_ptr(), b.data_ptr(), s.data_ptr(),
                                             y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows, d, float(eps),
                                             _stream()), "plx_add_ln_forward")
        ctx.save_for_backward(s, w, mean, rstd)
        ctx.params = (weight, bias)
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        lib = _native.lib("plx_rms")
        s, w, mean, rstd = ctx.saved_tensors
        d = s.shape[-1]
        rows = s.numel() // d
        if dy is None:  # only the residual stream is used downstream
            return ds, ds, None, None, None
        dy = dy.contiguous().to(s.dtype)
        dx = torch.empty_like(s)
        nb = lib.plx_ln_bwd_blocks(rows, d)
        part = torch.empty((2, nb, d), dtype=torch.float32, device=s.device)
        if ds is None:
            _native.check(lib.plx_ln_backward(s.data_ptr(), w.data_ptr(), dy.data_ptr(), mean.data_ptr(),
                                              rstd.data_ptr(), dx.data_ptr(), part[0].data_ptr(), part[1].data_ptr(),
                                              rows, d, _stream()), "plx_ln_backward")
        else:
            ds = ds.contiguous().to(s.dtype)
            _native.check(lib.plx_add_ln_backward(s.data_ptr(), w.data_ptr(), dy.data_ptr(), mean.data_ptr(),
                                                  rstd.data_ptr(), ds.data_ptr(), dx.data_ptr(), part[0].data_ptr(),
                                                  part[1].data_ptr(), rows, d, _stream()), "plx_add_ln_backward")
        dw, db = _param_grads([part[0], part[1]], list(ctx.params), d)
        return dx, dx, dw, db, None


def add_layer_norm(x: torch.Tensor, res: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor,
                   eps: float = 1e-5):
    """(s, y) = (x + res, LayerNorm(s)): the pre-norm transformer's residual add fused into the next norm for bf16 GPU
    rows of d <= 1024 (one wave per row); the separate add and :func:`layer_norm` otherwise."""
    if (supported(x) and res.dtype == x.dtype and res.shape == x.shape and x.shape[-1] <= 1024 and x.is_contiguous()
            and res.is_contiguous()):
        return _AddLayerNorm.apply(x, res, weight, bias, eps)
    s = x + res
    return s, layer_norm(s, weight, bias, eps)


class LayerNorm(torch.nn.Module):
    """``nn.LayerNorm(d)`` (same parameter names, fp32 weight / bias) on the fused kernels for bf16 GPU inputs."""

    def __init__(self, d: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.normalized_shape = (d,)
        self.weight = torch.nn.Parameter(torch.ones(d))
        self.bias = torch.nn.Parameter(torch.zeros(d))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return layer_norm(x, self.weight, self.bias, self.eps)
