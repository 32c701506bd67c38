"""RMSNorm and LayerNorm: fused HIP kernels (csrc/rmsnorm.hip) for bf16 CUDA tensors (bf16 in and out, fp32
statistics and parameters), PyTorch composition otherwise."""
from __future__ import annotations

import torch

from polyaxon_amd.ops import _native


def rms_norm_reference(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
    return y.to(x.dtype)


def _stream() -> int:
    return _native.current_stream()


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
        ctx.wdtype = weight.dtype
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
        return dx, part.sum(0).to(ctx.wdtype), None


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
        ctx.dtypes = (weight.dtype, bias.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.lib("plx_rms")
        x, w, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        d = x.shape[-1]
        rows = x.numel() // d
        dx = torch.empty_like(x)
        nb = lib.plx_rms_bwd_blocks(rows)
        part = torch.empty((2, nb, d), dtype=torch.float32, device=x.device)
        _native.check(lib.plx_ln_backward(x.data_ptr(), w.data_ptr(), dy.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                          dx.data_ptr(), part[0].data_ptr(), part[1].data_ptr(), rows, d, _stream()),
                      "plx_ln_backward")
        dwb = part.sum(1)
        return dx, dwb[0].to(ctx.dtypes[0]), dwb[1].to(ctx.dtypes[1]), None


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """LayerNorm over the last dim.  Under bf16 autocast the input is taken as bf16 and the output stays bf16 (what
    the next GEMM reads); the fused kernels need d % 8 == 0 and d <= 8192."""
    if x.is_cuda and x.dtype != torch.bfloat16 and torch.is_autocast_enabled("cuda"):
        x = x.to(torch.bfloat16)
    if supported(x):
        return _LayerNorm.apply(x, weight, bias, eps)
    return layer_norm_reference(x, weight, bias, eps)


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
