"""Flash attention on the hand-written CDNA4 kernels (csrc/attn_kernels.hip): causal or full, GQA, bf16, head_dim
64 / 128, fp32 accumulation and softmax statistics.

``flash_attention(q, k, v)`` takes head-major ``[B, H, S, D]`` / ``[B, Hkv, S, D]`` tensors (what ops/lm.qkv_rope
produces) and returns the output already in ``[B, S, H, D]`` order -- the layout the output projection reads --
so no transpose copy follows attention.  Backward recomputes the probabilities from the saved log-sum-exp
(FlashAttention-2): a row-dot kernel for delta = rowsum(dO * O), a dQ kernel and a dK/dV kernel that owns a
128-key block x one query head (fp32 per-head partials summed over the GQA group by a reduce kernel;
no atomics).

CPU tensors, fp32 and other head dims use the plain fp32 math definition (``_reference``); bf16 with head_dim
64 / 128 on a GPU -- every training config -- always runs the HIP kernels.
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import torch

from polyaxon_amd.ops import _native


class _Strides(ctypes.Structure):
    _fields_ = [("b", ctypes.c_longlong), ("h", ctypes.c_longlong), ("s", ctypes.c_longlong)]


class _AttnArgs(ctypes.Structure):
    _fields_ = [("q", ctypes.c_void_p), ("k", ctypes.c_void_p), ("v", ctypes.c_void_p), ("o", ctypes.c_void_p),
                ("dout", ctypes.c_void_p), ("out", ctypes.c_void_p), ("dq", ctypes.c_void_p),
                ("dk", ctypes.c_void_p), ("dv", ctypes.c_void_p), ("lse2", ctypes.c_void_p),
                ("delta", ctypes.c_void_p),
                ("sq", _Strides), ("sk", _Strides), ("sv", _Strides), ("so", _Strides), ("sdo", _Strides),
                ("sdq", _Strides), ("sdk", _Strides), ("sdv", _Strides),
                ("B", ctypes.c_int), ("H", ctypes.c_int), ("Hkv", ctypes.c_int), ("S", ctypes.c_int),
                ("Skv", ctypes.c_int), ("causal", ctypes.c_int), ("c", ctypes.c_float), ("scale", ctypes.c_float),
                ("zero", ctypes.c_void_p)]


_ZERO = {}


def _zero_page(dev) -> torch.Tensor:
    return _native.cached(_ZERO, dev, lambda: torch.zeros(64, dtype=torch.bfloat16, device=dev))


def _bhs(t: torch.Tensor, layout: str) -> _Strides:
    """element strides (batch, head, seq) of a [B,H,S,D] ('bhsd') or [B,S,H,D] ('bshd') tensor"""
    if layout == "bhsd":
        return _Strides(t.stride(0), t.stride(1), t.stride(2))
    return _Strides(t.stride(0), t.stride(2), t.stride(1))


def _check(lib_args_size: int) -> None:
    if lib_args_size != ctypes.sizeof(_AttnArgs):
        raise RuntimeError(f"AttnArgs layout mismatch: HIP {lib_args_size} vs ctypes {ctypes.sizeof(_AttnArgs)}")


def _args(q, k, v, causal: bool, scale: float) -> _AttnArgs:
    B, H, S, D = q.shape
    a = _AttnArgs()
    a.q, a.k, a.v = q.data_ptr(), k.data_ptr(), v.data_ptr()
    a.sq, a.sk, a.sv = _bhs(q, "bhsd"), _bhs(k, "bhsd"), _bhs(v, "bhsd")
    a.B, a.H, a.Hkv, a.S, a.Skv = B, H, k.shape[1], S, k.shape[2]
    a.causal = int(causal)
    a.scale = scale
    a.c = scale * 1.4426950408889634
    a.zero = _zero_page(q.device).data_ptr()
    return a


def _reference(q, k, v, causal, scale):
    """Plain fp32 math (matmul + softmax): the CPU path and the path for shapes / dtypes the HIP kernel does not
    take (fp32 reference models, head_dim other than 64 / 128).  No SDPA, so no library attention kernel."""
    rep = q.shape[1] // k.shape[1]
    kk = k.repeat_interleave(rep, 1) if rep > 1 else k
    vv = v.repeat_interleave(rep, 1) if rep > 1 else v
    s = torch.matmul(q.float(), kk.float().transpose(-1, -2)) * scale
    if causal:
        S, Sk = q.shape[2], k.shape[2]
        s = s.masked_fill(torch.ones(S, Sk, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    o = torch.matmul(s.softmax(-1), vv.float()).to(q.dtype)
    return o.transpose(1, 2)


_CHECKED = False


def _lib():
    """The attention library, its argument-block layout checked once against this module's (8 waves per forward /
    dQ / dK-dV workgroup; the 4-wave variants stay reachable for the tests through plx_attn_set_*_waves)."""
    global _CHECKED
    lib = _native.lib("plx_attn")
    if not _CHECKED:
        _check(lib.plx_attn_args_size())
        _CHECKED = True
    return lib


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal: bool, scale: float):
        lib = _lib()
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        B, H, S, D = q.shape
        out = torch.empty(B, S, H, D, dtype=q.dtype, device=q.device)
        lse2 = torch.empty(B, H, S, dtype=torch.float32, device=q.device)
        a = _args(q, k, v, causal, scale)
        a.out, a.so, a.lse2 = out.data_ptr(), _bhs(out, "bshd"), lse2.data_ptr()
        rc = lib.plx_attn_fwd(ctypes.byref(a), D, torch.cuda.current_stream(q.device).cuda_stream)
        _native.check(rc, "plx_attn_fwd")
        ctx.save_for_backward(q, k, v, out, lse2)
        ctx.causal, ctx.scale = causal, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse2 = ctx.saved_tensors
        lib = _lib()
        dout = dout.contiguous()
        B, H, S, D = q.shape
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty(B, H, S, dtype=torch.float32, device=q.device)
        a = _args(q, k, v, ctx.causal, ctx.scale)
        a.o, a.so = out.data_ptr(), _bhs(out, "bshd")
        a.dout, a.sdo = dout.data_ptr(), _bhs(dout, "bshd")
        a.dq, a.sdq = dq.data_ptr(), _bhs(dq, "bhsd")
        a.dk, a.sdk = dk.data_ptr(), _bhs(dk, "bhsd")
        a.dv, a.sdv = dv.data_ptr(), _bhs(dv, "bhsd")
        a.lse2, a.delta = lse2.data_ptr(), delta.data_ptr()
        nbytes = int(lib.plx_attn_bwd_workspace(B, H, k.shape[1], k.shape[2], D))
        ws = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=q.device) if nbytes else None
        rc = lib.plx_attn_bwd(ctypes.byref(a), D, ws.data_ptr() if ws is not None else None,
                              torch.cuda.current_stream(q.device).cuda_stream)
        _native.check(rc, "plx_attn_bwd")
        return dq, dk, dv, None, None


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                    scale: Optional[float] = None) -> torch.Tensor:
    """softmax(q k^T * scale [+ causal mask]) v with GQA (H % Hkv == 0).  q: [B,H,S,D], k/v: [B,Hkv,Skv,D].
    Returns [B, S, H, D]."""
    if q.dim() != 4 or k.dim() != 4 or v.shape != k.shape or q.shape[-1] != k.shape[-1]:
        raise ValueError("expected q [B,H,S,D] and k/v [B,Hkv,Skv,D]")
    if q.shape[1] % k.shape[1]:
        raise ValueError("query heads must be a multiple of key/value heads")
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else float(scale)
    if not q.is_cuda or q.dtype != torch.bfloat16 or q.shape[-1] not in (64, 128):
        return _reference(q, k, v, causal, scale)
    return _FlashAttention.apply(q, k, v, causal, scale)
