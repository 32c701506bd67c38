"""bf16 GEMMs of the transformer linears on the hand-written 256x256 MFMA kernel (csrc/gemm256.hip).

``linear(x, W, b)`` is y = x W^T + b with all three GEMMs of its training step on that kernel:

* forward  y[T][out]   = x[T][in] . W[out][in]^T  (both operands K-major),
* dgrad    dx[T][in]   = dy[T][out] . W[out][in]  (W read MN-major through the LDS transpose read),
* wgrad    dW[out][in] = dy^T . x, K = tokens     (both MN-major; split-K over fp32 slabs when the out x in tile grid
  alone cannot fill the 256 CUs).

The weight gradient can be written straight into a flat gradient slot (``out=``, ``accumulate=``): the kernel's
epilogue adds to the bf16 slot in place, so a weight used twice needs no separate gradient tensor.

Shapes the kernel does not take (a dimension not a multiple of 256, or K of 64) go to ``torch`` (hipBLASLt) —
:func:`supported` says which; on a GPU box a missing library raises instead of falling back (ops/_native.py).  The
LM trainers' shapes all fit (GPT-2's vocabulary is padded to 50432 rows, models/transformer.py).

Dispatch (``PLX_LM_GEMM``): ``auto`` (default) runs the kernel where it wins or ties on every MI355X box measured
(since round 6 every GEMM of the GPT-2 125M step) and hipBLASLt elsewhere; ``1`` always the kernel (the GPU tests),
``0`` always hipBLASLt.  Round 4 measured the kernel
and hipBLASLt on three boxes / cache states (profiles/r4_lm_gemm.md): the split-K weight gradients of the narrow
GPT-2 layers (and the tied head's) win 1.05-1.95x everywhere, a few Llama-3 8B weight / data gradients win by a few
percent, and the large forward / data-gradient shapes swing between 1.05x and 0.79x with the box (the kernel is
more clock-sensitive than hipBLASLt's), losing in the Llama training step (16.0k vs 18.0k tokens/s all-kernel vs
all-hipBLASLt on one box).  ``SCHEDULE`` holds the shapes that go to the kernel and the schedule each runs
(8 = the 8-wave ping-pong kernel, 5 = the 4-wave AGPR kernel, csrc/gemm256.hip); any other supported
shape goes to the kernel when it is a split-K shape (``plx_gemm256_splits > 1``: the narrow-output, long-reduction
weight gradients) and to hipBLASLt otherwise.  The choice is a pure function of the shape -- reproducible, and the
same kernel on every DP rank.  :func:`decisions` lists the shapes seen and what ran.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

from polyaxon_amd.ops import _native

TILE = 256
_ws: Dict[Tuple[str, int], torch.Tensor] = {}

_seen: Dict[Tuple[int, int, int, bool, bool], int] = {}  # shape -> schedule (-1 = hipBLASLt)

# (M, N, K, A K-major, B K-major) -> kernel schedule, for the GPT-2 125M (16 x 1024 tokens) / Llama-3 8B (1 x 4096)
# linears where the kernel beat hipBLASLt on every box (min ratio >= 0.98, mean >= 1.0 over
# profiles/r4_lm_gemm_variants_vs_hipblaslt.jsonl, r4_lm_gemm_hot.jsonl, r4_lm_gemm_cold.jsonl).
# fwd = (K, K), dgrad = (K, MN), wgrad = (MN, MN)
_FWD, _DGRAD, _WGRAD = (True, True), (True, False), (False, False)
SCHEDULE: Dict[Tuple[int, int, int, bool, bool], int] = {
    (M, N, K) + lay: v for (M, N, K, lay, v) in (
        # GPT-2: every weight gradient (split-K), the tied head's, the attention projection's data gradient
        (2304, 768, 16384, _WGRAD, 5), (768, 768, 16384, _WGRAD, 5), (3072, 768, 16384, _WGRAD, 5),
        (768, 3072, 16384, _WGRAD, 5), (50432, 768, 16384, _WGRAD, 5), (16384, 768, 768, _DGRAD, 9),
        # ... and, since round 6, every other GPT-2 linear: the forwards on the stream-K schedule.  The whole GPT-2
        # step on the kernel ties the mixed dispatch (708.9k vs 708.7k tokens/s over 4 + 3 alternating runs,
        # 702.5 / 697.3k vs 697.4 / 705.2k over 2 + 2 on another box; profiles/r6_lm_step_gpt2_kernel_only_ab.jsonl),
        # so no GPT-2 GEMM goes to hipBLASLt.
        (16384, 2304, 768, _FWD, 9), (16384, 768, 768, _FWD, 9), (16384, 3072, 768, _FWD, 9),
        (16384, 768, 3072, _FWD, 9), (16384, 50432, 768, _FWD, 9),
        # data gradients: the stream-K kernel everywhere but the head's (K = 50432, where the 4-wave one is 1.19 vs
        # 1.47 ms).  On the 192-tile N = 768 grids it beats the 4-wave one: QKV 0.064 vs 0.075 ms, MLP up 0.077 vs
        # 0.080, projection 0.027 vs 0.028 (profiles/r6_gemm_sched_gpt2.jsonl), +0.25 % on the step over 3
        # alternating pairs (r6_dgrad_sk_gpt2_step_ab.jsonl); the MLP down-projection's (N = 3072, K = 768):
        # 0.076-0.081 vs 0.086-0.088 ms (r6_lm_gemm_sk*.jsonl, r5)
        (16384, 768, 2304, _DGRAD, 9), (16384, 768, 3072, _DGRAD, 9), (16384, 768, 50432, _DGRAD, 5),
        (16384, 3072, 768, _DGRAD, 9),
        # Llama-3 8B: the weight gradients and the QKV data gradient
        (6144, 4096, 4096, _WGRAD, 5), (4096, 4096, 4096, _WGRAD, 5), (28672, 4096, 4096, _WGRAD, 5),
        (4096, 14336, 4096, _WGRAD, 5), (4096, 4096, 6144, _DGRAD, 5))}

# A/B override of the schedule for every kernel call (scripts/gemm_bench.py --waves); 0 = the table
FORCE_SCHEDULE = 0
SK = 9  # the persistent stream-K schedule (no accumulate: such calls run the 8-wave kernel)

# schedule of a kernel call outside the table, by layout (PLX_LM_GEMM=1, split-K shapes): the persistent stream-K
# kernel for the forward (both operands K-major: 2.85 vs 3.10 ms over one call of each of the 9 forward shapes in
# profiles/r6_lm_gemm_sk.jsonl; it was the 8-wave ping-pong kernel, 4.63 vs 4.91 ms per GPT-2 step against the
# 4-wave one), the 4-wave one for the data and weight gradients (4.40 vs 5.09, 45.2 vs 51.5; profiles/r5_lm_gemm.md).
# PLX_GEMM_WAVES overrides it.
_LAYOUT_SCHEDULE = {_FWD: SK, _DGRAD: 5, _WGRAD: 5}


def _schedule_of(M: int, N: int, K: int, a_kmajor: bool, b_kmajor: bool) -> int:
    if FORCE_SCHEDULE:
        return FORCE_SCHEDULE
    v = SCHEDULE.get((M, N, K, bool(a_kmajor), bool(b_kmajor)))
    if v:
        return v
    if os.environ.get("PLX_GEMM_WAVES"):
        return SK if os.environ["PLX_GEMM_WAVES"] == "9" else 0  # 9: stream-K; 8 / 5: the library's global knob
    return _LAYOUT_SCHEDULE.get((bool(a_kmajor), bool(b_kmajor)), 0)


def mode() -> str:
    m = os.environ.get("PLX_LM_GEMM", "auto")
    return m if m in ("0", "1", "auto") else "auto"


def enabled() -> bool:
    """PLX_LM_GEMM=0 routes the LM linears back to hipBLASLt (A/B knob)."""
    return mode() != "0"


def splits(M: int, N: int, K: int) -> int:
    return _native.size("plx_gemm", "plx_gemm256_splits", M, N, K)


def schedule(M: int, N: int, K: int, a_kmajor: bool, b_kmajor: bool) -> int:
    """What ``auto`` runs for a supported shape: the table's schedule, 0 (the library default) for a split-K shape
    outside it, -1 (hipBLASLt) otherwise."""
    v = SCHEDULE.get((M, N, K, bool(a_kmajor), bool(b_kmajor)))
    if v is not None:
        return v
    return 0 if splits(M, N, K) > 1 else -1


def _use_native(M, N, K, a_kmajor, b_kmajor) -> bool:
    m = mode()
    if m != "auto":
        return m == "1"
    key = (M, N, K, bool(a_kmajor), bool(b_kmajor))
    v = _seen.get(key)
    if v is None:
        v = _seen[key] = schedule(*key)
    return v >= 0


def decisions() -> Dict[str, Dict[str, object]]:
    """Shapes this process dispatched in ``auto`` mode: kernel (with its schedule) or hipBLASLt."""
    return {f"{M}x{N}x{K}:{'K' if ak else 'M'}{'K' if bk else 'N'}": {"native": v >= 0, "schedule": v}
            for (M, N, K, ak, bk), v in _seen.items()}


def _torch_gemm(a, b, M, N, K, a_kmajor, b_kmajor, out=None, accumulate=False, alpha=1.0):
    A = a.view(M, K) if a_kmajor else a.view(K, M).t()
    Bt = b.view(N, K).t() if b_kmajor else b.view(K, N)
    if out is None:
        return torch.mm(A, Bt) if alpha == 1.0 else torch.mm(A, Bt).mul_(alpha)
    if accumulate:
        out.addmm_(A, Bt, alpha=alpha)
    else:
        torch.mm(A, Bt, out=out)
        if alpha != 1.0:
            out.mul_(alpha)
    return out


def matmul(a, b, M, N, K, a_kmajor, b_kmajor, out=None, accumulate=False) -> torch.Tensor:
    """:func:`gemm` semantics on whichever of the MFMA kernel / hipBLASLt the dispatch picks."""
    if a.is_cuda and supported(M, N, K) and _use_native(M, N, K, a_kmajor, b_kmajor):
        return gemm(a, b, M, N, K, a_kmajor, b_kmajor, out=out, accumulate=accumulate)
    return _torch_gemm(a, b, M, N, K, a_kmajor, b_kmajor, out=out, accumulate=accumulate)


def supported(M: int, N: int, K: int) -> bool:
    return M > 0 and N > 0 and K > 0 and M % TILE == 0 and N % TILE == 0 and K % 64 == 0


def _workspace(device: torch.device, floats: int) -> torch.Tensor:
    """fp32 scratch (split-K slabs, stream-K partials) per (device, stream): launches on two streams of one device
    (trials sharing a GPU) never share one"""
    return _native.cached(_ws, (device.type, device.index or 0, _native.current_stream()),
                          lambda: torch.empty(max(floats, 1 << 20), dtype=torch.float32, device=device),
                          ok=lambda w: w.numel() >= floats)


def gemm(a: torch.Tensor, b: torch.Tensor, M: int, N: int, K: int, a_kmajor: bool, b_kmajor: bool,
         out: Optional[torch.Tensor] = None, accumulate: bool = False, alpha: float = 1.0,
         bias: Optional[torch.Tensor] = None, gelu_out: Optional[torch.Tensor] = None,
         gelu_h: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[M][N] (bf16, row-major, may be a strided view with unit column stride) = alpha * A . B (+ bias) (+ out).

    ``a`` is A[M][K] when ``a_kmajor`` else A stored [K][M]; ``b`` is B[N][K] when ``b_kmajor`` else [K][N].
    Both are contiguous bf16 (leading dimension = their row length).  ``bias``: [N], added in fp32 by the epilogue
    (cast to a contiguous fp32 copy if it is not one); not with ``accumulate``.  ``gelu_out``: a bf16 tensor shaped
    like ``out`` that also receives gelu_tanh(out) from the same epilogue (GPT-2's up-projection + activation).
    ``gelu_h``: a bf16 tensor laid out like ``out``; the epilogue stores bf16(A.B) * gelu_tanh'(gelu_h) instead (an
    MLP's GELU backward fused into the down-projection's data gradient; the stream-K schedule only, see
    :func:`gelu_bwd_supported`)."""
    if not supported(M, N, K):
        raise ValueError(f"gemm256 needs M, N % 256 == 0 and K % 64 == 0 (got {M}x{N}x{K})")
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not (a.is_contiguous() and b.is_contiguous()):
        raise ValueError("gemm256 takes contiguous bf16 operands")
    if a.numel() != M * K or b.numel() != N * K:
        raise ValueError(f"operand sizes {a.numel()}, {b.numel()} do not match {M}x{N}x{K}")
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs out")
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    if out.dtype != torch.bfloat16 or out.dim() != 2 or out.shape != (M, N) or out.stride(1) != 1:
        raise ValueError("out must be a [M][N] bf16 matrix with unit column stride")
    if bias is not None:
        if accumulate or bias.numel() != N:
            raise ValueError("bias needs numel N and no accumulate")
        bias = bias.to(torch.float32).contiguous()
        if bias.data_ptr() % 16:
            bias = bias.clone()
    if gelu_out is not None and (accumulate or gelu_out.dtype != torch.bfloat16 or gelu_out.shape != out.shape
                                 or gelu_out.stride() != out.stride() or gelu_out.data_ptr() % 16):
        raise ValueError("gelu_out must be a bf16 tensor laid out like out (and no accumulate)")
    lib = _native.lib("plx_gemm")
    v = _schedule_of(M, N, K, a_kmajor, b_kmajor)
    if gelu_h is not None:
        if (v != SK or accumulate or bias is not None or gelu_out is not None or not sk_supported(M, N, K)
                or gelu_h.dtype != torch.bfloat16 or gelu_h.shape != out.shape or gelu_h.stride() != out.stride()
                or gelu_h.data_ptr() % 16):
            raise ValueError("gelu_h needs the stream-K schedule, no bias / gelu_out / accumulate, and a bf16 tensor "
                             "laid out like out")
    if v == SK:
        if not accumulate and sk_supported(M, N, K):
            return _gemm_sk(lib, a, b, out, M, N, K, a_kmajor, b_kmajor, alpha, bias, gelu_out, gelu_h)
        v = 8  # accumulating calls and odd / short K: the 8-wave kernel
    ns = splits(M, N, K)
    ws = _workspace(a.device, ns * M * N).data_ptr() if ns > 1 else None
    lda = K if a_kmajor else M
    ldb = K if b_kmajor else N
    rc = lib.plx_gemm256_exv(a.data_ptr(), b.data_ptr(), out.data_ptr(), ws, M, N, K, lda, ldb, out.stride(0),
                             int(a_kmajor), int(b_kmajor), float(alpha), int(accumulate),
                             bias.data_ptr() if bias is not None else None,
                             gelu_out.data_ptr() if gelu_out is not None else None, v, _native.current_stream())
    if rc != 0:
        raise RuntimeError(f"plx_gemm256 failed ({rc}) for {M}x{N}x{K} a_kmajor={a_kmajor} b_kmajor={b_kmajor}")
    return out


def sk_supported(M: int, N: int, K: int) -> bool:
    """schedule 9 takes the kernel's shapes with an even K-tile count >= 4 (the chained ring)"""
    return supported(M, N, K) and (K // 64) % 2 == 0 and K >= 256


def sk_plan(M: int, N: int, K: int) -> Tuple[int, int, int]:
    """(persistent workgroups, stream-K tiles, K-tiles per workgroup in the stream-K phase) of schedule 9"""
    import ctypes
    t, i = ctypes.c_int(0), ctypes.c_int(0)
    g = _native.lib("plx_gemm").plx_gemm256_sk_plan(M, N, K, ctypes.byref(t), ctypes.byref(i))
    return g, t.value, i.value


def _gemm_sk(lib, a, b, out, M, N, K, a_kmajor, b_kmajor, alpha, bias, gelu_out, gelu_h=None):
    """schedule 9: the persistent stream-K kernel (csrc/gemm256.hip gemm256_sk_kernel)"""
    floats = _native.size("plx_gemm", "plx_gemm256_sk_ws", M, N, K)
    if floats < 0:
        raise ValueError(f"gemm256_sk does not take {M}x{N}x{K}")
    ws = _workspace(a.device, floats).data_ptr() if floats else None
    tickets = _native.counters(a.device, f"plx_gemm256_sk:{_native.current_stream()}", 1024)
    rc = lib.plx_gemm256_sk(a.data_ptr(), b.data_ptr(), out.data_ptr(), ws, tickets.data_ptr(), M, N, K,
                            K if a_kmajor else M, K if b_kmajor else N, out.stride(0), int(a_kmajor), int(b_kmajor),
                            float(alpha), bias.data_ptr() if bias is not None else None,
                            gelu_out.data_ptr() if gelu_out is not None else None,
                            gelu_h.data_ptr() if gelu_h is not None else None, _native.current_stream())
    if rc != 0:
        raise RuntimeError(f"plx_gemm256_sk failed ({rc}) for {M}x{N}x{K} a_kmajor={a_kmajor} b_kmajor={b_kmajor}")
    return out


def gelu_bwd_supported(T: int, d_ff: int, d: int) -> bool:
    """Can the data gradient dA[T][d_ff] = dy[T][d] . W_down[d][d_ff] carry the GELU backward in its epilogue (the
    dispatch runs it on the stream-K schedule)?"""
    if not (supported(T, d_ff, d) and sk_supported(T, d_ff, d)) or mode() == "0":
        return False
    return _use_native(T, d_ff, d, True, False) and _schedule_of(T, d_ff, d, True, False) == SK


def linear_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and enabled()):
        return False
    T = x.numel() // x.shape[-1]
    return supported(T, weight.shape[0], weight.shape[1]) and supported(T, weight.shape[1], weight.shape[0])


def forward(x2: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y[T][out] = x[T][in] . W[out][in]^T (+ bias): the bias rides in the GEMM epilogue (gemm256's fp32 bias add, or
    hipBLASLt's through addmm) instead of a separate read-modify-write pass over y"""
    T, fin = x2.shape
    N = weight.shape[0]
    if bias is None:
        return matmul(x2, weight, T, N, fin, True, True)
    if x2.is_cuda and supported(T, N, fin) and _use_native(T, N, fin, True, True):
        return gemm(x2, weight, T, N, fin, True, True, bias=bias)
    return torch.addmm(bias.to(x2.dtype), x2, weight.t())


# In `auto`, a forward with the GELU epilogue runs on the kernel (one launch, the activation a second store) instead
# of hipBLASLt + a separate GELU pass.  On the stream-K schedule that is +0.8 % on the GPT-2 step (709.2-711.3k vs
# 703.7-706.2k tokens/s, 3 alternating pairs, profiles/r6_gelu_native_sk_ab.jsonl; it was neutral on the 8-wave
# kernel, r5_gelu_native_ab.jsonl).  PLX_GELU_NATIVE=0: the table decides.
_GELU_NATIVE = os.environ.get("PLX_GELU_NATIVE", "1") != "0"


def forward_gelu(x2: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None):
    """(h, gelu_tanh(h)) with h = x . W^T (+ bias): on the MFMA kernel the activation is a second store of the same
    epilogue (no separate pass reading h back); on hipBLASLt addmm then F.gelu."""
    T, fin = x2.shape
    N = weight.shape[0]
    native = _use_native(T, N, fin, True, True)
    if not native and _GELU_NATIVE and mode() == "auto" and supported(T, N, fin):
        _seen[(T, N, fin, True, True)] = native = _LAYOUT_SCHEDULE[_FWD]  # decisions() reports what runs
    if x2.is_cuda and supported(T, N, fin) and native:
        h = torch.empty(T, N, dtype=torch.bfloat16, device=x2.device)
        a = torch.empty_like(h)
        gemm(x2, weight, T, N, fin, True, True, out=h, bias=bias, gelu_out=a)
        return h, a
    h = forward(x2, weight, bias)
    return h, torch.nn.functional.gelu(h, approximate="tanh")


def dgrad(dy2: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """dx[T][in] = dy[T][out] . W[out][in]"""
    T, fout = dy2.shape
    return matmul(dy2, weight, T, weight.shape[1], fout, True, False)


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, out: Optional[torch.Tensor] = None,
          accumulate: bool = False) -> torch.Tensor:
    """dW[out][in] (+)= dy[T][out]^T . x[T][in]"""
    T, fout = dy2.shape
    fin = x2.shape[1]
    if out is not None:
        out = out.view(fout, fin)
    return matmul(dy2, x2, fout, fin, T, False, False, out=out, accumulate=accumulate)
