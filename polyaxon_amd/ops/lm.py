"""Language-model hot ops: fused QKV split + RoPE + head-major relayout, fused SwiGLU, and a Linear whose
weight gradient is written by the GEMM straight into the flat (bf16) gradient buffer.

HIP kernels in csrc/lm_kernels.hip for bf16 CUDA tensors; every op has a plain PyTorch composition used on
CPU (tests, gloo runs) and as the numerics reference of the GPU tests.  On a GPU a bf16 input that the
kernel cannot take (odd head size, ...) raises instead of silently falling back.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from polyaxon_amd.ops import _native, side_stream

# weight gradients of the transformer blocks' linears on the side stream (ops/side_stream.py), overlapped with the
# data gradient queued after them when that one leaves CUs idle: GPT-2's N = 768 data gradients fill 192 of the 256
# CUs with 256x256 tiles, and the weight gradient beside them takes the rest.  PLX_LM_WGRAD_STREAM=0 runs them inline.
_WGRAD_SIDE = os.environ.get("PLX_LM_WGRAD_STREAM", "1") != "0"
_CUS = {}


def _idle_cus(dev: torch.device, M: int, N: int) -> bool:
    """Does an M x N GEMM output (256x256 tiles) leave CUs idle in its last wave?"""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    cus = _CUS.get(idx)
    if cus is None:
        cus = _CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    tiles = -(-M // 256) * -(-N // 256)
    return tiles % cus != 0


def _stream() -> int:
    return _native.current_stream()


def _native_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16


# ---------------------------------------------------------------------------------------------- QKV + RoPE
def qkv_rope_reference(qkv: torch.Tensor, B: int, S: int, H: int, KV: int, D: int,
                       rope: Optional[Tuple[torch.Tensor, torch.Tensor]]):
    q, k, v = qkv.view(B, S, H + 2 * KV, D).split([H, KV, KV], dim=2)
    q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    if rope is not None:
        cos, sin = rope
        c, s = cos[None, None, :S].to(q.dtype), sin[None, None, :S].to(q.dtype)

        def rot(x):
            d = x.shape[-1] // 2
            x1, x2 = x[..., :d], x[..., d:]
            return torch.cat([x1 * c - x2 * s, x1 * s + x2 * c], dim=-1)
        q, k = rot(q), rot(k)
    return q.contiguous(), k.contiguous(), v.contiguous()


class _QKVRope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, B, S, H, KV, D, rot):
        lib = _native.lib("plx_lm")
        qkv = qkv.contiguous()
        q = torch.empty((B, H, S, D), dtype=qkv.dtype, device=qkv.device)
        k = torch.empty((B, KV, S, D), dtype=qkv.dtype, device=qkv.device)
        v = torch.empty_like(k)
        _native.check(lib.plx_qkv_rope_fwd(qkv.data_ptr(), cos.data_ptr(), sin.data_ptr(), q.data_ptr(), k.data_ptr(),
                                           v.data_ptr(), B * S, S, H, KV, D, rot, _stream()), "plx_qkv_rope_fwd")
        ctx.save_for_backward(cos, sin)
        ctx.dims = (B, S, H, KV, D, rot, qkv.shape)
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        lib = _native.lib("plx_lm")
        cos, sin = ctx.saved_tensors
        B, S, H, KV, D, rot, shape = ctx.dims
        dq = dq.contiguous() if dq is not None else torch.zeros((B, H, S, D), dtype=torch.bfloat16, device=cos.device)
        dk = dk.contiguous() if dk is not None else torch.zeros((B, KV, S, D), dtype=torch.bfloat16, device=cos.device)
        dv = dv.contiguous() if dv is not None else torch.zeros((B, KV, S, D), dtype=torch.bfloat16, device=cos.device)
        dqkv = torch.empty(shape, dtype=dq.dtype, device=dq.device)
        _native.check(lib.plx_qkv_rope_bwd(dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), cos.data_ptr(), sin.data_ptr(),
                                           dqkv.data_ptr(), B * S, S, H, KV, D, rot, _stream()), "plx_qkv_rope_bwd")
        return dqkv, None, None, None, None, None, None, None, None


def qkv_rope(qkv: torch.Tensor, B: int, S: int, H: int, KV: int, D: int,
             rope: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
    """qkv [B, S, (H+2KV)*D] -> q [B,H,S,D], k/v [B,KV,S,D] (contiguous), q and k rotated when ``rope``
    = (cos, sin) fp32 [>=S, D/2] is given."""
    if not _native_ok(qkv):
        return qkv_rope_reference(qkv, B, S, H, KV, D, rope)
    if D % 16:
        raise ValueError(f"plx_qkv_rope needs head_dim % 16 == 0, got {D}")
    if rope is not None:
        cos = rope[0][:S].float().contiguous()
        sin = rope[1][:S].float().contiguous()
        rot = H + KV
    else:
        cos = sin = torch.zeros(1, dtype=torch.float32, device=qkv.device)
        rot = 0
    return _QKVRope.apply(qkv, cos, sin, B, S, H, KV, D, rot)


# ---------------------------------------------------------------------------------------------- SwiGLU
def swiglu_reference(h: torch.Tensor) -> torch.Tensor:
    g, u = h.chunk(2, dim=-1)
    return F.silu(g) * u


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        lib = _native.lib("plx_lm")
        h = h.contiguous()
        F2 = h.shape[-1]
        T = h.numel() // F2
        a = torch.empty(h.shape[:-1] + (F2 // 2,), dtype=h.dtype, device=h.device)
        _native.check(lib.plx_swiglu_fwd(h.data_ptr(), a.data_ptr(), T, F2 // 2, _stream()), "plx_swiglu_fwd")
        ctx.save_for_backward(h)
        return a

    @staticmethod
    def backward(ctx, da):
        lib = _native.lib("plx_lm")
        (h,) = ctx.saved_tensors
        da = da.contiguous()
        F2 = h.shape[-1]
        dh = torch.empty_like(h)
        _native.check(lib.plx_swiglu_bwd(da.data_ptr(), h.data_ptr(), dh.data_ptr(), h.numel() // F2, F2 // 2,
                                         _stream()), "plx_swiglu_bwd")
        return dh


def swiglu(h: torch.Tensor) -> torch.Tensor:
    """h [..., 2F] = gate | up -> silu(gate) * up."""
    if not _native_ok(h):
        return swiglu_reference(h)
    if h.shape[-1] % 16:
        raise ValueError("plx_swiglu needs the hidden size % 8 == 0")
    return _SwiGLU.apply(h)


# ---------------------------------------------------------------------------------------------- cross entropy
class _NextTokenXent(torch.autograd.Function):
    """mean over (b, s < S-1) of lse(logits[b, s]) - logits[b, s, tokens[b, s+1]] straight from the bf16 logits
    (csrc/lm_kernels.hip plx_xent_fwd / plx_xent_bwd): no slice copy, no fp32 logits, no log-softmax tensor; the
    backward writes bf16 (softmax - onehot) * dloss / rows into a logits-shaped gradient in one pass."""

    @staticmethod
    def forward(ctx, logits, tokens):
        lib = _native.lib("plx_lm")
        B, S, V = logits.shape
        rows = B * (S - 1)
        lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
        loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
        _native.check(lib.plx_xent_fwd(logits.data_ptr(), tokens.data_ptr(), lse.data_ptr(), loss.data_ptr(), B, S, V,
                                       _stream()), "plx_xent_fwd")
        ctx.save_for_backward(logits, tokens, lse)
        return loss.mean()

    @staticmethod
    def backward(ctx, g):
        lib = _native.lib("plx_lm")
        logits, tokens, lse = ctx.saved_tensors
        B, S, V = logits.shape
        grad = torch.empty_like(logits)
        g = g.detach().to(torch.float32).reshape(1).contiguous()
        _native.check(lib.plx_xent_bwd(logits.data_ptr(), tokens.data_ptr(), lse.data_ptr(), g.data_ptr(),
                                       grad.data_ptr(), B, S, V, _stream()), "plx_xent_bwd")
        return grad, None


def next_token_xent(logits: torch.Tensor, tokens: torch.Tensor) -> torch.Tensor:
    """Next-token cross entropy (targets = tokens shifted left), mean over B * (S - 1) positions: the fused HIP pair on
    bf16 CUDA logits [B, S, V] (contiguous, 16-byte aligned) with int64 tokens [B, S]; the fp32 reference otherwise."""
    if (logits.is_cuda and logits.dtype == torch.bfloat16 and logits.dim() == 3 and logits.is_contiguous()
            and logits.data_ptr() % 16 == 0 and tokens.dtype == torch.int64 and tokens.is_contiguous()
            and tokens.shape == logits.shape[:2] and logits.shape[1] >= 2):
        return _NextTokenXent.apply(logits, tokens)
    return F.cross_entropy(logits[:, :-1].reshape(-1, logits.shape[-1]).float(), tokens[:, 1:].reshape(-1))


class _ClassXent(torch.autograd.Function):
    """mean over rows of lse(logits[r]) - logits[r, labels[r]] from bf16 logits [N][V] (csrc/lm_kernels.hip
    plx_xent_cls_fwd / plx_xent_cls_bwd): replaces F.cross_entropy(logits.float(), labels)'s fp32 cast, log-softmax,
    NLL and their three backward kernels with one kernel each way (the ResNet head, polyflow/executor.py).

    Rows whose label lies outside [0, V) (F.cross_entropy's ignore_index -100) contribute no loss and no gradient;
    unless the caller guarantees every label is in range (``in_range``: the executor's own synthetic data), the mean
    divides by the number of valid rows, as F.cross_entropy does (two extra small reductions)."""

    @staticmethod
    def forward(ctx, logits, labels, in_range):
        lib = _native.lib("plx_lm")
        N, V = logits.shape
        lse = torch.empty(N, dtype=torch.float32, device=logits.device)
        loss = torch.empty(N, dtype=torch.float32, device=logits.device)
        _native.check(lib.plx_xent_cls_fwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), loss.data_ptr(), N, V,
                                           _stream()), "plx_xent_cls_fwd")
        nvalid = None if in_range else ((labels >= 0) & (labels < V)).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(logits, labels, lse, nvalid if nvalid is not None else lse.new_ones(()))
        ctx.in_range = in_range
        return loss.mean() if in_range else loss.sum() / nvalid

    @staticmethod
    def backward(ctx, g):
        lib = _native.lib("plx_lm")
        logits, labels, lse, nvalid = ctx.saved_tensors
        N, V = logits.shape
        grad = torch.empty_like(logits)
        g = g.detach().to(torch.float32).reshape(1)
        if not ctx.in_range:
            g = g / nvalid  # scale 1: the kernel multiplies by dloss only
        g = g.contiguous()
        _native.check(lib.plx_xent_cls_bwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), g.data_ptr(),
                                           grad.data_ptr(), N, V, 0.0 if ctx.in_range else 1.0, _stream()),
                      "plx_xent_cls_bwd")
        return grad, None, None


def class_xent(logits: torch.Tensor, labels: torch.Tensor, in_range: bool = False) -> torch.Tensor:
    """Classification cross entropy, mean over the rows with a label in [0, V) (F.cross_entropy semantics, ignore
    index -100 included): the fused HIP pair on bf16 CUDA logits [N, V] (contiguous) with int64 labels [N];
    F.cross_entropy on fp32 logits otherwise.  ``in_range``: the caller guarantees 0 <= label < V for every row
    (skips the valid-row count)."""
    if (logits.is_cuda and logits.dtype == torch.bfloat16 and logits.dim() == 2 and logits.is_contiguous()
            and labels.dtype == torch.int64 and labels.is_contiguous() and labels.shape == logits.shape[:1]):
        return _ClassXent.apply(logits, labels, bool(in_range))
    return F.cross_entropy(logits.float(), labels)


# ---------------------------------------------------------------------------------------------- bias gradient


def bias_grad(dy2: torch.Tensor, bias: torch.Tensor, gelu_h: Optional[torch.Tensor] = None, side: bool = False):
    """db = dy2.sum(0) for ``bias``.  With a direct fp32 flat-gradient slot (ops/flat.py) the sum is written -- or,
    for a slot already written this step, accumulated -- there and None is returned (no autograd ``grad += g``
    kernel; FlatDDP still sees the parameter through its post-accumulate hook); otherwise returned in the bias
    dtype.  The sum
    is the deterministic one-launch column reduction (csrc/lm_kernels.hip plx_colsum, fp32 accumulation) for a
    contiguous bf16 CUDA [T, N] with N % 8 == 0, torch's reduction otherwise.

    ``gelu_h``: dy2 is the gradient of gelu_tanh(gelu_h); returns (dh, db) with dh = dy2 * gelu_tanh'(gelu_h)
    computed in the same pass as its column sums (plx_gelu_bwd_colsum).

    ``side``: the bias belongs to this op only; a plain column sum into its (first-written) flat slot then runs on
    the side stream (PLX_LM_WGRAD_STREAM), beside the compute-bound GEMMs that follow it on the main stream."""
    from polyaxon_amd.ops.flat import direct_grad

    T, N = dy2.shape
    slot = direct_grad(bias)
    if slot is not None and not (slot.dtype == torch.float32 and slot.is_contiguous() and slot.numel() == N
                                 and slot.device == dy2.device):
        slot = None
    acc = bool(bias._plx_flat.mark_written(slot)) if slot is not None else False
    native = (_native_ok(dy2) and dy2.is_contiguous() and N % 8 == 0 and dy2.data_ptr() % 16 == 0
              and T > 0 and (N + 63) // 64 <= 4096 and (slot is not None or bias.dtype in (torch.float32, torch.bfloat16)))
    if gelu_h is not None:
        native = (native and gelu_h.dtype == torch.bfloat16 and gelu_h.is_contiguous() and gelu_h.shape == dy2.shape
                  and gelu_h.data_ptr() % 16 == 0)
    dh = None
    if native:
        lib = _native.lib("plx_lm")
        dev = dy2.device
        out = slot if slot is not None else torch.empty(N, dtype=bias.dtype, device=dev)
        mode = (2 if acc else 1) if out.dtype == torch.float32 else 0

        def colsum():  # partials and tickets of the stream it runs on
            part = torch.empty(lib.plx_colsum_splits(T, N), N, dtype=torch.float32, device=dev)
            cnt = _native.counters(dev, f"plx_colsum:{_stream()}")
            _native.check(lib.plx_colsum(dy2.data_ptr(), T, N, part.data_ptr(), cnt.data_ptr(), out.data_ptr(), mode,
                                         _stream()), "plx_colsum")
        if gelu_h is None:
            if side and _WGRAD_SIDE and slot is not None and not acc:  # +1.3 % on GPT-2, r6_lm_bias_side_ab.jsonl
                side_stream.run(colsum, (dy2,), dev)
            else:
                colsum()
        else:
            part = torch.empty(lib.plx_colsum_splits(T, N), N, dtype=torch.float32, device=dev)
            cnt = _native.counters(dev, f"plx_colsum:{_stream()}")
            dh = torch.empty_like(dy2)
            _native.check(lib.plx_gelu_bwd_colsum(dy2.data_ptr(), gelu_h.data_ptr(), dh.data_ptr(), T, N,
                                                  part.data_ptr(), cnt.data_ptr(), out.data_ptr(), mode, _stream()),
                          "plx_gelu_bwd_colsum")
    else:
        if gelu_h is not None:
            dy2 = dh = torch.ops.aten.gelu_backward(dy2, gelu_h, approximate="tanh")
        if slot is not None:
            with torch.no_grad():
                s = dy2.sum(0, dtype=torch.float32)
                slot.add_(s) if acc else slot.copy_(s)
        else:
            out = dy2.sum(0).to(bias.dtype)
    db = out if slot is None else None
    return db if gelu_h is None else (dh, db)


def _act_backward(ctx, dy2: torch.Tensor, h2: Optional[torch.Tensor]):
    """(dz, db) of a Linear (+ optional GELU) from the output gradient: with the activation fused, dz = dA * gelu'(h)
    and the bias gradient come out of one pass; otherwise dz = dy and db is the plain column sum."""
    if h2 is not None:
        if ctx.has_bias:
            return bias_grad(dy2, ctx.bias, gelu_h=h2)
        return torch.ops.aten.gelu_backward(dy2, h2, approximate="tanh"), None
    return dy2, (bias_grad(dy2, ctx.bias, side=getattr(ctx, "side", False)) if ctx.has_bias else None)


# ---------------------------------------------------------------------------------------------- direct-grad Linear
class _LinearDirect(torch.autograd.Function):
    """y = x W^T (+ b), optionally followed by GELU (tanh; ``act``).  Backward writes dW = dz^T x with the GEMM's
    output pointer on the parameter's flat gradient slot (``p.grad``, bf16 in lp mode): no separate gradient tensor
    and no autograd ``grad += g`` read-modify-write.  The flat buffer is zeroed by the optimizer, so the first write
    of a step is a plain GEMM (beta = 0) and any later one (a weight used twice) accumulates (beta = 1).  With the
    activation fused, its backward and the bias gradient are one pass (``bias_grad(..., gelu_h=h)``)."""

    @staticmethod
    def forward(ctx, x, weight, bias, slot, flat, act=None):
        # a bias that takes no gradient (the logit mask of a padded vocabulary) skips the column-sum pass
        ctx.slot, ctx.flat, ctx.has_bias = slot, flat, bias is not None and bias.requires_grad
        ctx.bias, ctx.act = bias, act
        y = F.linear(x, weight, bias if bias is None or bias.dtype == x.dtype else bias.to(x.dtype))
        if act is None:
            ctx.save_for_backward(x, weight)
            return y
        ctx.save_for_backward(x, weight, y)
        return F.gelu(y, approximate="tanh")

    @staticmethod
    def backward(ctx, dy):
        x, weight, *h = ctx.saved_tensors
        n = dy.shape[-1]
        dy2, db = _act_backward(ctx, dy.reshape(-1, n).contiguous() if h else dy.reshape(-1, n),
                                h[0].reshape(-1, n) if h else None)
        dx = (dy2 @ weight).view(*dy.shape[:-1], weight.shape[1]) if ctx.needs_input_grad[0] else None
        x2 = x.reshape(-1, x.shape[-1]).to(dy2.dtype)
        g = ctx.slot
        if ctx.flat.mark_written(g):
            torch.addmm(g, dy2.t(), x2, out=g)
        else:
            torch.mm(dy2.t(), x2, out=g)
        return dx, None, db, None, None, None


class _LinearMfma(torch.autograd.Function):
    """y = x W^T (+ b) (then GELU with ``act``) with forward, data-gradient and weight-gradient GEMMs on the
    hand-written 256x256 MFMA kernel (ops/gemm.py, csrc/gemm256.hip).  ``slot``/``flat`` as in
    :class:`_LinearDirect`: when given, dW is written (or, for a weight already written this step, accumulated by
    the kernel's epilogue) straight into the flat gradient slot."""

    @staticmethod
    def forward(ctx, x, weight, bias, slot, flat, act=None, side=False):
        from polyaxon_amd.ops import gemm

        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        ctx.slot, ctx.flat, ctx.has_bias, ctx.xshape = slot, flat, bias is not None and bias.requires_grad, x.shape
        ctx.bias, ctx.act, ctx.side = bias, act, side
        if act is None:
            y = gemm.forward(x2, weight, bias)
            ctx.save_for_backward(x2, weight)
        else:  # GELU as a second store of the GEMM epilogue (ops/gemm.py forward_gelu)
            h, y = gemm.forward_gelu(x2, weight, bias)
            ctx.save_for_backward(x2, weight, h)
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from polyaxon_amd.ops import gemm

        x2, weight, *h = ctx.saved_tensors
        dy2, db = _act_backward(ctx, dy.reshape(-1, dy.shape[-1]).contiguous(), h[0] if h else None)
        dw = None
        if ctx.slot is not None:
            _wgrad_into(gemm, dy2, x2, ctx.slot, ctx.flat, True,  # queued before the data gradient
                        side=(x2.shape[0], x2.shape[1]) if ctx.side else None)
        elif ctx.needs_input_grad[1]:
            dw = gemm.wgrad(dy2, x2)
        dx = gemm.dgrad(dy2, weight).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        return dx, dw, db, None, None, None, None


class _SideJoin(torch.autograd.Function):
    """Identity whose backward makes the main stream wait for every side-stream launch so far (side_stream.join)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        side_stream.join(g.device)
        return g


def join_before_backward(x: torch.Tensor) -> torch.Tensor:
    """Mark ``x`` (a tied embedding's output): the ops that consume its gradient -- the embedding's backward, whose
    weight-gradient accumulation writes the slot the tied head's side-stream weight gradient wrote -- run after the
    side stream has finished.  Identity on the CPU and outside autograd."""
    if not (x.is_cuda and x.requires_grad and torch.is_grad_enabled()):
        return x
    return _SideJoin.apply(x)


def _wgrad_into(gemm, dz2, x2, slot, flat, needs, side=None):
    """dW = dz^T x: written / accumulated into the flat slot when there is one (returns None), else returned.
    ``side`` = (M, N) of the data gradient queued next: the weight is used by this op only (no other op of the step
    writes its slot), so the slot write may run on the side stream beside that GEMM when it leaves CUs idle; only the
    optimizer and FlatDDP read the slot, after side_stream.join / fence."""
    if slot is not None:
        acc = bool(flat.mark_written(slot))
        if side is not None and _WGRAD_SIDE and not acc and _idle_cus(dz2.device, *side):
            # (the planner's full 256-block split on the side stream too: a 128-block target tied, 64 was -23 %,
            # profiles/r6_lm_side_split_target_ab.jsonl)
            # (token chunks for the unsplit tied head, so its long workgroups free CUs sooner: neutral,
            # profiles/r6_lm_head_wgrad_chunk_ab.jsonl)
            side_stream.run(lambda: gemm.wgrad(dz2, x2, out=slot, accumulate=False), (dz2, x2), dz2.device)
        else:
            gemm.wgrad(dz2, x2, out=slot, accumulate=acc)
        return None
    return gemm.wgrad(dz2, x2) if needs else None


class _GeluMlpMfma(torch.autograd.Function):
    """GPT-2's MLP, y = down(gelu_tanh(up(x))), with all six GEMMs on the MFMA kernel and the GELU backward in the
    down-projection's data-gradient epilogue: dh = bf16(dy . W_down) * gelu_tanh'(h) is stored once, instead of dA
    being stored and a separate pass reading dA and h back to write dh (csrc/gemm256.hip ``gelu_h``; the same
    roundings as that pass).  The up-projection's bias gradient is then a plain column sum of dh.  +2.1 % on the
    GPT-2 125M step (712.7-715.6k vs 695.8-700.0k tokens/s, 4 alternating pairs, profiles/r6_gelu_mlp_ab.jsonl).
    ``slots``: the two weights' flat gradient slots (or None), as in :class:`_LinearMfma`."""

    @staticmethod
    def forward(ctx, x, w_up, b_up, w_down, b_down, slot_up, slot_down, flat_up, flat_down):
        from polyaxon_amd.ops import gemm

        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        h, a = gemm.forward_gelu(x2, w_up, b_up)
        y = gemm.forward(a, w_down, b_down)
        ctx.save_for_backward(x2, w_up, h, a, w_down)
        ctx.slots, ctx.flats, ctx.xshape = (slot_up, slot_down), (flat_up, flat_down), x.shape
        ctx.b_up, ctx.b_down = b_up, b_down
        ctx.has_b = (b_up is not None and b_up.requires_grad, b_down is not None and b_down.requires_grad)
        return y.view(*x.shape[:-1], w_down.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from polyaxon_amd.ops import gemm

        x2, w_up, h, a, w_down = ctx.saved_tensors
        T, d_ff = h.shape
        d = w_down.shape[0]
        dy2 = dy.reshape(-1, d).contiguous()
        db_down = bias_grad(dy2, ctx.b_down, side=True) if ctx.has_b[1] else None
        # a side-stream weight gradient forks from the main stream as it stands: queue it before the data gradient
        # it should overlap, not after (it would wait for it)
        # both weight gradients go beside the MLP's data gradients when the narrow one (T x d) leaves CUs idle:
        # GPT-2 +3.6 % on the step (r6_lm_wgrad_side_ab.jsonl), both on the side stream 0.3 % ahead of dw_up alone
        dw_down = _wgrad_into(gemm, dy2, a, ctx.slots[1], ctx.flats[1], ctx.needs_input_grad[3], side=(T, d))
        dh = gemm.gemm(dy2, w_down, T, d_ff, d, True, False, gelu_h=h)  # dA . gelu'(h) in the epilogue
        db_up = bias_grad(dh, ctx.b_up, side=True) if ctx.has_b[0] else None
        dw_up = _wgrad_into(gemm, dh, x2, ctx.slots[0], ctx.flats[0], ctx.needs_input_grad[1], side=(T, d))
        dx = gemm.dgrad(dh, w_up).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        return dx, dw_up, db_up, dw_down, db_down, None, None, None, None


def _direct_slot(x: torch.Tensor, weight: torch.Tensor):
    """(slot, flat) when ``weight``'s gradient is written straight into its flat slot (lp mode, direct grads)"""
    slot = getattr(weight, "grad", None)
    flat = getattr(weight, "_plx_flat", None)
    direct = (flat is not None and getattr(weight, "_plx_direct_grad", False) and slot is not None
              and weight.requires_grad and torch.is_grad_enabled() and slot.dtype == weight.dtype
              and x.dtype == weight.dtype and slot.is_contiguous())
    return (slot, flat) if direct else (None, None)


def gelu_mlp(x: torch.Tensor, w_up: torch.Tensor, b_up: Optional[torch.Tensor], w_down: torch.Tensor,
             b_down: Optional[torch.Tensor]) -> torch.Tensor:
    """down(gelu_tanh(up(x))): one op with the GELU backward fused into the down-projection's data gradient
    (:class:`_GeluMlpMfma`) when every GEMM takes the MFMA kernel and that data gradient runs on the stream-K
    schedule; the two :func:`linear` ops otherwise."""
    from polyaxon_amd.ops import gemm

    if (x.is_cuda and x.dtype == torch.float32 and w_up.dtype == torch.bfloat16
            and torch.is_autocast_enabled("cuda")):
        x = x.to(torch.bfloat16)
    d_ff, d = w_up.shape
    T = x.numel() // x.shape[-1] if x.dim() else 0
    if (torch.is_grad_enabled() and w_up.is_contiguous() and w_down.is_contiguous() and w_down.shape == (d, d_ff)
            and gemm.linear_supported(x, w_up) and gemm.supported(T, d, d_ff) and gemm.gelu_bwd_supported(T, d_ff, d)):
        su, fu = _direct_slot(x, w_up)
        sd, fd = _direct_slot(x, w_down)
        return _GeluMlpMfma.apply(x, w_up, b_up, w_down, b_down, su, sd, fu, fd)
    return linear(linear(x, w_up, b_up, act="gelu_tanh"), w_down, b_down)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
           act: Optional[str] = None, side: bool = False) -> torch.Tensor:
    """F.linear on the MFMA GEMM kernel when the shapes fit it (ops/gemm.py: tokens, in and out multiples of 256,
    bf16, PLX_LM_GEMM != 0), with the weight gradient written into the flat gradient slot when ``weight`` is a flat
    parameter in lp mode with direct grads; hipBLASLt (F.linear / the direct-gradient form) otherwise.
    ``act="gelu_tanh"`` applies GPT-2's GELU inside the op, so its backward is fused with the bias gradient."""
    if act not in (None, "gelu_tanh"):
        raise ValueError(f"unknown activation {act!r}")
    if (x.is_cuda and x.dtype == torch.float32 and weight.dtype == torch.bfloat16
            and torch.is_autocast_enabled("cuda")):
        x = x.to(torch.bfloat16)  # what autocast's F.linear does; here it keeps the LayerNorm outputs on the MFMA path
    slot = getattr(weight, "grad", None)
    flat = getattr(weight, "_plx_flat", None)
    direct = (flat is not None and getattr(weight, "_plx_direct_grad", False) and slot is not None
              and weight.requires_grad and torch.is_grad_enabled() and slot.dtype == weight.dtype
              and x.dtype == weight.dtype and slot.is_contiguous())
    from polyaxon_amd.ops import gemm

    if weight.is_contiguous() and gemm.linear_supported(x, weight):
        if direct:
            return _LinearMfma.apply(x, weight, bias, slot, flat, act, side)
        return _LinearMfma.apply(x, weight, bias, None, None, act)
    if direct:
        return _LinearDirect.apply(x, weight, bias, slot, flat, act)
    y = F.linear(x, weight, bias if bias is None or bias.dtype == x.dtype else bias.to(x.dtype))
    return y if act is None else F.gelu(y, approximate="tanh")
