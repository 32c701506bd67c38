"""Decoder-only transformers for the BASELINE.json language-model configs:

* GPT-2 125M — the Bayesian-GP search config (``gpt2_125m``: 12 layers, d=768, 12 heads, LayerNorm,
  GELU MLP, learned positions, tied embeddings, vocab 50257, context 1024);
* Llama-3 8B — the distributed PyTorchJob-equivalent config (``llama3_8b``: 32 layers, d=4096, 32 query /
  8 KV heads (GQA), RMSNorm, SwiGLU 14336, RoPE theta 500000, vocab 128256).

MI355X layout choices: bf16 autocast compute with fp32 master weights in a flat buffer (ops/flat.py) so
the optimizer is one fused kernel; attention on the hand-written CDNA4 flash attention (csrc/attn_kernels.hip,
GQA-native, output already in [B, S, H, D]); QKV and gate/up projections are single fused GEMMs (one
hipBLASLt call instead of 3 / 2);
RMSNorm in fp32 accumulate; optional activation checkpointing per block for long contexts.
The reference ships no models: these exist so the framework's HPO and distributed paths
can be exercised on the named configs with random weights and synthetic tokens.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from polyaxon_amd.ops import lm as lm_ops
from polyaxon_amd.ops import rmsnorm as _rms
from polyaxon_amd.ops.attention import flash_attention


@dataclass
class TransformerConfig:
    vocab_size: int = 50257
    n_layers: int = 12
    d_model: int = 768
    n_heads: int = 12
    n_kv_heads: Optional[int] = None
    d_ff: int = 3072
    max_seq_len: int = 1024
    norm: str = "layernorm"       # layernorm | rmsnorm
    mlp: str = "gelu"             # gelu | swiglu
    pos: str = "learned"          # learned | rope
    rope_theta: float = 10000.0
    tie_embeddings: bool = True
    norm_eps: float = 1e-5
    bias: bool = True
    checkpoint: bool = False
    # embedding / head rows are padded to a multiple of this (GPT-2's 50257 -> 50432 = 197 x 256, so the logits,
    # their data gradient and the tied-weight gradient are gemm256 shapes); the padded logits carry a -inf bias, so
    # the softmax, the loss and every gradient of the real vocabulary are unchanged and the padded rows get 0
    vocab_multiple: int = int(os.environ.get("PLX_VOCAB_MULTIPLE", "256"))  # A/B knob: 1 = no padding

    @property
    def kv_heads(self) -> int:
        return self.n_kv_heads or self.n_heads

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    @property
    def vocab_rows(self) -> int:
        m = max(1, self.vocab_multiple)
        return (self.vocab_size + m - 1) // m * m


def gpt2_125m(**kw) -> TransformerConfig:
    return TransformerConfig(**kw)


def llama3_8b(**kw) -> TransformerConfig:
    base = dict(vocab_size=128256, n_layers=32, d_model=4096, n_heads=32, n_kv_heads=8, d_ff=14336,
                max_seq_len=8192, norm="rmsnorm", mlp="swiglu", pos="rope", rope_theta=500000.0,
                tie_embeddings=False, bias=False)
    base.update(kw)
    return TransformerConfig(**base)


def tiny_llama(**kw) -> TransformerConfig:
    base = dict(vocab_size=256, n_layers=2, d_model=64, n_heads=4, n_kv_heads=2, d_ff=128, max_seq_len=64,
                norm="rmsnorm", mlp="swiglu", pos="rope", tie_embeddings=False, bias=False)
    base.update(kw)
    return TransformerConfig(**base)


class RMSNorm(nn.Module):
    def __init__(self, d: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(d))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from polyaxon_amd.ops import rmsnorm as _rms

        return _rms.rms_norm(x, self.weight, self.eps)


def rope_cache(seq_len: int, head_dim: int, theta: float, device, dtype=torch.float32):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, device=device, dtype=torch.float32) / head_dim))
    t = torch.arange(seq_len, device=device, dtype=torch.float32)
    freqs = torch.outer(t, inv)
    return freqs.cos().to(dtype), freqs.sin().to(dtype)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    # x: [B, H, S, D]; rotate pairs (even, odd) interleaved as two halves (Llama convention)
    d = x.shape[-1] // 2
    x1, x2 = x[..., :d], x[..., d:]
    c, s = cos[None, None, : x.shape[2]], sin[None, None, : x.shape[2]]
    return torch.cat([x1 * c - x2 * s, x1 * s + x2 * c], dim=-1)


class Attention(nn.Module):
    def __init__(self, cfg: TransformerConfig):
        super().__init__()
        self.cfg = cfg
        hd = cfg.head_dim
        self.qkv = nn.Linear(cfg.d_model, (cfg.n_heads + 2 * cfg.kv_heads) * hd, bias=cfg.bias)
        self.proj = nn.Linear(cfg.n_heads * hd, cfg.d_model, bias=cfg.bias)

    def forward(self, x, rope=None):
        B, S, _ = x.shape
        cfg = self.cfg
        hd = cfg.head_dim
        qkv = lm_ops.linear(x, self.qkv.weight, self.qkv.bias, side=True)
        if qkv.dtype == torch.bfloat16 and qkv.is_cuda:
            # one HIP pass: split + RoPE + head-major relayout (ops/lm.py)
            q, k, v = lm_ops.qkv_rope(qkv, B, S, cfg.n_heads, cfg.kv_heads, hd, rope)
        else:
            q, k, v = qkv.split([cfg.n_heads * hd, cfg.kv_heads * hd, cfg.kv_heads * hd], dim=-1)
            q = q.view(B, S, cfg.n_heads, hd).transpose(1, 2)
            k = k.view(B, S, cfg.kv_heads, hd).transpose(1, 2)
            v = v.view(B, S, cfg.kv_heads, hd).transpose(1, 2)
            if rope is not None:
                cs = (rope[0].to(q.dtype), rope[1].to(q.dtype))
                q, k = apply_rope(q, *cs), apply_rope(k, *cs)
        # hand-written CDNA4 flash attention (ops/attention.py, csrc/attn_kernels.hip): GQA straight into the
        # kernel (no repeat_interleave of K/V), output written in [B, S, H, D] so the projection reads it as is
        y = flash_attention(q, k, v, causal=True)
        return lm_ops.linear(y.reshape(B, S, cfg.n_heads * hd), self.proj.weight, self.proj.bias, side=True)


class MLP(nn.Module):
    def __init__(self, cfg: TransformerConfig):
        super().__init__()
        self.kind = cfg.mlp
        if cfg.mlp == "swiglu":
            self.up = nn.Linear(cfg.d_model, 2 * cfg.d_ff, bias=cfg.bias)  # fused gate|up GEMM
        else:
            self.up = nn.Linear(cfg.d_model, cfg.d_ff, bias=cfg.bias)
        self.down = nn.Linear(cfg.d_ff, cfg.d_model, bias=cfg.bias)

    def forward(self, x):
        if self.kind == "swiglu":
            h = lm_ops.swiglu(lm_ops.linear(x, self.up.weight, self.up.bias, side=True))
        else:  # GELU inside the op, its backward in the down-projection's data-gradient epilogue (ops/lm.py gelu_mlp)
            return lm_ops.gelu_mlp(x, self.up.weight, self.up.bias, self.down.weight, self.down.bias)
        return lm_ops.linear(h, self.down.weight, self.down.bias, side=True)


class Block(nn.Module):
    def __init__(self, cfg: TransformerConfig):
        super().__init__()
        Norm = (lambda d: RMSNorm(d, cfg.norm_eps)) if cfg.norm == "rmsnorm" else (
            lambda d: _rms.LayerNorm(d, eps=cfg.norm_eps))  # fused bf16 LayerNorm (csrc/rmsnorm.hip)
        self.n1, self.n2 = Norm(cfg.d_model), Norm(cfg.d_model)
        self.attn, self.mlp = Attention(cfg), MLP(cfg)

    def forward(self, x, rope=None):
        x = x + self.attn(self.n1(x), rope)
        return x + self.mlp(self.n2(x))


class Transformer(nn.Module):
    def __init__(self, cfg: TransformerConfig):
        super().__init__()
        self.cfg = cfg
        rows = cfg.vocab_rows
        self.embed = nn.Embedding(rows, cfg.d_model)
        self.pos = nn.Embedding(cfg.max_seq_len, cfg.d_model) if cfg.pos == "learned" else None
        self.blocks = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layers)])
        self.norm = RMSNorm(cfg.d_model, cfg.norm_eps) if cfg.norm == "rmsnorm" else _rms.LayerNorm(cfg.d_model)
        self.head = None if cfg.tie_embeddings else nn.Linear(cfg.d_model, rows, bias=False)
        if rows > cfg.vocab_size:  # fp32 logit bias: 0 on the vocabulary, -inf on the padding rows
            mask = torch.zeros(rows)
            mask[cfg.vocab_size:] = float("-inf")
            self.register_buffer("logit_mask", mask, persistent=False)
        else:
            self.logit_mask = None
        self._rope = None
        self.reset_parameters()

    def init_spec(self):
        """(param, kind, scale) for the fused in-place re-initialiser (GPT-2 / Llama conventions)."""
        spec = []
        resid_scale = 0.02 / math.sqrt(2 * self.cfg.n_layers)
        for name, p in self.named_parameters():
            if p.dim() == 1:
                spec.append((p, "const", 0.0 if name.endswith("bias") else 1.0))
            elif name.endswith("proj.weight") or name.endswith("down.weight"):
                spec.append((p, "normal", resid_scale))
            else:
                spec.append((p, "normal", 0.02))
        return spec

    @torch.no_grad()
    def reset_parameters(self):
        for p, kind, scale in self.init_spec():
            if kind == "normal":
                p.normal_(0.0, scale)
            else:
                p.fill_(scale)

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        B, S = tokens.shape
        x = self.embed(tokens)
        if self.head is None:  # tied head: its weight gradient may run on the side stream (lm_ops.linear side)
            x = lm_ops.join_before_backward(x)
        rope = None
        if self.pos is not None:
            x = x + self.pos(torch.arange(S, device=tokens.device))[None]
        else:
            if self._rope is None or self._rope[0].shape[0] < S or self._rope[0].device != tokens.device:
                self._rope = rope_cache(max(S, 16), self.cfg.head_dim, self.cfg.rope_theta, tokens.device)
            rope = (self._rope[0][:S], self._rope[1][:S])  # fp32 tables; the attention casts as needed
        if not (self.cfg.checkpoint and self.training):
            # every residual add is fused into the norm that reads its sum (ops/rmsnorm.py add_layer_norm /
            # add_rms_norm) -- the same computation as Block.forward, one pass fewer over the residual per add
            r = None
            for blk in self.blocks:
                x, h = self._add_norm(x, r, blk.n1)
                r = blk.attn(h, rope)
                x, h = self._add_norm(x, r, blk.n2)
                r = blk.mlp(h)
            x = self._add_norm(x, r, self.norm)[1]
        else:
            for blk in self.blocks:
                if self.cfg.checkpoint and self.training:
                    x = checkpoint(blk, x, rope, use_reentrant=False)
                else:
                    x = blk(x, rope)
            x = self.norm(x)
        # tied: the head's weight gradient is written first (into the flat slot, or returned to autograd) and the
        # embedding's arrives after it through autograd's accumulation, so both paths add up
        w = self.embed.weight if self.head is None else self.head.weight
        # side: the head's weight gradient beside its 192-tile data gradient and the blocks below (GPT-2: +1.6 %,
        # profiles/r6_lm_head_side_ab.jsonl); the embedding's backward waits for it (join_before_backward above)
        return lm_ops.linear(x, w, self.logit_mask, side=True)

    @staticmethod
    def _add_norm(x, r, norm):
        if r is None:
            return x, norm(x)
        if isinstance(norm, RMSNorm):
            return _rms.add_rms_norm(x, r, norm.weight, norm.eps)
        return _rms.add_layer_norm(x, r, norm.weight, norm.bias, norm.eps)

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())


def lm_loss(logits: torch.Tensor, tokens: torch.Tensor) -> torch.Tensor:
    """Next-token cross entropy (targets = tokens shifted left), mean over B * (S - 1) positions: the fused HIP kernels
    on bf16 GPU logits (ops/lm.py next_token_xent), F.cross_entropy in fp32 otherwise."""
    return lm_ops.next_token_xent(logits, tokens)
