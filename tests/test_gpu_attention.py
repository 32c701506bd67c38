"""Hand-written CDNA4 flash attention (csrc/attn_kernels.hip) against an fp32 PyTorch reference of the same op:
softmax(q k^T * scale [+ causal mask]) v with GQA, forward and dQ / dK / dV."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(q, k, v, causal, scale):
    rep = q.shape[1] // k.shape[1]
    kk = k.float().repeat_interleave(rep, 1)
    vv = v.float().repeat_interleave(rep, 1)
    s = torch.einsum("bhqd,bhkd->bhqk", q.float(), kk) * scale
    if causal:
        S, Sk = q.shape[2], k.shape[2]
        m = torch.ones(S, Sk, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(m, float("-inf"))
    return torch.einsum("bhqk,bhkd->bhqd", s.softmax(-1), vv).transpose(1, 2)  # [B, S, H, D]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


CASES = [
    (2, 4, 4, 256, 64, True),
    (1, 8, 2, 384, 128, True),
    (2, 4, 2, 200, 128, True),   # sequence not a multiple of the 128-row / 64-key tiles
    (1, 4, 4, 256, 128, False),
    (2, 6, 2, 136, 64, False),
    (1, 2, 1, 1024, 128, True),
]


@pytest.mark.parametrize("B,H,Hkv,S,D,causal", CASES)
def test_flash_attention_matches_fp32_reference(cuda, B, H, Hkv, S, D, causal):
    from polyaxon_amd.ops.attention import flash_attention

    torch.manual_seed(0)
    q = torch.randn(B, H, S, D, device=cuda).to(torch.bfloat16).requires_grad_()
    k = torch.randn(B, Hkv, S, D, device=cuda).to(torch.bfloat16).requires_grad_()
    v = torch.randn(B, Hkv, S, D, device=cuda).to(torch.bfloat16).requires_grad_()
    scale = 1.0 / math.sqrt(D)
    out = flash_attention(q, k, v, causal=causal)
    assert out.shape == (B, S, H, D) and out.dtype == torch.bfloat16
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref = _ref(qr, kr, vr, causal, scale)
    assert _rel(out, ref) < 1e-2, _rel(out, ref)
    assert float((out.float() - ref).abs().max()) < 3e-2
    g = torch.randn_like(ref)
    out.backward(g.to(torch.bfloat16))
    ref.backward(g)
    for name, a, b in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        assert _rel(a, b) < 2e-2, (name, _rel(a, b))


def test_flash_attention_large_logit_spikes(cuda):
    """A key row that dominates late tiles forces big running-max jumps (the online-softmax rescale path)."""
    from polyaxon_amd.ops.attention import flash_attention

    torch.manual_seed(1)
    B, H, S, D = 1, 2, 512, 128
    q = torch.randn(B, H, S, D, device=cuda)
    k = torch.randn(B, H, S, D, device=cuda)
    v = torch.randn(B, H, S, D, device=cuda)
    k[:, :, 300] = q[:, :, 400] * 4.0   # query 400 sees a huge score at key 300 (tile 4 of 8)
    k[:, :, 70] = q[:, :, 90] * 3.0
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    out = flash_attention(q, k, v, causal=True)
    ref = _ref(q, k, v, True, 1 / math.sqrt(D))
    assert _rel(out, ref) < 1e-2
    assert float((out.float() - ref).abs().max()) < 5e-2


def test_transformer_uses_hip_attention(cuda):
    """The LM block runs the HIP kernel (no SDPA) and trains: loss falls on a repeated batch."""
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops import _native

    torch.manual_seed(0)
    cfg = tiny_llama(d_model=256, n_heads=2, n_kv_heads=1, max_seq_len=128)  # head_dim 128, GQA 2:1
    m = Transformer(cfg).to(cuda)
    opt = torch.optim.AdamW(m.parameters(), lr=3e-3)
    tok = torch.randint(0, cfg.vocab_size, (2, 128), device=cuda)
    losses = []
    for _ in range(30):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = lm_loss(m(tok), tok)
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0] * 0.7
    assert "plx_attn" in _native._loaded


@pytest.mark.parametrize("waves", [4, 8])
def test_flash_attention_forward_wave_counts(cuda, waves):
    """Both forward workgroup shapes (4 waves / 128 queries, 8 waves / 256 queries) against fp32, causal and full,
    with a sequence that leaves a ragged last query block and key tile."""
    from polyaxon_amd.ops import attention

    lib = attention._lib()
    lib.plx_attn_set_fwd_waves(waves)
    try:
        torch.manual_seed(2)
        for causal, D in ((True, 128), (False, 64), (True, 64)):
            q = torch.randn(2, 4, 328, D, device=cuda).to(torch.bfloat16)
            k = torch.randn(2, 2, 328, D, device=cuda).to(torch.bfloat16)
            v = torch.randn(2, 2, 328, D, device=cuda).to(torch.bfloat16)
            out = attention.flash_attention(q, k, v, causal=causal)
            ref = _ref(q, k, v, causal, 1 / math.sqrt(D))
            assert _rel(out, ref) < 1e-2, (waves, causal, D, _rel(out, ref))
    finally:
        lib.plx_attn_set_fwd_waves(8)


@pytest.mark.parametrize("dq_waves,dkdv_waves", [(4, 4), (8, 8)])
def test_flash_attention_backward_wave_counts(cuda, dq_waves, dkdv_waves):
    """Both dQ and dK/dV workgroup shapes against the fp32 reference: GQA and plain heads, causal and full, a
    sequence that leaves ragged key blocks (the 8-wave dK/dV block is 256 keys)."""
    from polyaxon_amd.ops import attention

    lib = attention._lib()
    lib.plx_attn_set_dq_waves(dq_waves)
    lib.plx_attn_set_dkdv_waves(dkdv_waves)
    try:
        torch.manual_seed(3)
        for H, Hkv, causal, D in ((4, 2, True, 128), (4, 4, False, 64), (2, 2, True, 128)):
            q = torch.randn(1, H, 328, D, device=cuda).to(torch.bfloat16).requires_grad_()
            k = torch.randn(1, Hkv, 328, D, device=cuda).to(torch.bfloat16).requires_grad_()
            v = torch.randn(1, Hkv, 328, D, device=cuda).to(torch.bfloat16).requires_grad_()
            out = attention.flash_attention(q, k, v, causal=causal)
            qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
            ref = _ref(qr, kr, vr, causal, 1 / math.sqrt(D))
            g = torch.randn_like(ref)
            out.backward(g.to(torch.bfloat16))
            ref.backward(g)
            for name, x, y in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
                assert _rel(x, y) < 2e-2, (dq_waves, dkdv_waves, H, Hkv, causal, D, name, _rel(x, y))
    finally:
        lib.plx_attn_set_dq_waves(8)
        lib.plx_attn_set_dkdv_waves(8)
