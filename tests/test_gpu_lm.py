"""GPU tests of the language-model HIP kernels (csrc/lm_kernels.hip) against plain PyTorch fp32 references, and
of the lp-mode (bf16 weights/grads + fp32 master, direct weight-gradient GEMMs) model against the fp32 model."""
import pytest
import torch
import torch.nn.functional as F

from polyaxon_amd.ops import _native

pytestmark = pytest.mark.gpu


def _rope_tables(S, D, theta, dev):
    from polyaxon_amd.models.transformer import rope_cache

    return rope_cache(S, D, theta, dev)


@pytest.mark.parametrize("B,S,H,KV,D,use_rope", [(2, 64, 4, 2, 128, True), (1, 128, 32, 8, 128, True),
                                                 (2, 32, 12, 12, 64, False), (3, 16, 2, 1, 16, True)])
def test_qkv_rope_matches_fp32(cuda, B, S, H, KV, D, use_rope):
    from polyaxon_amd.ops.lm import qkv_rope, qkv_rope_reference

    assert _native.lib("plx_lm") is not None
    torch.manual_seed(0)
    qkv = torch.randn(B, S, (H + 2 * KV) * D, device=cuda).to(torch.bfloat16).requires_grad_()
    rope = _rope_tables(S, D, 500000.0, cuda) if use_rope else None
    q, k, v = qkv_rope(qkv, B, S, H, KV, D, rope)
    assert q.shape == (B, H, S, D) and k.shape == (B, KV, S, D) and v.is_contiguous()
    ref_in = qkv.detach().float().requires_grad_()
    qr, kr, vr = qkv_rope_reference(ref_in, B, S, H, KV, D, rope)
    for a, b in ((q, qr), (k, kr), (v, vr)):
        torch.testing.assert_close(a.float(), b, rtol=1e-2, atol=1e-2)
    gq, gk, gv = (torch.randn_like(t) for t in (q, k, v))
    torch.autograd.backward([q, k, v], [gq, gk, gv])
    torch.autograd.backward([qr, kr, vr], [gq.float(), gk.float(), gv.float()])
    torch.testing.assert_close(qkv.grad.float(), ref_in.grad, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("T,Fh", [(1, 8), (37, 1376), (4096, 14336)])
def test_swiglu_matches_fp32(cuda, T, Fh):
    from polyaxon_amd.ops.lm import swiglu, swiglu_reference

    torch.manual_seed(1)
    h = (torch.randn(T, 2 * Fh, device=cuda) * 2).to(torch.bfloat16).requires_grad_()
    a = swiglu(h)
    hr = h.detach().float().requires_grad_()
    ar = swiglu_reference(hr)
    torch.testing.assert_close(a.float(), ar, rtol=1e-2, atol=1e-2)
    g = torch.randn_like(a)
    a.backward(g)
    ar.backward(g.float())
    torch.testing.assert_close(h.grad.float(), hr.grad, rtol=2e-2, atol=2e-2)


def test_lp_model_matches_fp32_model(cuda):
    """tiny Llama: loss and master-weight gradients of the lp path (HIP RoPE/SwiGLU/RMSNorm kernels, bf16 flat
    weights, direct weight-gradient GEMMs) vs the same model in fp32 without any of them."""
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams

    cfg = tiny_llama(d_model=128, n_heads=4, n_kv_heads=2, d_ff=256, vocab_size=512)
    tokens = torch.randint(0, 512, (2, 64), device=cuda)
    torch.manual_seed(0)
    with torch.device(cuda):
        m32 = Transformer(cfg)
    torch.manual_seed(0)
    with torch.device(cuda):
        mlp = Transformer(cfg)
    f32 = FlatParams(m32, cuda, channels_last=False)
    flp = FlatParams(mlp, cuda, channels_last=False, lp_dtype=torch.bfloat16)
    flp.enable_direct_grads(True)
    torch.testing.assert_close(f32.params, flp.params)
    l32 = lm_loss(m32(tokens), tokens)
    l32.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        llp = lm_loss(mlp(tokens), tokens)
    llp.backward()
    assert abs(float(l32) - float(llp)) < 0.05
    assert len(flp._written) > 0  # the direct-gradient GEMMs ran
    g32 = f32.grads
    glp = torch.cat([flp.lp_grads.float(), flp.grads])
    cos = F.cosine_similarity(g32, glp, dim=0)
    assert float(cos) > 0.99, float(cos)
    for seg in f32.segments:  # every parameter gets a gradient of the right size
        a = g32[seg.offset: seg.offset + seg.numel]
        b = glp[seg.offset: seg.offset + seg.numel]
        assert float(b.norm()) > 0 and abs(float(a.norm()) - float(b.norm())) <= 0.1 * float(a.norm()) + 1e-4, seg.name


@pytest.mark.parametrize("arch", ["llama", "gpt2"])
def test_optimizer_in_backward_matches_monolithic_step_on_gpu(cuda, arch):
    """FlatDDP(optimizer=...) on the GPU: per-bucket plx_adamw_mixed / plx_adamw_flat launches on the optimizer
    stream during the backward (lp mode: bf16 weights, fp32 master) give bitwise the trajectory of one update pass
    after the backward, and the main stream sees the updated bf16 weights in the next forward."""
    from polyaxon_amd.models.transformer import Transformer, gpt2_125m, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW
    from polyaxon_amd.parallel.ddp import FlatDDP

    res = {}
    for in_bwd in (False, True):
        torch.manual_seed(0)
        cfg = (tiny_llama(d_model=256, n_heads=2, n_kv_heads=1, max_seq_len=128) if arch == "llama" else
               gpt2_125m(vocab_size=256, n_layers=2, d_model=256, n_heads=2, d_ff=1024, max_seq_len=128))
        with torch.device(cuda):
            model = Transformer(cfg)  # gpt2: tied embeddings, learned positions, LayerNorm, GELU, biases
        flat = FlatParams(model, cuda, channels_last=False, lp_dtype=torch.bfloat16)
        flat.enable_direct_grads(True)
        opt = FusedAdamW(flat, lr=3e-3, weight_decay=0.1)
        ddp = FlatDDP(flat, bucket_mb=0.05, optimizer=opt if in_bwd else None)
        gen = torch.Generator(device=cuda).manual_seed(9)
        losses = []
        for _ in range(4):
            tok = torch.randint(0, 256, (2, 128), device=cuda, generator=gen)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = lm_loss(model(tok), tok)
            loss.backward()
            ddp.finish()
            opt.step_()
            opt.step += 1
            losses.append(float(loss))
        torch.cuda.synchronize()
        res[in_bwd] = (losses, flat.params.clone(), flat.lp_params.clone(), ddp)
    assert res[False][0] == res[True][0]
    assert torch.equal(res[False][1], res[True][1]) and torch.equal(res[False][2], res[True][2])
    d = res[True][3]
    assert len(d.buckets) > 3 and d.stepped == 4 * len(d.buckets)


@pytest.mark.parametrize("B,S,V", [(2, 5, 50257), (3, 17, 256), (1, 2, 1000), (4, 33, 130001), (2, 9, 50432),
                                   (1, 4, 65536)])
def test_next_token_xent_matches_fp32(cuda, B, S, V):
    """The fused cross entropy (csrc/lm_kernels.hip plx_xent_fwd / _bwd) on bf16 logits -- odd vocabularies whose rows
    start mid-chunk included, GPT-2's padded 50432 -- against F.cross_entropy of the same logits in fp32: loss and
    logits gradient (the last position of every sequence gets a zero gradient), with a non-unit incoming gradient."""
    from polyaxon_amd.ops.lm import next_token_xent

    torch.manual_seed(0)
    logits = (torch.randn(B, S, V, device=cuda) * 3).to(torch.bfloat16).requires_grad_()
    tokens = torch.randint(0, V, (B, S), device=cuda)
    loss = next_token_xent(logits, tokens)
    (loss * 1.7).backward()
    ref_in = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(ref_in[:, :-1].reshape(-1, V), tokens[:, 1:].reshape(-1))
    (ref * 1.7).backward()
    assert abs(float(loss) - float(ref)) < 1e-4 * max(1.0, abs(float(ref)))
    g, gr = logits.grad.float(), ref_in.grad
    assert float(g[:, -1].abs().max()) == 0.0
    torch.testing.assert_close(g, gr, rtol=1e-2, atol=1e-2 * float(gr.abs().max()))


def test_next_token_xent_unit_gradient_and_ignored_tokens(cuda):
    """Targets outside [0, V) (-100 and > V) give zero loss rows and zero gradient rows, with the usual unit incoming
    gradient, against F.cross_entropy with ignore_index -- whose mean skips the ignored rows, so the reference is
    rescaled to the fused mean over all rows.  (A one-pass forward+gradient kernel holding each row in registers was
    measured neutral on the GPT-2 step, 711.9-715.0k vs 712.4-715.3k tokens/s, profiles/r6_xent_onepass_ab.jsonl,
    and removed.)"""
    from polyaxon_amd.ops.lm import next_token_xent

    torch.manual_seed(1)
    B, S, V = 2, 12, 50432
    logits = (torch.randn(B, S, V, device=cuda) * 3).to(torch.bfloat16).requires_grad_()
    tokens = torch.randint(0, V, (B, S), device=cuda)
    tokens[0, 3] = -100
    tokens[1, 7] = V + 5
    loss = next_token_xent(logits, tokens)
    loss.backward()
    tgt = tokens[:, 1:].reshape(-1).clone()
    valid = (tgt >= 0) & (tgt < V)
    tgt[~valid] = -100
    ref_in = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(ref_in[:, :-1].reshape(-1, V), tgt, ignore_index=-100, reduction="sum") / tgt.numel()
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-4 * max(1.0, abs(float(ref)))
    g, gr = logits.grad.float(), ref_in.grad
    assert float(g[:, -1].abs().max()) == 0.0 and float(g[0, 2].abs().max()) == 0.0 and float(g[1, 6].abs().max()) == 0.0
    torch.testing.assert_close(g, gr, rtol=1e-2, atol=1e-2 * float(gr.abs().max()))


@pytest.mark.parametrize("N,V", [(256, 1000), (8, 10), (3, 1001), (1, 7), (64, 50257)])
def test_class_xent_matches_fp32(cuda, N, V):
    """The classification variant of the fused cross entropy (plx_xent_cls_fwd / _bwd: the ResNet head's loss in the
    resident executor) against F.cross_entropy of the same logits in fp32: loss and logits gradient with a non-unit
    incoming gradient, row lengths that are not a multiple of 8 bf16 (rows start mid-chunk)."""
    from polyaxon_amd.ops.lm import class_xent

    torch.manual_seed(1)
    logits = (torch.randn(N, V, device=cuda) * 3).to(torch.bfloat16).requires_grad_()
    labels = torch.randint(0, V, (N,), device=cuda)
    loss = class_xent(logits, labels)
    (loss * 1.7).backward()
    ref_in = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(ref_in, labels)
    (ref * 1.7).backward()
    assert abs(float(loss) - float(ref)) < 1e-4 * max(1.0, abs(float(ref)))
    g, gr = logits.grad.float(), ref_in.grad
    torch.testing.assert_close(g, gr, rtol=1e-2, atol=1e-2 * float(gr.abs().max()))


@pytest.mark.parametrize("in_range", [False, True])
def test_class_xent_ignored_and_out_of_range_labels(cuda, in_range):
    """labels outside [0, V) (ignore_index -100, or V itself) are never read; they add no loss and no
    gradient.  Default: the mean is over the valid rows as in F.cross_entropy(ignore_index=-100); ``in_range``
    (caller-guaranteed labels) divides by every row -- checked here on all-valid labels."""
    from polyaxon_amd.ops.lm import class_xent

    N, V = 64, 1000
    torch.manual_seed(3)
    logits = (torch.randn(N, V, device=cuda) * 3).to(torch.bfloat16).requires_grad_()
    labels = torch.randint(0, V, (N,), device=cuda)
    if not in_range:
        labels[::5] = -100
        labels[3] = V  # out of range: treated as ignored (torch would raise)
    loss = class_xent(logits, labels, in_range=in_range)
    (loss * 0.9).backward()
    ref_in = logits.detach().float().requires_grad_()
    ref_labels = labels.clone()
    ref_labels[ref_labels >= V] = -100
    ref = F.cross_entropy(ref_in, ref_labels, ignore_index=-100)
    (ref * 0.9).backward()
    assert abs(float(loss) - float(ref)) < 1e-4 * max(1.0, abs(float(ref)))
    g, gr = logits.grad.float(), ref_in.grad
    torch.testing.assert_close(g, gr, rtol=1e-2, atol=1e-2 * float(gr.abs().max()))
    if not in_range:
        assert float(g[::5].abs().max()) == 0.0 and float(g[3].abs().max()) == 0.0


@pytest.mark.parametrize("T,N", [(16384, 768), (16384, 3072), (1000, 2304), (37, 264), (1, 8)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bias_grad_colsum_matches_fp32(cuda, T, N, dtype):
    """plx_colsum (csrc/lm_kernels.hip, the Linear bias gradient) against an fp64 column sum of the same bf16 matrix:
    tiles that end mid-tile (N % 64 != 0), a single row, both output dtypes, and bitwise-identical repeats (the
    last-arriver reduction runs in a fixed order)."""
    from polyaxon_amd.ops import lm as lm_ops

    assert _native.available("plx_lm")
    g = torch.Generator(device="cuda").manual_seed(T * 7 + N)
    dy = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
    bias = torch.zeros(N, dtype=dtype, device="cuda")
    out = lm_ops.bias_grad(dy, bias)
    assert out.dtype == dtype and out.shape == (N,)
    ref = dy.double().sum(0)
    tol = 1e-4 * T ** 0.5 + (0.01 * ref.abs().max().item() if dtype == torch.bfloat16 else 0.0)
    torch.testing.assert_close(out.double(), ref, rtol=1e-2 if dtype == torch.bfloat16 else 1e-5, atol=tol)
    assert torch.equal(lm_ops.bias_grad(dy, bias), out)


def test_direct_bias_and_norm_grads_into_flat_slots(cuda):
    """lp-mode flat parameters with direct gradients: the Linear bias (plx_colsum) and LayerNorm weight / bias
    (plx_partial_colsum) gradients land in their fp32 flat slots -- stored by the first backward, accumulated by the
    second -- and match fp32 autograd of the same computation run twice."""
    from polyaxon_amd.ops import lm as lm_ops
    from polyaxon_amd.ops import rmsnorm as rms
    from polyaxon_amd.ops.flat import FlatParams

    torch.manual_seed(3)
    d, n, T = 256, 512, 2048

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.norm = rms.LayerNorm(d)
            self.fc = torch.nn.Linear(d, n)

        def forward(self, x):
            return lm_ops.linear(self.norm(x), self.fc.weight, self.fc.bias)

    ref = M().cuda()
    with torch.no_grad():
        ref.norm.weight.uniform_(0.5, 1.5)
        ref.norm.bias.normal_()
        ref.fc.bias.normal_()
    m = M().cuda()
    m.load_state_dict(ref.state_dict())
    flat = FlatParams(m, torch.device("cuda"), lp_dtype=torch.bfloat16)
    flat.enable_direct_grads(True)
    flat.zero_grads()
    x = torch.randn(T, d, device="cuda").to(torch.bfloat16)
    dy = torch.randn(T, n, device="cuda").to(torch.bfloat16)
    for _ in range(2):
        m(x).backward(dy)
    xr = x.float()
    for _ in range(2):
        y = torch.nn.functional.linear(torch.nn.functional.layer_norm(xr, (d,), ref.norm.weight, ref.norm.bias),
                                       ref.fc.weight.bfloat16().float(), ref.fc.bias)
        y.backward(dy.float())
    for name, rp in (("fc.bias", ref.fc.bias), ("norm.weight", ref.norm.weight), ("norm.bias", ref.norm.bias)):
        slot = flat.parameter(name).grad
        assert slot.dtype == torch.float32
        torch.testing.assert_close(slot, rp.grad, rtol=3e-2, atol=3e-2 * rp.grad.abs().max().item()), name


@pytest.mark.parametrize("T,N", [(16384, 3072), (777, 264)])
def test_gelu_backward_bias_fused_matches_fp32(cuda, T, N):
    """plx_gelu_bwd_colsum (csrc/lm_kernels.hip): dh = dA * gelu_tanh'(h) against fp32 aten.gelu_backward of the same
    bf16 inputs, and the bias gradient against the fp64 column sum of the dh it wrote."""
    from polyaxon_amd.ops import lm as lm_ops

    g = torch.Generator(device="cuda").manual_seed(T + N)
    da = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
    h = (torch.randn(T, N, device="cuda", generator=g) * 3).to(torch.bfloat16)
    bias = torch.zeros(N, device="cuda")
    dh, db = lm_ops.bias_grad(da, bias, gelu_h=h)
    ref = torch.ops.aten.gelu_backward(da.float(), h.float(), approximate="tanh")
    torch.testing.assert_close(dh.float(), ref, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(db.double(), dh.double().sum(0), rtol=1e-5, atol=1e-4 * T ** 0.5)


@pytest.mark.parametrize("arch", ["llama", "gpt2"])
def test_side_stream_weight_gradients_are_bitwise_the_inline_ones(cuda, arch, monkeypatch):
    """The transformer blocks' weight-gradient GEMMs on the side stream (ops/lm.py _WGRAD_SIDE, queued before the data
    gradient they overlap) write the same flat-slot gradients, bit for bit, as the same kernels inline; the loss's
    backward joins the side stream before it returns."""
    from polyaxon_amd.models.transformer import Transformer, gpt2_125m, lm_loss, tiny_llama
    from polyaxon_amd.ops import lm
    from polyaxon_amd.ops.flat import FlatParams

    grads = {}
    for side in (False, True):
        monkeypatch.setattr(lm, "_WGRAD_SIDE", side)
        torch.manual_seed(0)
        cfg = (tiny_llama(d_model=256, n_heads=2, n_kv_heads=1, d_ff=512, max_seq_len=256) if arch == "llama" else
               gpt2_125m(vocab_size=512, n_layers=2, d_model=256, n_heads=2, d_ff=1024, max_seq_len=256))
        with torch.device(cuda):
            model = Transformer(cfg)
        flat = FlatParams(model, cuda, channels_last=False, lp_dtype=torch.bfloat16)
        flat.enable_direct_grads(True)
        tok = torch.randint(0, 256, (2, 256), device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = lm_loss(model(tok), tok)
        loss.backward()
        grads[side] = torch.cat([flat.lp_grads.float(), flat.grads]).clone()
    assert torch.isfinite(grads[True]).all() and float(grads[True].norm()) > 0
    assert torch.equal(grads[True], grads[False])
