"""GPU tests: RMSNorm / LayerNorm HIP kernels vs fp32 reference, transformer/LM trainer, MLP grid group through polyflow."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("rows,d", [(1, 64), (37, 768), (512, 4096), (3, 8192)])
def test_rmsnorm_matches_fp32(cuda, rows, d):
    from polyaxon_amd.ops.rmsnorm import rms_norm, rms_norm_reference

    torch.manual_seed(0)
    x = (torch.randn(rows, d, device=cuda) * 3).to(torch.bfloat16).requires_grad_()
    w = (torch.rand(d, device=cuda) + 0.5).requires_grad_()
    y = rms_norm(x, w, 1e-5)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    yr = rms_norm_reference(xr, wr, 1e-5)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    g = torch.randn(rows, d, device=cuda).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-2 * rows ** 0.5)


@pytest.mark.parametrize("rows,d", [(1, 64), (37, 768), (5000, 768), (6001, 1024), (70000, 512), (4099, 1032),
                                    (3, 8192)])
def test_layernorm_matches_fp32(cuda, rows, d):
    """Fused bf16 LayerNorm (csrc/rmsnorm.hip plx_ln_*) vs fp32 F.layer_norm: output, dx, dweight, dbias; an input
    with a large offset exercises the two-pass (mean, then centred variance) statistics."""
    from polyaxon_amd.ops.rmsnorm import layer_norm, layer_norm_reference

    torch.manual_seed(0)
    x = (torch.randn(rows, d, device=cuda) * 3 + 20).to(torch.bfloat16).requires_grad_()
    w = (torch.rand(d, device=cuda) + 0.5).requires_grad_()
    b = torch.randn(d, device=cuda).requires_grad_()
    y = layer_norm(x, w, b, 1e-5)
    assert y.dtype == torch.bfloat16
    xr = x.detach().float().requires_grad_()
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = layer_norm_reference(xr, wr, br, 1e-5)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    g = torch.randn(rows, d, device=cuda).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=3e-2 * float(xr.grad.abs().max()))
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-2 * rows ** 0.5)
    torch.testing.assert_close(b.grad, br.grad, rtol=2e-2, atol=2e-2 * rows ** 0.5)


def test_tiny_llama_trains_on_gpu(cuda):
    from polyaxon_amd.trainers import train_lm

    # one fixed batch: fresh random tokens every step cannot go below ln(vocab) = 5.55
    loss = train_lm(["--model", "tiny", "--steps", "30", "--bs", "8", "--seq", "64", "--lr", "3e-3", "--fixed_batch"])
    assert loss < 5.0


def test_mlp_grid_group_on_gpu(tmp_path):
    """BASELINE config 2 through polyflow: 4 concurrent trials sharing GPU 0 (gpu: 0.25 each)."""
    from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
    from polyaxon_amd.polyflow.scheduler import Polyflow

    flow = Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0)])).start()
    try:
        spec = {"version": 1, "kind": "group",
                "hptuning": {"concurrency": 4, "matrix": {"lr": {"values": [0.01, 0.05]},
                                                          "bs": {"values": [128, 256]}}},
                "environment": {"resources": {"gpu": {"limits": 0.25}}},
                "run": {"cmd": f"PYTHONPATH={ROOT}${{PYTHONPATH:+:$PYTHONPATH}} {sys.executable} -m polyaxon_amd.trainers mlp "
                               "--lr={{ lr }} --bs={{ bs }} --steps=50"}}
        g = flow.submit(spec, cwd=ROOT)
        assert flow.wait("group", g["id"], timeout=600) == "succeeded"
        xps = flow.store.list_experiments(group_id=g["id"], sort="metric.loss")
        assert len(xps) == 4 and all(x["status"] == "succeeded" for x in xps)
        assert all("loss" in x["last_metric"] for x in xps)
        spans = sorted((x["started_at"], x["finished_at"]) for x in xps)
        assert max(sum(1 for s, f in spans if s <= t < f) for t, _ in spans) >= 2  # really concurrent
    finally:
        flow.shutdown()


@pytest.mark.parametrize("rows,d", [(37, 768), (4099, 1024), (300, 264)])
def test_add_layernorm_matches_fp32(cuda, rows, d):
    """Fused residual add + LayerNorm (plx_add_ln_forward / _backward) vs the bf16 add then fp32 F.layer_norm: both
    outputs, the gradient of both inputs (norm backward + residual gradient), dweight, dbias."""
    from polyaxon_amd.ops.rmsnorm import add_layer_norm, layer_norm_reference

    torch.manual_seed(1)
    x = (torch.randn(rows, d, device=cuda) * 2 + 5).to(torch.bfloat16).requires_grad_()
    r = torch.randn(rows, d, device=cuda).to(torch.bfloat16).requires_grad_()
    w = (torch.rand(d, device=cuda) + 0.5).requires_grad_()
    b = torch.randn(d, device=cuda).requires_grad_()
    s, y = add_layer_norm(x, r, w, b, 1e-5)
    sr = (x.detach() + r.detach()).float().requires_grad_()  # the bf16 add, then fp32
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = layer_norm_reference(sr, wr, br, 1e-5)
    assert torch.equal(s, (x + r).detach())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    gs = torch.randn(rows, d, device=cuda).to(torch.bfloat16)
    gy = torch.randn(rows, d, device=cuda).to(torch.bfloat16)
    torch.autograd.backward([s, y], [gs, gy])  # both gradients at once: the fused dx = LN backward + ds kernel
    yr.backward(gy.float())
    ref_dx = sr.grad + gs.float()
    torch.testing.assert_close(x.grad.float(), ref_dx, rtol=3e-2, atol=3e-2 * float(ref_dx.abs().max()))
    torch.testing.assert_close(r.grad.float(), ref_dx, rtol=3e-2, atol=3e-2 * float(ref_dx.abs().max()))
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-2 * rows ** 0.5)
    torch.testing.assert_close(b.grad, br.grad, rtol=2e-2, atol=2e-2 * rows ** 0.5)


@pytest.mark.parametrize("arch", ["gpt2", "llama"])
def test_fused_residual_norm_path_matches_block_path(cuda, arch):
    """Transformer.forward (every residual add fused into the next LayerNorm / RMSNorm) against the plain
    Block.forward loop on the same weights: logits and the loss gradient of every parameter."""
    from polyaxon_amd.models.transformer import Transformer, gpt2_125m, lm_loss, tiny_llama

    torch.manual_seed(0)
    cfg = (gpt2_125m(vocab_size=512, n_layers=2, d_model=256, n_heads=4, d_ff=1024, max_seq_len=128) if arch == "gpt2"
           else tiny_llama(vocab_size=512, d_model=256, n_heads=4, n_kv_heads=2, d_ff=512, max_seq_len=128))
    with torch.device(cuda):
        model = Transformer(cfg)
    tok = torch.randint(0, 512, (2, 128), device=cuda)

    def block_path(m):
        x = m.embed(tok)
        rope = None
        if m.pos is not None:
            x = x + m.pos(torch.arange(tok.shape[1], device=cuda))[None]
        else:
            m(tok[:, :2])  # builds the rope cache
            rope = (m._rope[0][:tok.shape[1]], m._rope[1][:tok.shape[1]])
        for blk in m.blocks:
            x = blk(x, rope)
        x = m.norm(x)
        return torch.nn.functional.linear(x, m.embed.weight if m.head is None else m.head.weight)

    out = {}
    for name, fn in (("fused", model), ("blocks", block_path)):
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = model(tok) if name == "fused" else fn(model)
            loss = lm_loss(logits, tok)
        loss.backward()
        out[name] = (logits.float(), {n: p.grad.float().clone() for n, p in model.named_parameters()})
    torch.testing.assert_close(out["fused"][0], out["blocks"][0], rtol=3e-2, atol=3e-2)
    for n, g in out["blocks"][1].items():
        gf = out["fused"][1][n]
        assert float((gf - g).norm()) <= 0.03 * float(g.norm()) + 1e-6, n



@pytest.mark.parametrize("rows,d", [(37, 4096), (300, 264)])
def test_add_rmsnorm_matches_fp32(cuda, rows, d):
    """Fused residual add + RMSNorm (plx_add_rms_forward / _backward) vs the bf16 add then the fp32 reference: both
    outputs, the gradient of both inputs (norm backward + residual gradient in one pass) and dweight."""
    from polyaxon_amd.ops.rmsnorm import add_rms_norm, rms_norm_reference

    torch.manual_seed(2)
    x = torch.randn(rows, d, device=cuda).to(torch.bfloat16).requires_grad_()
    r = torch.randn(rows, d, device=cuda).to(torch.bfloat16).requires_grad_()
    w = (torch.rand(d, device=cuda) + 0.5).requires_grad_()
    s, y = add_rms_norm(x, r, w, 1e-5)
    sr = (x.detach() + r.detach()).float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    xf = sr
    yr = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    assert torch.equal(s, (x + r).detach())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    gs = torch.randn(rows, d, device=cuda).to(torch.bfloat16)
    gy = torch.randn(rows, d, device=cuda).to(torch.bfloat16)
    torch.autograd.backward([s, y], [gs, gy])
    yr.backward(gy.float())
    ref_dx = sr.grad + gs.float()
    torch.testing.assert_close(x.grad.float(), ref_dx, rtol=3e-2, atol=3e-2 * float(ref_dx.abs().max()))
    torch.testing.assert_close(r.grad.float(), ref_dx, rtol=3e-2, atol=3e-2 * float(ref_dx.abs().max()))
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-2 * rows ** 0.5)


def test_padded_gpt2_vocab_head_on_gemm256(cuda, monkeypatch):
    """GPT-2's real vocabulary (50257) padded to 50432 rows: the tied head, its data gradient and the tied-weight
    gradient run on gemm256 (PLX_LM_GEMM=1) with the -inf logit bias in the epilogue; loss and gradients match the
    unpadded model (head on hipBLASLt, 50257 is no gemm256 shape), the padding rows get a zero gradient."""
    from polyaxon_amd.models.transformer import Transformer, gpt2_125m, lm_loss
    from polyaxon_amd.ops import gemm

    monkeypatch.setenv("PLX_LM_GEMM", "1")
    kw = dict(n_layers=1, d_model=256, n_heads=4, d_ff=1024, max_seq_len=256)
    torch.manual_seed(0)
    with torch.device(cuda):
        mp = Transformer(gpt2_125m(**kw)).to(torch.bfloat16)
        mu = Transformer(gpt2_125m(vocab_multiple=1, **kw)).to(torch.bfloat16)
    sd = mp.state_dict()
    sd["embed.weight"] = sd["embed.weight"][:50257]
    mu.load_state_dict(sd)
    assert gemm.supported(512, 50432, 256) and not gemm.supported(512, 50257, 256)
    tok = torch.randint(0, 50257, (2, 256), device=cuda)
    res = {}
    for name, m in (("padded", mp), ("plain", mu)):
        logits = m(tok)
        assert ("Mfma" in type(logits.grad_fn).__name__) == (name == "padded"), type(logits.grad_fn).__name__
        loss = lm_loss(logits, tok)
        loss.backward()
        res[name] = (float(loss), m.embed.weight.grad.float())
    assert abs(res["padded"][0] - res["plain"][0]) <= 2e-2 * abs(res["plain"][0])
    gp, gu = res["padded"][1], res["plain"][1]
    assert float(gp[50257:].abs().max()) == 0.0
    assert float((gp[:50257] - gu).norm()) <= 0.03 * float(gu.norm())


