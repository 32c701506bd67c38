"""GPT-2's padded vocabulary (models/transformer.py ``vocab_multiple``): 50257 -> 50432 embedding / head rows with a
-inf logit bias on the padding, so the logits GEMMs are gemm256 shapes.  The padded model must be the same function
as the unpadded one: equal loss, equal gradients on every real row, zero gradient on the padding rows."""
import torch

from polyaxon_amd.models.transformer import Transformer, gpt2_125m, lm_loss, tiny_llama


def _pair(tie: bool):
    kw = dict(vocab_size=300, n_layers=1, d_model=64, n_heads=2, d_ff=128, max_seq_len=16, tie_embeddings=tie)
    torch.manual_seed(0)
    mp = Transformer(gpt2_125m(**kw))                      # rows padded to 512
    mu = Transformer(gpt2_125m(vocab_multiple=1, **kw))    # 300 rows
    sd = mp.state_dict()
    for k in list(sd):
        if sd[k].shape[:1] == (512,):
            sd[k] = sd[k][:300]
    mu.load_state_dict(sd)
    return mp, mu


def test_vocab_rows_rounding():
    assert gpt2_125m().vocab_rows == 50432 and 50432 % 256 == 0
    assert tiny_llama(vocab_size=128256).vocab_rows == 128256
    assert gpt2_125m(vocab_multiple=1).vocab_rows == 50257


def test_padded_vocab_is_the_same_function():
    for tie in (True, False):
        mp, mu = _pair(tie)
        assert mp.embed.weight.shape[0] == 512 and mu.embed.weight.shape[0] == 300
        tok = torch.randint(0, 300, (2, 16), generator=torch.Generator().manual_seed(1))
        lp_logits = mp(tok)
        assert lp_logits.shape[-1] == 512 and torch.isinf(lp_logits[..., 300:]).all()
        lp, lu = lm_loss(lp_logits, tok), lm_loss(mu(tok), tok)
        torch.testing.assert_close(lp, lu, rtol=1e-5, atol=1e-5)
        lp.backward()
        lu.backward()
        gu = dict(mu.named_parameters())
        for n, p in mp.named_parameters():
            g = p.grad
            if g.shape[:1] == (512,):
                assert float(g[300:].abs().max()) == 0.0, n
                g = g[:300]
            torch.testing.assert_close(g, gu[n].grad, rtol=1e-4, atol=1e-6, msg=n)


def test_lm_trainer_copy_task_learns_on_cpu():
    """``trainers lm --data copy`` (the copy-task stream of the resident GPT-2 program, used by the process-mode BO
    comparison scripts/gpt2_bo_process.py): the loss falls below chance (ln V) within a few hundred steps."""
    import math

    from polyaxon_amd.trainers import train_lm

    loss = train_lm(["--model", "tiny", "--cpu", "--bs", "8", "--seq", "64", "--period", "16", "--steps", "300",
                     "--lr", "3e-3", "--data", "copy", "--log_every", "300"])
    assert math.isfinite(loss) and loss < 0.97 * math.log(256), loss
