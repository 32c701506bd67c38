"""GPU check of the language-model path: causality under bf16 autocast (perturb token t, logits before t must not
move) and the loss trajectory on random tokens (must stay near ln(vocab) for a few steps)."""
import math

import torch

from polyaxon_amd.models.transformer import Transformer, llama3_8b, lm_loss
from polyaxon_amd.ops.flat import FlatParams
from polyaxon_amd.ops.optim import FusedAdamW

dev = torch.device("cuda", 0)
torch.manual_seed(0)
cfg = llama3_8b(n_layers=2)
with torch.device(dev):
    m = Transformer(cfg)
flat = FlatParams(m, dev, channels_last=False)
step = torch.zeros(1, dtype=torch.int32, device=dev)
opt = FusedAdamW(flat, lr=1e-5, betas=(0.9, 0.95), weight_decay=0.0, step_counter=step)
t = torch.randint(0, cfg.vocab_size, (1, 512), device=dev)
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
    a = m(t).float()
    t2 = t.clone()
    t2[:, 300] = (t2[:, 300] + 7) % cfg.vocab_size
    b = m(t2).float()
print("causal leak (max |dlogit| before 300):", (a[:, :300] - b[:, :300]).abs().max().item(),
      " at 300:", (a[:, 300] - b[:, 300]).abs().max().item())
print("ln(vocab) =", math.log(cfg.vocab_size))
for it in range(10):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = lm_loss(m(t), t)
    loss.backward()
    opt.step_()
    step += 1
    print("step", it, "loss", float(loss))
