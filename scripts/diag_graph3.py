"""Eager vs hipGraph replay of one ResNet-50 training step from identical state: per-parameter update diff.

Finds which parameter updates differ when the step is replayed from a captured graph."""
import sys

import torch

sys.path.insert(0, ".")
from polyaxon_amd.models.resnet import resnet50  # noqa: E402
from polyaxon_amd.polyflow.executor import ResidentTrialExecutor  # noqa: E402

dev = torch.device("cuda", 0)
native = "--miopen" not in sys.argv
bs = 64
torch.manual_seed(0)
x = torch.randn(bs, 3, 224, 224).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (bs,))
exs = {}
for graph in (False, True):
    ex = ResidentTrialExecutor(resnet50(native_conv=native), (x, y), dev, use_graph=graph)
    ex.capture(warmup=2)
    exs[graph] = ex
deltas = {}
for graph, ex in exs.items():
    ex.reset(seed=7)
    ex.set_hparams(lr=0.1, momentum=0.9, weight_decay=1e-4)
    torch.cuda.synchronize()
    p0 = ex.flat.params.detach().clone()
    ex.run(1)
    torch.cuda.synchronize()
    deltas[graph] = (ex.flat.params.detach() - p0).clone()
    print(f"graph={graph} loss={ex.losses().tolist()}", flush=True)
segs = exs[False].flat.segments
bad = 0
for s in segs:
    a = deltas[False][s.offset:s.offset + s.numel]
    b = deltas[True][s.offset:s.offset + s.numel]
    rel = float((a - b).norm() / (a.norm() + 1e-12))
    if rel > 0.05 or not torch.isfinite(b).all():
        bad += 1
        print(f"DIFF {s.name:40s} rel={rel:.3e} |eager|={float(a.norm()):.3e} |graph|={float(b.norm()):.3e}", flush=True)
print(f"native={native}: {bad} of {len(segs)} parameter updates differ by > 5%")
