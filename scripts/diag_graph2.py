"""Find which parameter segments get wrong gradients in the 2nd trial of a graph-replayed executor."""
import sys, torch
sys.path.insert(0, '.')
from polyaxon_amd.models.resnet import resnet50
from polyaxon_amd.polyflow.executor import ResidentTrialExecutor
dev = torch.device('cuda', 0)
torch.backends.cudnn.benchmark = '--tune' in sys.argv
bs = 128
x = torch.randn(bs, 3, 224, 224).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (bs,))
exs = {}
for graph in (False, True):
    ex = ResidentTrialExecutor(resnet50(), (x, y), dev, use_graph=graph)
    ex.capture(warmup=3)
    ex.reset(seed=5); ex.set_hparams(lr=0.1, momentum=0.9, weight_decay=1e-4); ex.run(4)
    ex.reset(seed=5); ex.set_hparams(lr=0.5, momentum=0.9, weight_decay=1e-4)
    torch.cuda.synchronize()
    exs[graph] = ex
a, b = exs[False], exs[True]
print('after reset: params equal', torch.equal(a.flat.params, b.flat.params), 'mom', float(b.opt.momentum_buf.abs().max()),
      'grads', float(a.flat.grads.abs().max()), float(b.flat.grads.abs().max()), 'bufs', torch.equal(a.buffers, b.buffers), flush=True)
for ex in (a, b):
    ex.run(1)
torch.cuda.synchronize()
print('loss', a.losses().tolist()[-1], b.losses().tolist()[-1])
bad = 0
for seg in a.flat.segments:
    ga = a.opt.momentum_buf[seg.offset: seg.offset + seg.numel]
    gb = b.opt.momentum_buf[seg.offset: seg.offset + seg.numel]
    rel = float((ga - gb).norm() / (ga.norm() + 1e-12))
    if rel > 0.05:
        bad += 1
        print(f"{seg.name:45s} {seg.shape} rel={rel:.3f} |a|={float(ga.norm()):.4g} |b|={float(gb.norm()):.4g}", flush=True)
print('bad segments', bad, 'of', len(a.flat.segments))
