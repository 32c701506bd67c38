"""Check trial training trajectories: eager vs hipGraph, MIOpen immediate vs find(tune), repeatability."""
import sys, time, torch
sys.path.insert(0, '.')
from polyaxon_amd.models.resnet import resnet50
from polyaxon_amd.polyflow.executor import ResidentTrialExecutor
dev = torch.device('cuda', 0)
tune = '--tune' in sys.argv
bs = int(sys.argv[sys.argv.index('--bs') + 1]) if '--bs' in sys.argv else 256
torch.backends.cudnn.benchmark = tune
x = torch.randn(bs, 3, 224, 224).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (bs,))
for graph in (False, True, True):
    ex = ResidentTrialExecutor(resnet50(), (x, y), dev, use_graph=graph)
    t = time.time(); ex.capture(warmup=3); tc = time.time() - t
    for lr in (0.1, 0.5):
        ex.reset(seed=5)
        ex.set_hparams(lr=lr, momentum=0.9, weight_decay=1e-4)
        ex.run(24)
        torch.cuda.synchronize()
        l = ex.losses().tolist()
        print(f"tune={tune} graph={graph} lr={lr} capture={tc:.1f}s", [round(v, 3) for v in l[::3]], flush=True)
    del ex
