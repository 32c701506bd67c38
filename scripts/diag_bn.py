import torch, torch.nn.functional as F, sys, time
sys.path.insert(0, '.')
from polyaxon_amd.models.resnet import resnet50
from polyaxon_amd.polyflow.executor import ResidentTrialExecutor
from polyaxon_amd.ops.bn_fused import bn_act
dev = torch.device('cuda', 0)
# 1) op check at large M with S > 1
for shape in [(32, 64, 112, 112), (64, 256, 56, 56), (64, 2048, 7, 7)]:
    x = (torch.randn(shape, device=dev) * 3 + 1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    c = shape[1]
    w = torch.rand(c, device=dev) + 0.5; b = torch.randn(c, device=dev)
    rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
    xa = x.clone().requires_grad_(); wa = w.clone().requires_grad_(); ba = b.clone().requires_grad_()
    y = bn_act(xa, wa, ba, rm, rv, True, 0.1, 1e-5, None, True)
    xr = x.float().requires_grad_(); wr = w.clone().requires_grad_(); br = b.clone().requires_grad_()
    yr = F.relu(F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5))
    g = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(g); yr.backward(g.float())
    print(shape, 'y', float((y.float()-yr).abs().max()), 'dx', float((xa.grad.float()-xr.grad).abs().max()), float(xr.grad.abs().max()),
          'dw', float((wa.grad-wr.grad).abs().max()), float(wr.grad.abs().max()), 'db', float((ba.grad-br.grad).abs().max()), flush=True)
# 2) training curves fused vs unfused
x = torch.randn(64, 3, 224, 224).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (64,))
for fused in (True, False):
    for graph in (False, True):
        ex = ResidentTrialExecutor(resnet50(fused=fused), (x, y), dev, use_graph=graph)
        ex.capture(warmup=2)
        ex.reset(seed=5)
        ex.set_hparams(lr=0.1, momentum=0.9, weight_decay=1e-4)
        ex.run(12)
        torch.cuda.synchronize()
        print('fused', fused, 'graph', graph, [round(v, 3) for v in ex.losses().tolist()], flush=True)
