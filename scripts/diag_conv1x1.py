"""Time ResNet-50 1x1 convs: MIOpen conv2d vs hipBLASLt GEMM on the NHWC view (fwd + dgrad + wgrad)."""
import torch, time, sys
import torch.nn.functional as F
dev = torch.device('cuda', 0)
torch.backends.cudnn.benchmark = '--tune' in sys.argv
shapes = [(256, 64, 56, 56, 256), (256, 256, 56, 56, 64), (256, 512, 28, 28, 128), (256, 128, 28, 28, 512),
          (256, 1024, 14, 14, 256), (256, 256, 14, 14, 1024), (256, 2048, 7, 7, 512), (256, 512, 7, 7, 2048)]
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / it * 1e3
tot = [0, 0]
for n, cin, h, w, cout in shapes:
    x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_()
    wt = torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_()
    g = torch.randn(n, cout, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    def conv():
        y = F.conv2d(x, wt); y.backward(g)
    x2 = x.detach().permute(0, 2, 3, 1).reshape(-1, cin).requires_grad_()
    w2 = wt.detach().reshape(cout, cin).requires_grad_()
    g2 = g.permute(0, 2, 3, 1).reshape(-1, cout)
    def mm():
        y = x2 @ w2.t(); y.backward(g2)
    a, b = bench(conv), bench(mm)
    tot[0] += a; tot[1] += b
    fl = 3 * 2 * n * h * w * cin * cout
    print(f"{(n,cin,h,w,cout)} miopen {a:.3f} ms ({fl/a/1e9:.0f} TF)  gemm {b:.3f} ms ({fl/b/1e9:.0f} TF)", flush=True)
print("total", tot)
