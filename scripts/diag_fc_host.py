"""Host-side cost per call of the ResNet-50 classifier GEMMs (bs 256, 2048 -> 1000) on hipBLASLt via torch, with the
GPU kept busy so only enqueue time is measured: forward addmm, dgrad mm, wgrad mm; and the autograd backward of the
linear + cross entropy head alone (enqueue time of loss.backward())."""
import json
import time

import torch
import torch.nn.functional as F


def host_us(fn, n=200):
    for _ in range(5):  # library handles, heuristics and allocator warm
        fn()
    torch.cuda.synchronize()
    big = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    for _ in range(20):
        big.fill_(1)  # several ms of GPU work queued first: the loop below measures enqueue time only
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return round((t1 - t0) / n * 1e6, 2)


def main():
    dev = torch.device("cuda", 0)
    x = torch.randn(256, 2048, device=dev, dtype=torch.bfloat16)
    w = torch.randn(1000, 2048, device=dev, dtype=torch.bfloat16)
    b = torch.randn(1000, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(256, 1000, device=dev, dtype=torch.bfloat16)
    y = torch.randint(0, 1000, (256,), device=dev)
    res = {
        "addmm_fwd_us": host_us(lambda: torch.addmm(b, x, w.t())),
        "mm_dgrad_us": host_us(lambda: dy @ w),
        "mm_wgrad_us": host_us(lambda: dy.t() @ x),
        "elementwise_add_us": host_us(lambda: x.add(x)),
    }
    xr = x.clone().requires_grad_()
    wr = w.clone().requires_grad_()
    br = b.clone().requires_grad_()

    def head():
        loss = F.cross_entropy(F.linear(xr, wr, br).float(), y)
        loss.backward()

    res["linear_xent_fwd_bwd_us"] = host_us(head, 100)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
