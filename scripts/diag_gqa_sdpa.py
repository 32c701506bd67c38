"""Time SDPA with materialised GQA K/V (repeat_interleave) against enable_gqa=True, fwd+bwd, Llama-3 8B layer shape."""
import torch
import torch.nn.functional as F

dev = torch.device("cuda", 0)
B, S, H, KV, D = 1, 4096, 32, 8, 128
q = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, KV, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, KV, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
g = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16)


def rep():
    kk, vv = k.repeat_interleave(H // KV, 1), v.repeat_interleave(H // KV, 1)
    y = F.scaled_dot_product_attention(q, kk, vv, is_causal=True)
    y.backward(g)
    return y


def gqa():
    y = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
    y.backward(g)
    return y


for name, fn in (("repeat", rep), ("enable_gqa", gqa)):
    try:
        y = fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(name, "ms fwd+bwd:", round(s.elapsed_time(e) / 10, 3), flush=True)
    except Exception as ex:  # noqa
        print(name, "failed:", repr(ex)[:300], flush=True)
q.grad = k.grad = v.grad = None
y1 = rep()
g1 = (q.grad.clone(), k.grad.clone())
q.grad = k.grad = v.grad = None
y2 = gqa()
print("max |dy|", float((y1 - y2).abs().max()), "max |dq|", float((g1[0] - q.grad).abs().max()),
      "max |dk|", float((g1[1] - k.grad).abs().max()))
