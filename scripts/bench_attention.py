"""Attention microbenchmark: HIP flash attention vs torch SDPA (AOTriton) at the LM shapes, fwd and fwd+bwd.

    python scripts/bench_attention.py
"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from polyaxon_amd.ops.attention import flash_attention  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    only = sys.argv[1:]  # optional filters: shape names and/or "hip" / "sdpa"
    dev = torch.device("cuda", 0)
    shapes = [("llama3_8b", 1, 32, 8, 4096, 128), ("llama3_8b_s2048_b4", 4, 32, 8, 2048, 128),
              ("gpt2_125m", 16, 12, 12, 1024, 64)]
    impls = [i for i in ("hip", "sdpa") if i in only] or ["hip", "sdpa"]
    for name, B, H, Hkv, S, D in shapes:
        if [o for o in only if o not in ("hip", "sdpa")] and name not in only:
            continue
        torch.manual_seed(0)
        q = torch.randn(B, H, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, Hkv, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, Hkv, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        g = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16)
        flops_fwd = 4 * B * H * S * S * D / 2  # causal
        res = {"shape": name, "B": B, "H": H, "Hkv": Hkv, "S": S, "D": D}
        for impl in impls:
            if impl == "hip":
                f = lambda: flash_attention(q, k, v, causal=True)  # noqa: E731
            else:
                f = lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True,  # noqa: E731
                                                           enable_gqa=H != Hkv).transpose(1, 2)
            with torch.no_grad():
                t_f = timeit(f)

            def fb():
                o = f()
                o.backward(g)

            t_fb = timeit(fb, iters=10)
            res[impl] = {"fwd_ms": round(t_f, 3), "fwd_bwd_ms": round(t_fb, 3),
                         "fwd_tflops": round(flops_fwd / t_f / 1e9, 1),
                         "fwd_bwd_tflops": round(3.5 * flops_fwd / t_fb / 1e9, 1)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
