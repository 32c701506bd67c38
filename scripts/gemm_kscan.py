"""Per-tile fixed cost of the LM GEMM kernel: time one output shape at several K and fit t(K) = a + b K.  ``a`` is
the per-launch cost plus, per output tile round, the ring fill before the K loop and the epilogue after it (what
a persistent, epilogue-overlapped kernel could hide); ``b`` the K loop's rate.  hipBLASLt alongside.

    python scripts/gemm_kscan.py [--M 16384] [--N 50432] [--ks 256,512,768,1536,3072] [--waves 8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polyaxon_amd.ops import gemm  # noqa: E402


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def fit(xs, ys):
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    return my - b * mx, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=50432)
    ap.add_argument("--ks", default="256,512,768,1536,3072")
    ap.add_argument("--waves", type=int, default=8)
    a = ap.parse_args()
    gemm.FORCE_SCHEDULE = a.waves
    dev = torch.device("cuda", 0)
    ks = [int(k) for k in a.ks.split(",")]
    out = torch.empty(a.M, a.N, dtype=torch.bfloat16, device=dev)
    tk, tt = [], []
    for k in ks:
        x = torch.randn(a.M, k, device=dev).to(torch.bfloat16)
        w = (torch.randn(a.N, k, device=dev) * 0.02).to(torch.bfloat16)
        t_k = timed(lambda: gemm.gemm(x, w, a.M, a.N, k, True, True, out=out))
        t_t = timed(lambda: torch.mm(x, w.t(), out=out))
        tk.append(t_k)
        tt.append(t_t)
        print(json.dumps({"M": a.M, "N": a.N, "K": k, "kernel_us": round(t_k, 1), "hipblaslt_us": round(t_t, 1),
                          "kernel_tflops": round(2.0 * a.M * a.N * k / t_k / 1e6, 1),
                          "hipblaslt_tflops": round(2.0 * a.M * a.N * k / t_t / 1e6, 1)}), flush=True)
        del x, w
    tiles = (a.M // 256) * (a.N // 256)
    for name, ys in (("kernel", tk), ("hipblaslt", tt)):
        c0, c1 = fit(ks, ys)
        print(json.dumps({"fit": name, "fixed_us": round(c0, 1), "us_per_64k": round(c1 * 64, 2),
                          "tile_rounds": round(tiles / 256, 2), "fixed_us_per_round": round(c0 / (tiles / 256), 2)}))


if __name__ == "__main__":
    main()
