"""The GPT-2 LM GEMMs on the MFMA kernel (ops/gemm.py gemm) under the conditions of the training step, one at a time:
plain, + fp32 bias epilogue, + bias + GELU second store (the up-projection), and a fresh output allocation per call
(the step's torch.empty), against hipBLASLt (torch) doing the same.  One JSON line per (shape, variant).

    python scripts/lm_gemm_epilogue_ab.py [--reps 20] [--waves 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polyaxon_amd.ops import gemm  # noqa: E402

T = 16 * 1024
SHAPES = [("qkv", 768, 2304), ("proj", 768, 768), ("up", 768, 3072), ("down", 3072, 768), ("head", 768, 50432)]


def timed(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--waves", type=int, default=5)
    a = ap.parse_args()
    gemm.FORCE_SCHEDULE = a.waves
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, fin, fout in SHAPES:
        x = (torch.randn(T, fin, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        w = (torch.randn(fout, fin, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        b = torch.randn(fout, device=dev, generator=g) * 0.1
        dy = (torch.randn(T, fout, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        out = torch.empty(T, fout, dtype=torch.bfloat16, device=dev)
        act = torch.empty_like(out)
        res = {}
        res["plain"] = timed(lambda: gemm.gemm(x, w, T, fout, fin, True, True, out=out), a.reps)
        res["bias"] = timed(lambda: gemm.gemm(x, w, T, fout, fin, True, True, out=out, bias=b), a.reps)
        res["bias_gelu"] = timed(lambda: gemm.gemm(x, w, T, fout, fin, True, True, out=out, bias=b, gelu_out=act),
                                 a.reps)
        res["fresh_out"] = timed(lambda: gemm.gemm(x, w, T, fout, fin, True, True), a.reps)
        res["dgrad"] = timed(lambda: gemm.gemm(dy, w, T, fin, fout, True, False), a.reps)
        bb = b.to(torch.bfloat16)
        res["torch_bias"] = timed(lambda: torch.addmm(bb, x, w.t()), a.reps)
        res["torch_bias_gelu"] = timed(lambda: torch.nn.functional.gelu(torch.addmm(bb, x, w.t()), approximate="tanh"),
                                       a.reps)
        res["torch_dgrad"] = timed(lambda: torch.mm(dy, w), a.reps)
        print(json.dumps({"linear": name, "M": T, "N": fout, "K": fin, **{k: round(v, 1) for k, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
