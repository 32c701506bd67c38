"""Time LM GEMM shapes on several kernel schedules, interleaved in one process, against torch (hipBLASLt).

    python scripts/gemm_sched_ab.py [--reps 50] [--rounds 3] [--model gpt2|llama] [--variants 5,8,9,9f,torch]

Variants: ``5`` (4-wave), ``8`` (8-wave), ``9`` (persistent stream-K, the planner's own split rule), ``9f``
(stream-K splitting the whole partial wave: plx_gemm256_set_sk_force(1)).  One JSON line per (shape, variant): the
median over rounds of the per-call ms (each round times ``reps`` back-to-back calls with events).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from polyaxon_amd.ops import _native, gemm  # noqa: E402

_LAYOUT = {"fwd": (True, True), "dgrad": (True, False), "wgrad": (False, False)}
SHAPES = [  # GPT-2 125M at 16 x 1024 tokens: the data gradients and forwards whose tile grid is 192 (N = 768)
    ("qkv dgrad", 16384, 768, 2304, "dgrad"), ("up dgrad", 16384, 768, 3072, "dgrad"),
    ("proj dgrad", 16384, 768, 768, "dgrad"), ("head dgrad", 16384, 768, 50432, "dgrad"),
    ("proj fwd", 16384, 768, 768, "fwd"), ("down fwd", 16384, 768, 3072, "fwd"),
]


LLAMA = [  # Llama-3 8B at 1 x 4096 tokens: forwards and data gradients (auto sends most of them to hipBLASLt)
    ("qkv fwd", 4096, 6144, 4096, "fwd"), ("o fwd", 4096, 4096, 4096, "fwd"), ("gateup fwd", 4096, 28672, 4096, "fwd"),
    ("down fwd", 4096, 4096, 14336, "fwd"), ("head fwd", 4096, 128256, 4096, "fwd"),
    ("o dgrad", 4096, 4096, 4096, "dgrad"), ("gateup dgrad", 4096, 4096, 28672, "dgrad"),
    ("down dgrad", 4096, 14336, 4096, "dgrad"), ("head dgrad", 4096, 4096, 128256, "dgrad"),
]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="5,8,9,9f,torch")
    ap.add_argument("--model", default="gpt2", choices=("gpt2", "llama"))
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _native.lib("plx_gemm")
    variants = args.variants.split(",")
    for name, M, N, K, layout in (SHAPES if args.model == "gpt2" else LLAMA):
        ak, bk = _LAYOUT[layout]
        torch.manual_seed(0)
        a = (torch.randn((M, K) if ak else (K, M), device=dev) * 0.5).to(torch.bfloat16)
        b = (torch.randn((N, K) if bk else (K, N), device=dev) * 0.5).to(torch.bfloat16)
        A = a if ak else a.t()
        B = b.t() if bk else b
        ref = (A.float() @ B.float())
        times = {v: [] for v in variants}
        errs = {}
        for _ in range(args.rounds):
            for v in variants:
                def call():
                    if v == "torch":
                        return torch.mm(A, B)
                    gemm.FORCE_SCHEDULE = int(v.rstrip("f"))
                    lib.plx_gemm256_set_sk_force(1 if v.endswith("f") else 0)
                    return gemm.gemm(a, b, M, N, K, ak, bk)
                out = call()
                errs[v] = float((out.float() - ref).abs().max() / ref.abs().max())
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.reps)
        gemm.FORCE_SCHEDULE = 0
        lib.plx_gemm256_set_sk_force(0)
        for v in variants:
            t = sorted(times[v])[len(times[v]) // 2]
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "variant": v, "ms": round(t, 4),
                              "tflops": round(2 * M * N * K / t / 1e9, 1), "rel_err": round(errs[v], 5)}), flush=True)


if __name__ == "__main__":
    main()
