"""Run one LM GEMM shape a few times on the kernel (a given schedule) and on torch (hipBLASLt), for PMC passes.

    python scripts/gemm_one.py M N K [--layout fwd|dgrad|wgrad] [--sched 9] [--reps 3]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from polyaxon_amd.ops import gemm  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("--layout", default="fwd", choices=("fwd", "dgrad", "wgrad"))
    ap.add_argument("--sched", type=int, default=9)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    M, N, K = args.M, args.N, args.K
    ak, bk = {"fwd": (True, True), "dgrad": (True, False), "wgrad": (False, False)}[args.layout]
    dev = torch.device("cuda", 0)
    a = torch.randn((M, K) if ak else (K, M), device=dev).to(torch.bfloat16)
    b = torch.randn((N, K) if bk else (K, N), device=dev).to(torch.bfloat16)
    A = a if ak else a.t()
    B = b.t() if bk else b
    gemm.FORCE_SCHEDULE = args.sched
    for _ in range(args.reps):
        gemm.gemm(a, b, M, N, K, ak, bk)
        torch.mm(A, B)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
