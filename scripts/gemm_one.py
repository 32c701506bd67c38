"""Run one LM GEMM shape on the MFMA kernel a few times (a small target for rocprofv3 counter passes).

    python scripts/gemm_one.py --M 4096 --N 28672 --K 4096 --layout nt --reps 5 [--torch] [--waves 5]

``--torch``: the same product through torch (hipBLASLt) instead; ``--waves``: the kernel schedule (8 or 5).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polyaxon_amd.ops import gemm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=4096)
ap.add_argument("--N", type=int, default=28672)
ap.add_argument("--K", type=int, default=4096)
ap.add_argument("--layout", default="nt", choices=["nt", "nn", "tn"])
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--torch", action="store_true")
ap.add_argument("--waves", type=int, default=0)
a = ap.parse_args()
ak, bk = {"nt": (True, True), "nn": (True, False), "tn": (False, False)}[a.layout]
dev = torch.device("cuda", 0)
A = (torch.rand(a.M * a.K, device=dev) * 2 - 1).to(torch.bfloat16)
B = (torch.rand(a.N * a.K, device=dev) * 2 - 1).to(torch.bfloat16)
gemm.FORCE_SCHEDULE = a.waves
if a.torch:
    Am = A.view(a.M, a.K) if ak else A.view(a.K, a.M).t()
    Bm = B.view(a.N, a.K).t() if bk else B.view(a.K, a.N)
for _ in range(a.reps):
    if a.torch:
        torch.mm(Am, Bm)
    else:
        gemm.gemm(A, B, a.M, a.N, a.K, ak, bk)
torch.cuda.synchronize()
print("ok")
