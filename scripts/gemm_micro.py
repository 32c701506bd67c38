"""One LM GEMM shape, each kernel schedule (and hipBLASLt) launched `reps` times: the workload for rocprofv3 PMC passes
(scripts/gpu_gemm_pmc.sh).

    python scripts/gemm_micro.py [reps=5] [M N K] [schedules=8,5,7]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from polyaxon_amd.ops import gemm  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    M, N, K = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (4096, 28672, 4096)
    scheds = [int(v) for v in (sys.argv[5] if len(sys.argv) > 5 else "8,5,7").split(",")]
    dev = torch.device("cuda", 0)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    for s in scheds:
        gemm.FORCE_SCHEDULE = s
        for _ in range(reps):
            gemm.gemm(x, w, M, N, K, True, True)
    gemm.FORCE_SCHEDULE = 0
    for _ in range(reps):
        x @ w.t()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
