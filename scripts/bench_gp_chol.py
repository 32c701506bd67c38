"""Blocked fp64 Cholesky (csrc/gp_chol.hip) timing: batched factorisations with appended rows.

    python scripts/bench_gp_chol.py            # one JSON line per (nb, n, extra rows) config

Under ``rocprofv3 --kernel-trace --stats`` this splits panel vs trailing-update time.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from polyaxon_amd.polytune.bo import HipGP

    hip = HipGP("cuda")
    rng = np.random.RandomState(0)
    for nb, n, extra in [(1, 1000, 1), (25, 1000, 1), (9, 1000, 1), (1, 1000, 1001), (25, 256, 1), (1, 2048, 1)]:
        M = rng.randn(n, n)
        K = M @ M.T / n + np.eye(n)
        base = torch.zeros((nb, n + extra, n), dtype=torch.float64, device="cuda")
        base[:, :n] = torch.tensor(K, device="cuda")
        base[:, n:] = 1.0
        A = base.clone()
        hip.chol_aug(A, n)
        torch.cuda.synchronize()
        reps = 10
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ms = []
        for _ in range(reps):
            A.copy_(base)
            ev[0].record()
            hip.chol_aug(A, n)
            ev[1].record()
            torch.cuda.synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
        flops = nb * (n ** 3 / 3 + extra * n * n)
        t = float(np.median(ms))
        print(json.dumps({"bench": "gp_chol_aug_f64", "nb": nb, "n": n, "extra_rows": extra, "ms": round(t, 3),
                          "gflops": round(flops / t / 1e6, 1), "panels": (n + 31) // 32}), flush=True)


if __name__ == "__main__":
    main()
