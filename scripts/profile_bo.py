"""Phase breakdown of one device BO suggestion (LML search, fit, warm-up + refinement + ascent).

    python scripts/profile_bo.py --n 1000 --d 8 --m 100000 [--reps 3]

Prints one JSON line per repetition with per-phase milliseconds (each phase bracketed by a device sync).
Under ``rocprofv3 --kernel-trace --stats`` it gives the per-kernel split of the same suggestion.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--m", type=int, default=100000)
    ap.add_argument("--n-iter", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from polyaxon_amd.polytune.bo import GPState, UtilityFunction, _kind
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    cfg = HPTuningConfig.from_dict({
        "seed": 7,
        "bo": {"n_iterations": 10, "n_initial_trials": 5, "metric": {"name": "loss", "optimization": "minimize"},
               "utility_function": {"acquisition_function": "ucb", "kappa": 2.576, "n_warmup": a.m,
                                    "n_iter": a.n_iter,
                                    "gaussian_process": {"kernel": "matern", "length_scale": 1.0, "nu": 1.9}}},
        "matrix": {f"x{i}": {"uniform": [-2.0, 2.0]} for i in range(a.d)}})
    rng = np.random.RandomState(a.n)
    X = rng.uniform(-2, 2, size=(a.n, a.d))
    y = -np.sum((X - 0.3) ** 2, axis=1)
    bounds = np.array([[-2.0, 2.0]] * a.d)
    uf = UtilityFunction(cfg.bo.utility_function, seed=7, backend="hip")
    g = uf.gp_config

    def sync():
        torch.cuda.synchronize()
        return time.perf_counter()

    for rep in range(a.reps + 1):
        t0 = sync()
        uf.fit(X[:2], y[:2]) if uf._hip is None else None  # builds HipGP / loads the library once
        t0 = sync()
        ls = uf._hip.fit_length_scale(X, y, _kind(g.kernel, g.nu), g.nu, g.length_scale)
        t1 = sync()
        uf._gp = GPState(X, y, ls, _kind(g.kernel, g.nu), g.nu, None, None, float("nan"))
        uf._dev = uf._hip.fit(uf._gp)
        t2 = sync()
        x = uf.max_compute(float(y.max()), bounds, a.m, a.n_iter)
        t3 = sync()
        if rep == 0:
            continue  # warm-up
        print(json.dumps({"n": a.n, "d": a.d, "m": a.m, "rep": rep, "length_scale": round(ls, 5),
                          "lml_search_ms": round((t1 - t0) * 1e3, 2), "fit_ms": round((t2 - t1) * 1e3, 2),
                          "acq_search_ms": round((t3 - t2) * 1e3, 2), "total_ms": round((t3 - t0) * 1e3, 2),
                          "x_objective": round(float(np.sum((x - 0.3) ** 2)), 4)}), flush=True)


if __name__ == "__main__":
    main()
