#!/usr/bin/env python3
"""Benchmarks for the BASELINE.json configs other than the headline (bench.py), one JSON line per result.

    python scripts/bench_suite.py --only iris,hb_reduce,bo,mlp_grid,lm_gpt2,lm_llama8b [--quick]

* ``iris``       config 1: tracked in-process run latency and metric-ingest rate of the tracking client
                 (reference: one REST POST per metric, throttled at 20 req/s -- BASELINE.md design constants).
* ``mlp_grid``   config 2: grid lr x bs over the 2-layer MLP through the polyflow scheduler, 4 concurrent trials
                 on one GPU (gpu: 0.25 each); trials/hour, trial-to-trial gap, peak concurrency.
* ``hb_reduce``  SURVEY.md §6 protocol 1: Hyperband rung reduction for 64 brackets x 81 configs, device top-k
                 kernel vs the reference's per-bracket Python sort.
* ``bo``         SURVEY.md §6 protocol 1: BO suggestion latency (GP fit + acquisition maximisation) at
                 n_obs in {10, 100, 1000}, d in {3, 8, 16}, m in {5, 1e5}: reference-exact backend (sklearn
                 GPR Matern nu=1.9 + scipy L-BFGS-B, the reference's algorithm) vs the HIP backend.
* ``lm_gpt2``    config 4 compute: GPT-2 125M bf16 training tokens/s on one GPU (a DP=2 trial is two of these
                 plus the RCCL all-reduce, measured by the driver's multi-GPU runs).
* ``lm_llama8b`` config 5 compute: Llama-3 8B bf16 training tokens/s and step time on ONE GPU (DP=1; the DP=8
                 job adds the bucketed RCCL all-reduce over xGMI).
Synthetic data and random-init weights throughout (no datasets / checkpoints on the box).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def emit(rec: dict) -> None:
    print(json.dumps(rec), flush=True)


# ------------------------------------------------------------------------------------------- config 1
def bench_iris(quick: bool) -> None:
    from sklearn.datasets import load_iris
    from sklearn.linear_model import LogisticRegression
    from sklearn.model_selection import cross_val_score

    from polyaxon_amd.client import Experiment

    tmp = tempfile.mkdtemp(prefix="plx-iris-")
    store = os.path.join(tmp, "polyaxon.sqlite")
    X, y = load_iris(return_X_y=True)
    lat = []
    for i in range(3 if quick else 10):
        t0 = time.perf_counter()
        with Experiment(project="iris", store_path=store) as xp:
            xp.log_params(C=1.0, max_iter=200)
            scores = cross_val_score(LogisticRegression(C=1.0, max_iter=200), X, y, cv=5)
            for fold, s in enumerate(scores):
                xp.log_metrics(step=fold, accuracy=float(s))
            xp.log_metrics(accuracy_mean=float(scores.mean()))
        lat.append((time.perf_counter() - t0) * 1e3)
    n = 2000 if quick else 20000
    with Experiment(project="iris", store_path=store) as xp:
        t0 = time.perf_counter()
        for i in range(n):
            xp.log_metrics(step=i, loss=1.0 / (i + 1), accuracy=i / n)
        xp.close()
        dt = time.perf_counter() - t0
    emit({"bench": "iris_tracking", "config": "BASELINE config 1 (CPU)", "tracked_run_ms_median": round(sorted(lat)[len(lat) // 2], 1),
          "tracked_run_ms_min": round(min(lat), 1), "metric_ingest_per_s": round(n / dt, 1),
          "reference_ingest_per_s_bound": 20.0, "note": "reference: REST POST per metric, throttle scope 'high' = 20/s"})


# ------------------------------------------------------------------------------------------- config 2
def bench_mlp_grid(quick: bool) -> None:
    from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
    from polyaxon_amd.polyflow.scheduler import Polyflow

    root = tempfile.mkdtemp(prefix="plx-grid-")
    flow = Polyflow(root, allocator=DeviceAllocator([Device(0)])).start()
    steps = 100 if quick else 200
    try:
        spec = {"version": 1, "kind": "group",
                "hptuning": {"concurrency": 4, "matrix": {"lr": {"values": [0.001, 0.003, 0.01, 0.03]},
                                                          "bs": {"values": [128, 256, 512, 1024]}}},
                "environment": {"resources": {"gpu": {"limits": 0.25}}},
                "run": {"cmd": f"PYTHONPATH={ROOT} {sys.executable} -m polyaxon_amd.trainers mlp "
                               f"--lr={{{{ lr }}}} --bs={{{{ bs }}}} --steps={steps}"}}
        t0 = time.time()
        g = flow.submit(spec, cwd=ROOT)
        status = flow.wait("group", g["id"], timeout=1200)
        wall = time.time() - t0
        xps = flow.store.list_experiments(group_id=g["id"], sort="metric.loss")
        spans = sorted((x["started_at"], x["finished_at"]) for x in xps if x["started_at"] and x["finished_at"])
        peak = max(sum(1 for s, f in spans if s <= t < f) for t, _ in spans) if spans else 0
        gaps = sorted(flow.stats["gaps_ms"])
        durs = sorted(f - s for s, f in spans)
        emit({"bench": "mlp_grid", "config": "BASELINE config 2: grid lr x bs, 2-layer MLP, 1 GPU, 4 concurrent",
              "status": status, "trials": len(xps), "wall_s": round(wall, 2),
              "trials_per_hour": round(len(xps) / wall * 3600, 1), "peak_concurrency": peak,
              "trial_s_median": round(durs[len(durs) // 2], 2) if durs else None,
              "gap_ms_median": round(gaps[len(gaps) // 2], 2) if gaps else None,
              "gap_ms_max": round(gaps[-1], 2) if gaps else None,
              "best": {k: xps[0]["declarations"].get(k) for k in ("lr", "bs")} if xps else None,
              "best_loss": xps[0]["last_metric"].get("loss") if xps else None,
              "reference_gap_floor_s": "1 s countdown hops + 30 s start poll (BASELINE.md)"})
    finally:
        flow.shutdown()


# ------------------------------------------------------------------------------------------- HB reduction
def bench_hb_reduce(quick: bool) -> None:
    import numpy as np
    import torch

    from polyaxon_amd.polytune.kernels import topk_order

    B, C = 64, 81
    rng = np.random.RandomState(0)
    m = rng.rand(B, C).astype(np.float32)
    counts = np.full(B, C, dtype=np.int32)
    # reference: per bracket, sort (id, metric) pairs and keep the top n (iteration_managers/hyperband.py:52-77)
    reps = 20 if quick else 200
    t0 = time.perf_counter()
    for _ in range(reps):
        for b in range(B):
            pairs = sorted(((i, float(m[b, i])) for i in range(C)), key=lambda t: t[1])
            _ = [i for i, _ in pairs[:C // 3]]
    ref_us = (time.perf_counter() - t0) / reps * 1e6
    rec = {"bench": "hb_reduce", "brackets": B, "configs": C, "reference_python_sort_us": round(ref_us, 1)}
    if torch.cuda.is_available():
        dev = torch.device("cuda", 0)
        md, cd = torch.from_numpy(m).to(dev), torch.from_numpy(counts).to(dev)
        for _ in range(10):
            topk_order(md, cd, maximize=False)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(reps):
            order = topk_order(md, cd, maximize=False)
        ev1.record()
        torch.cuda.synchronize()
        rec["hip_topk_us"] = round(ev0.elapsed_time(ev1) / reps * 1e3, 2)
        ref_order = np.argsort(m, axis=1, kind="stable")
        rec["hip_matches_reference"] = bool(np.array_equal(order.cpu().numpy()[:, :C], ref_order))
    emit(rec)


# ------------------------------------------------------------------------------------------- BO latency
def _bo_cfg(d: int, m: int, n_iter: int):
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    return HPTuningConfig.from_dict({
        "seed": 7,
        "bo": {"n_iterations": 10, "n_initial_trials": 5, "metric": {"name": "loss", "optimization": "minimize"},
               "utility_function": {"acquisition_function": "ucb", "kappa": 2.576, "n_warmup": m, "n_iter": n_iter,
                                    "gaussian_process": {"kernel": "matern", "length_scale": 1.0, "nu": 1.9,
                                                         "n_restarts_optimizer": 0}}},
        "matrix": {f"x{i}": {"uniform": [-2.0, 2.0]} for i in range(d)}})


def bench_bo(quick: bool, backends) -> None:
    import numpy as np

    from polyaxon_amd.polytune.bo import BOOptimizer

    grid = [(n, d, m) for n in (10, 100, 1000) for d in (3, 8, 16) for m in (5, 100000)]
    if quick:
        grid = [(n, d, m) for (n, d, m) in grid if d == 8]
    for n, d, m in grid:
        rng = np.random.RandomState(n * 31 + d)
        configs = [{f"x{i}": float(v) for i, v in enumerate(row)} for row in rng.uniform(-2, 2, size=(n, d))]
        metrics = [float(sum((c[f"x{i}"] - 0.3) ** 2 for i in range(d))) for c in configs]
        rec = {"bench": "bo_suggestion_latency", "n_obs": n, "d": d, "m": m}
        for be in backends:
            # the reference's effort: n_iter = 10 L-BFGS-B seeds; the device backend: 8 batched refinement rounds
            opt = BOOptimizer(_bo_cfg(d, m, 10 if be == "reference" else 8), backend=be)
            opt.add_observations(configs, metrics)
            if be == "hip":
                opt.get_suggestion()  # warm (module load, allocator)
            reps = 1 if (be == "reference" and (n >= 1000 or m > 5)) else 3
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                s = opt.get_suggestion()
                ts.append(time.perf_counter() - t0)
            rec[f"{be}_ms"] = round(min(ts) * 1e3, 2)
            rec[f"{be}_objective"] = round(float(sum((s[f"x{i}"] - 0.3) ** 2 for i in range(d))), 4)
        if "reference_ms" in rec and "hip_ms" in rec:
            rec["speedup"] = round(rec["reference_ms"] / rec["hip_ms"], 2)
        emit(rec)


# ------------------------------------------------------------------------------------------- LMs
def _run_lm(model: str, bs: int, seq: int, steps: int, extra=()) -> dict:
    cmd = [sys.executable, "-m", "polyaxon_amd.trainers", "lm", "--model", model, "--bs", str(bs), "--seq", str(seq),
           "--steps", str(steps), "--log_every", "1000", *extra]
    t0 = time.time()
    p = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, env={**os.environ, "PYTHONPATH": ROOT})
    if p.returncode != 0:
        return {"error": p.stderr[-2000:], "rc": p.returncode}
    out = json.loads(p.stdout.strip().splitlines()[-1])
    out["process_s"] = round(time.time() - t0, 1)
    return out


def bench_lm_gpt2(quick: bool) -> None:
    r = _run_lm("gpt2_125m", 16, 1024, 12 if quick else 30)
    emit({"bench": "lm_gpt2_125m", "config": "BASELINE config 4 compute (per DP rank)", "bs": 16, "seq": 1024, **r})


def bench_lm_llama8b(quick: bool) -> None:
    bs, seq = 1, 4096
    r = _run_lm("llama3_8b", bs, seq, 6 if quick else 10, extra=("--lr", "1e-5"))
    if "tokens_per_s" in r:
        r["ms_per_step"] = round(bs * seq / r["tokens_per_s"] * 1e3, 1)
        # 6*N*T matmul FLOPs + attention 12*L*d*S*T (causal half) ~ model FLOPs utilisation vs 2.5 PF dense bf16
        n_params = r.get("params_m", 8030) * 1e6
        flops_tok = 6 * n_params + 6 * 32 * 4096 * seq
        r["model_tflops"] = round(flops_tok * r["tokens_per_s"] / 1e12, 1)
    emit({"bench": "lm_llama3_8b", "config": "BASELINE config 5 compute, DP=1 (one MI355X)", "bs": bs, "seq": seq, **r})


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="iris,hb_reduce,bo,mlp_grid,lm_gpt2,lm_llama8b")
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--bo-backends", default="reference,hip")
    a = ap.parse_args()
    for name in a.only.split(","):
        t0 = time.time()
        try:
            if name == "bo":
                bench_bo(a.quick, a.bo_backends.split(","))
            else:
                globals()[f"bench_{name}"](a.quick)
        except Exception as e:  # keep going: one JSON line per section either way
            emit({"bench": name, "error": repr(e)[:2000]})
        print(f"[bench_suite] {name} done in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
