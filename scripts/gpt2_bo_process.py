"""BASELINE config 4 in PROCESS mode: the same 16-trial Bayesian-GP group over GPT-2 125M as
``bench.py --config gpt2_bo`` (same seed, matrix, acquisition, 100 steps of bs 16 x 1024 on the copy task), but
every trial is a fresh ``python -m polyaxon_amd.trainers lm`` process spawned by polyflow -- the reference's model
(a pod per trial, /root/reference/polyaxon/hpsearch/tasks/bo.py).  Prints one JSON line: trials/h, best loss and
the trial-to-trial gap (next trial's start - previous trial's finish, from the store's timestamps).

    python scripts/gpt2_bo_process.py [--steps 100] [--initial 4] [--iterations 3] [--concurrency 4]
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

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--initial", type=int, default=4)
    ap.add_argument("--iterations", type=int, default=3)
    ap.add_argument("--concurrency", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--model", default="gpt2_125m")
    ap.add_argument("--bs", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    args = ap.parse_args()
    import yaml

    cmd = (f"{sys.executable} -m polyaxon_amd.trainers lm --model {args.model} --bs {args.bs} --seq {args.seq} "
           f"--steps {args.steps} --log_every {args.steps} --data copy "
           "--lr={{ lr }} --weight_decay={{ weight_decay }} --beta2={{ beta2 }}")
    spec = {"version": 1, "kind": "group", "project": "gpt2_bo_process",
            "hptuning": {"seed": args.seed, "concurrency": args.concurrency,
                         "matrix": {"lr": {"loguniform": [math.log(1e-4), math.log(3e-3)]},
                                    "weight_decay": {"uniform": [0.0, 0.2]},
                                    "beta2": {"uniform": [0.9, 0.999]}},
                         "bo": {"n_initial_trials": args.initial, "n_iterations": args.iterations,
                                "n_suggestions": args.concurrency,
                                "metric": {"name": "loss", "optimization": "minimize"},
                                "utility_function": {"acquisition_function": "ucb", "kappa": 1.5,
                                                     "gaussian_process": {"kernel": "matern", "length_scale": 1.0,
                                                                          "nu": 2.5},
                                                     "n_warmup": 10000, "n_iter": 8}}},
            "environment": {"resources": {"gpu": 1}},
            "run": {"cmd": cmd}}
    root = tempfile.mkdtemp(prefix="plx_bo_proc_")
    path = os.path.join(root, "gpt2_bo_process.yml")
    with open(path, "w") as f:
        yaml.safe_dump(spec, f)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PLX_ROOT=os.path.join(root, "plx"),
               PYTHONPATH=os.pathsep.join(p for p in (repo, os.environ.get("PYTHONPATH", "")) if p))
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "polyaxon_amd.cli", "-p", "gpt2_bo_process", "run", "-f", path,
                        "--gpus", "1"], env=env, capture_output=True, text=True, cwd=repo)
    wall = time.time() - t0
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-3000:] + r.stderr[-3000:])
        raise SystemExit(r.returncode)
    from polyaxon_amd.polyflow.paths import Paths
    from polyaxon_amd.store.db import Store

    st = Store(os.path.join(Paths(env["PLX_ROOT"]).root, "polyaxon.sqlite"))
    xs = [x for x in st.list_experiments() if x.get("group_id") is not None]
    done = sorted((x for x in xs if x["started_at"] and x["finished_at"]), key=lambda x: x["started_at"])
    losses = [x["last_metric"].get("loss") for x in done if isinstance(x.get("last_metric"), dict)]
    losses = [v for v in losses if v is not None]
    gaps = [b["started_at"] - a["finished_at"] for a, b in zip(done, done[1:])]
    span = done[-1]["finished_at"] - done[0]["started_at"] if done else float("nan")
    durs = sorted(x["finished_at"] - x["started_at"] for x in done)
    print(json.dumps({"bench": "gpt2_bo_process_mode", "trials": len(done), "statuses": sorted({x["status"] for x in xs}),
                      "trials_per_hour": round(3600 * len(done) / span, 1) if done else None,
                      "sweep_s": round(span, 1), "wall_s": round(wall, 1), "best_loss": min(losses) if losses else None,
                      "trial_s_median": round(durs[len(durs) // 2], 2) if durs else None,
                      "gap_s_median": round(sorted(gaps)[len(gaps) // 2], 3) if gaps else None,
                      "gap_s_max": round(max(gaps), 3) if gaps else None,
                      "steps_per_trial": args.steps, "tokens_per_trial": args.steps * args.bs * args.seq,
                      "data": "synthetic copy task (ops/synth.py), random-init GPT-2 125M"}))


if __name__ == "__main__":
    main()
