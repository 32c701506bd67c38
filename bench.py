#!/usr/bin/env python3
"""Headline benchmark: HPO trials/hour (whole node) + wall-clock-to-target, ResNet-50 Hyperband sweep.

BASELINE.json config 3 ("Hyperband/ASHA sweep of ResNet-50 on synthetic ImageNet-shape data, 8×MI355X,
64 brackets").  One rank per GPU (torchrun); every rank is a resident polyflow trial executor running its
own Hyperband brackets (brackets are independent successive-halving runs, so they are spread over GPUs
with no cross-GPU barrier; weak scaling: per-GPU work is fixed as N grows).

A benchmark "step" is ONE trial = one Polyaxon experiment: a ResNet-50 config trained for its rung's
resource (1 resource unit = ``--unit-steps`` full training steps: bf16 forward + backward + fused SGD
update at ``--batch`` 224×224 images), with fresh random weights (restart) or its HBM snapshot (resume
promotion), its metric reduced on the device, and the rung's top-k decided by the HIP kernel.  The timed
region is exactly K trials per rank after W untimed warm-up trials; value = N·K / max-rank-time · 3600.

Data: synthetic ImageNet-shape tensors, random-init weights (no datasets / checkpoints available).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from polyaxon_amd.models.resnet import resnet50  # noqa: E402
from polyaxon_amd.polyflow.executor import ResidentTrialExecutor  # noqa: E402
from polyaxon_amd.polyflow.sweep import HyperbandSweep  # noqa: E402
from polyaxon_amd.polytune.managers import HyperbandSearchManager  # noqa: E402
from polyaxon_amd.spec.hptuning import HPTuningConfig  # noqa: E402

T0 = time.perf_counter()
METRIC = "HPO trials/hour (whole node) + wall-clock-to-target, ResNet-50 Hyperband sweep"


def hptuning(seed: int, max_iter: int, eta: int) -> HPTuningConfig:
    return HPTuningConfig.from_dict({
        "seed": seed,
        "concurrency": 1,
        "hyperband": {"max_iter": max_iter, "eta": eta, "resource": {"name": "units", "type": "int"},
                      "metric": {"name": "loss", "optimization": "minimize"}, "resume": True},
        "matrix": {
            "lr": {"loguniform": [math.log(0.02), math.log(0.8)]},
            "momentum": {"uniform": [0.8, 0.95]},
            "weight_decay": {"loguniform": [math.log(1e-5), math.log(1e-3)]},
        },
    })


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=13, help="timed trials per GPU")
    ap.add_argument("--warmup", type=int, default=2, help="untimed warm-up trials per GPU")
    ap.add_argument("--batch", type=int, default=256, help="per-trial batch (one trial per GPU)")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--unit-steps", type=int, default=8, help="training steps per Hyperband resource unit")
    ap.add_argument("--max-iter", type=int, default=9)
    ap.add_argument("--eta", type=int, default=3)
    ap.add_argument("--target", type=float, default=2.0, help="loss target for wall-clock-to-target")
    ap.add_argument("--graph", action="store_true", help="replay the step as a hipGraph (slower for ResNet-50 on ROCm 7, see profiles/README.md)")
    ap.add_argument("--unfused", action="store_true", help="PyTorch BN/ReLU instead of the HIP kernels")
    ap.add_argument("--miopen-1x1", action="store_true", help="MIOpen for the 1x1 convs instead of the MFMA GEMMs")
    ap.add_argument("--tune", action="store_true", help="exhaustive MIOpen find (cudnn.benchmark)")
    ap.add_argument("--verbose", action="store_true", help="print every trial's record to stderr")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    torch.backends.cudnn.benchmark = args.tune

    def log(msg):
        if rank == 0:
            print(f"[bench +{time.perf_counter() - T0:.1f}s] {msg}", file=sys.stderr, flush=True)

    gen = torch.Generator(device="cpu").manual_seed(1234 + rank)
    x = torch.randn(args.batch, 3, args.image, args.image, generator=gen).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), generator=gen)
    model = resnet50(fused=not args.unfused, native_conv=not args.miopen_1x1)
    ex = ResidentTrialExecutor(model, (x, y), dev, use_graph=args.graph)

    log("model built; capturing training step")
    t_cap = time.perf_counter()
    ex.capture()
    capture_s = time.perf_counter() - t_cap
    log(f"captured in {capture_s:.1f}s; warm-up trials")

    # ---- warm-up trials (untimed): same code path as the sweep
    warm = HyperbandSweep(HyperbandSearchManager(hptuning(10_000 + rank, args.max_iter, args.eta)), ex,
                          args.unit_steps, seed=10_000 + rank)
    if args.warmup > 0:
        warm.run(max_trials=args.warmup)
        # plus one short bracket with a rung promotion (snapshot -> top-k reduction -> resume): the first
        # promotion of a cold process otherwise pays ~0.8 s of lazily paged-in library code inside the timed
        # region (measured on a fresh box: trial 9 took 1.2 s instead of 0.42 s)
        HyperbandSweep(HyperbandSearchManager(hptuning(20_000 + rank, 3, 3)), ex, 1, seed=20_000 + rank).run()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    log("timed region")
    # ---- timed region: exactly K trials per rank
    start_ev = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    start_ev.record()
    done, p = 0, 0
    records = []
    while done < args.steps:
        sweep = HyperbandSweep(HyperbandSearchManager(hptuning(rank * 1000 + p + 1, args.max_iter, args.eta)), ex,
                               args.unit_steps, seed=rank * 1000 + p + 1)
        res = sweep.run(max_trials=args.steps - done)
        done += len(res.trials)
        records.extend(res.trials)
        p += 1
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0

    # ---- post-processing (outside the timed region)
    train_steps = sum(r.steps for r in records)
    # wall-clock to target: first trial (by device end time) whose committed metric is <= target
    t_target = math.inf
    for r in records:
        if r.metric is None:
            continue
        if r.metric <= args.target and r.end_event is not None:
            t_target = min(t_target, start_ev.elapsed_time(r.end_event) / 1000.0)
    best = min((r.metric for r in records if r.metric is not None), default=math.nan)
    if args.verbose:
        prev = 0.0
        for r in records:
            t_end = start_ev.elapsed_time(r.end_event) if r.end_event is not None else float("nan")
            log(f"trial {r.trial} cfg {r.config_id} it {r.iteration}/{r.bracket_iteration} res {r.resource} "
                f"steps {r.steps} ends {t_end:.1f} ms (+{t_end - prev:.1f}) metric {r.metric}")
            prev = t_end
    t = torch.tensor([elapsed, -t_target if math.isfinite(t_target) else -math.inf, train_steps, best],
                     dtype=torch.float64, device=dev)
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx[:2], op=dist.ReduceOp.MAX)  # max elapsed, min time-to-target
        tot = t[2:3].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        bst = t[3:4].clone()
        dist.all_reduce(bst, op=dist.ReduceOp.MIN)
        t = torch.cat([mx[:2], tot, bst])
    elapsed_max = float(t[0])
    ttt = -float(t[1])
    total_steps = float(t[2])
    n = world
    value = n * args.steps / elapsed_max * 3600.0
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "trials/hour",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic ImageNet-shape (224x224x3, 1000 classes), random-init weights",
            "config": {
                "model": "resnet50",
                "global_batch": args.batch * n,
                "per_trial_batch": args.batch,
                "seq_len": None,
                "image_size": args.image,
                "parallelism": f"trial-parallel x{n} (1 resident trial executor per GPU, independent brackets)",
                "search": f"hyperband max_iter={args.max_iter} eta={args.eta} resume=true",
                "unit_steps": args.unit_steps,
                "brackets_per_gpu": "repeat",
            },
            "wall_clock_to_target_s": round(ttt, 3) if math.isfinite(ttt) else None,
            "target_loss": args.target,
            "best_loss": round(float(t[3]), 4),
            "train_images_per_s": round(total_steps * args.batch / elapsed_max, 1),
            "graph_capture_s": round(capture_s, 2),
            "hip_graph": ex.graph is not None,
            "graph_check_error": ex.graph_check_error,
            "fused_bn": not args.unfused,
            "mfma_1x1_conv": not args.miopen_1x1,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
