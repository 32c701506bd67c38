"""Learning curves of the resident GPT-2 trial program on a synthetic token task (the config-4 objective), per
learning rate: does a trial budget separate the learning rates?  One JSON line per (lr, step) with the mean loss of
the last 4 steps, through the same executor the BO trials run on.

    python scripts/copy_task_probe.py [--lrs 1e-4,3e-4,1e-3,3e-3] [--steps 400] [--every 25] [--active-vocab 4096]
                                      [--period 64] [--wd 0.1] [--beta2 0.95] [--task copy|chain] [--chain-p 4093]
"""
import argparse
import json
import time

import torch

from polyaxon_amd.polyflow.programs import build_program


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lrs", default="1e-4,3e-4,1e-3,3e-3")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--every", type=int, default=25)
    ap.add_argument("--active-vocab", type=int, default=4096)
    ap.add_argument("--period", type=int, default=64)
    ap.add_argument("--wd", type=float, default=0.1)
    ap.add_argument("--beta2", type=float, default=0.95)
    ap.add_argument("--task", default="copy", choices=("copy", "chain"))
    ap.add_argument("--chain-p", type=int, default=4093)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    prog = build_program("gpt2", {"batch": 16, "seq": 1024, "unit_steps": 4, "data_seed": 1234,
                                  "active_vocab": args.active_vocab, "period": args.period, "task": args.task,
                                  "chain_p": args.chain_p}, dev)
    prog.warm()
    ex = prog.executor
    out = torch.full((1, 1), float("nan"), device=dev)
    for lr in (float(v) for v in args.lrs.split(",")):
        ex.reset(seed=7)
        ex.set_hparams(lr=lr, beta1=0.9, beta2=args.beta2, eps=1e-8, weight_decay=args.wd)
        t0 = time.perf_counter()
        for s in range(args.every, args.steps + 1, args.every):
            ex.run(args.every)
            ex.commit(out[0], 0, window=4)
            torch.cuda.synchronize()
            print(json.dumps({"lr": lr, "step": s, "loss": round(float(out[0, 0]), 4),
                              "s": round(time.perf_counter() - t0, 2)}), flush=True)
    print(json.dumps({"info": prog.info}), flush=True)


if __name__ == "__main__":
    main()
