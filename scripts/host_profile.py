"""Host-side (Python) time of the resident executor's training step: cProfile over a few ResNet-50 steps on the GPU,
after warm-up, with the step's wall time and the host time per step (the step returns once every kernel is queued;
a host time close to the GPU time means the GPU can starve at the forward -> backward hand-off).

    python scripts/host_profile.py [--steps 20] [--top 40] [--sort tottime]
"""
import argparse
import cProfile
import io
import json
import pstats
import time

import torch

from polyaxon_amd.polyflow.programs import build_program


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--sort", default="tottime")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    prog = build_program("resnet50", {"batch": 256}, dev)
    prog.warm()
    ex = prog.executor
    ex.reset(seed=1)
    ex.set_hparams(lr=0.1, momentum=0.9, weight_decay=1e-4)
    ex.run(5)
    torch.cuda.synchronize()
    # host time per step: time to queue the steps (the GPU runs behind) vs the wall time to finish them
    t0 = time.perf_counter()
    ex.run(a.steps)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    # backward on this thread (not the autograd engine's device thread), so cProfile sees its Python too
    torch.autograd.set_multithreading_enabled(False)
    pr = cProfile.Profile()
    pr.enable()
    ex.run(a.steps)
    pr.disable()
    torch.autograd.set_multithreading_enabled(True)
    torch.cuda.synchronize()
    print(json.dumps({"steps": a.steps, "host_ms_per_step": round(t_host / a.steps * 1e3, 2),
                      "wall_ms_per_step": round(t_wall / a.steps * 1e3, 2)}), flush=True)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(a.sort).print_stats(a.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
