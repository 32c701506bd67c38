"""Host (Python) cost of one eager ResNet-50 training step vs its GPU time, on the resident executor the bench uses.

Enqueues 20 steps without synchronising and reports the host time per step (when the loop returns) against the
GPU time per step (after the final synchronize); then cProfiles 5 enqueued steps and prints the top functions by
own time, so per-op Python overhead can be attacked where it is."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    from polyaxon_amd.polyflow.programs import build_program

    dev = torch.device("cuda", 0)
    prog = build_program("resnet50", {"batch": 256, "image": 224, "unit_steps": 4, "signal": 0.5, "data_seed": 1234},
                         dev)
    prog.warm()
    ex = prog.executor
    ex.reset(seed=1)
    ex.set_hparams(lr=0.1, momentum=0.9, weight_decay=1e-4)
    ex.run(3)
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    ex.run(n)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"host_ms_per_step": round((t1 - t0) / n * 1e3, 3), "gpu_ms_per_step": round((t2 - t0) / n * 1e3, 3)}))
    pr = cProfile.Profile()
    pr.enable()
    ex.run(5)
    pr.disable()
    torch.cuda.synchronize()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(30)
    print(buf.getvalue())


if __name__ == "__main__":
    main()
