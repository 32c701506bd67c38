"""Host cost of a kernel launch with and without a live RCCL communicator in the process.

    python scripts/launch_overhead.py [--n 20000]

Prints one JSON line: microseconds per tiny launch (torch add_ on a 1-element tensor, host-timed, GPU idle) before
and after creating a 1-rank RcclComm (csrc/rccl_comm.cpp).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_launch(x, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        x.add_(1.0)
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return dt / n * 1e6


ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=20000)
a = ap.parse_args()
x = torch.zeros(1, device="cuda")
per_launch(x, 1000)
before = [per_launch(x, a.n) for _ in range(3)]
from polyaxon_amd.parallel.rccl import RcclComm  # noqa: E402

comm = RcclComm(RcclComm.new_unique_id(), 1, 0, 0)
per_launch(x, 1000)
after = [per_launch(x, a.n) for _ in range(3)]
comm.close()
closed = [per_launch(x, a.n) for _ in range(3)]
print(json.dumps({"us_per_launch_before": [round(v, 2) for v in before],
                  "us_per_launch_with_rccl": [round(v, 2) for v in after],
                  "us_per_launch_after_close": [round(v, 2) for v in closed]}))
