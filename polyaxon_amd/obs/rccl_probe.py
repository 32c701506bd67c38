"""Child-process RCCL smoke test for ``/_status`` ("store, GPUs, RCCL smoke test").

The reference's status check round-trips a health task through every worker queue
(/root/reference/polyaxon/checks/worker.py:16-45).  The device-side equivalent here is one real RCCL round trip: a
world-1 framework communicator (csrc/rccl_comm.cpp, the one every DP trial uses) created on one GPU, a few small
all-reduces on a HIP stream, the result checked and the latency reported.  It runs in a short-lived child process
so the API / scheduler process never imports torch or maps the HIP runtime (the GPU-free control plane,
tests/test_gpu_free_scheduler.py):

    python -m polyaxon_amd.obs.rccl_probe          -> one JSON line {"status": "ok" | "error" | "skipped", ...}
"""
from __future__ import annotations

import json
import sys
import time


def probe(iters: int = 10) -> dict:
    import torch

    if not torch.cuda.is_available():
        return {"status": "skipped", "message": "no HIP device visible"}
    from polyaxon_amd.parallel.rccl import RcclComm

    dev = torch.cuda.current_device()
    t0 = time.perf_counter()
    comm = RcclComm(RcclComm.new_unique_id(), 1, 0, dev, timeout_s=30, init_timeout_s=30)
    init_ms = (time.perf_counter() - t0) * 1e3
    try:
        x = torch.full((1024,), 3.0, device=f"cuda:{dev}")
        comm.all_reduce(x)  # warm-up (first launch loads RCCL's kernels)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(iters):
            comm.all_reduce(x, op="sum")
        torch.cuda.synchronize()
        lat_us = (time.perf_counter() - t1) / iters * 1e6
        comm.check()
        ok = bool(torch.all(x == 3.0))
        return {"status": "ok" if ok else "error", "message": "" if ok else "all-reduce returned wrong values",
                "device": dev, "init_ms": round(init_ms, 2), "all_reduce_us": round(lat_us, 2),
                "backend": "RCCL (framework communicator)"}
    finally:
        comm.close()


def main() -> int:
    try:
        res = probe()
    except Exception as e:  # report, never hang or crash the caller
        res = {"status": "error", "message": f"{type(e).__name__}: {e}"}
    print(json.dumps(res), flush=True)
    return 0 if res["status"] in ("ok", "skipped") else 1


if __name__ == "__main__":
    sys.exit(main())
