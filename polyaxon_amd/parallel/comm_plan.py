"""Gradient-bucket sizing for the data-parallel collectives over MI355X xGMI.

The reference ships no collective code (its PyTorch jobs call NCCL themselves); the bucket size of
:class:`~polyaxon_amd.parallel.ddp.FlatDDP` is the one knob that decides how well the RCCL all-reduce (or ZeRO-1
reduce-scatter + all-gather) of a DP trial uses the links.  This module picks it from a cost model of the hardware
instead of a constant tuned for a switched fabric:

* **Topology.**  An 8-GPU MI355X node is a fully connected xGMI mesh: every GPU has 7 point-to-point links, one to
  each peer (~153 GB/s each).  A ring collective over W <= 8 ranks can run W - 1 edge-disjoint rings (the complete
  directed graph on W vertices decomposes into W - 1 directed Hamiltonian cycles for every W but 4 and 6, Tillson's
  theorem; there the model is an upper bound), so the bus bandwidth grows with W - 1 links instead of being capped by
  one switch port:
  ``busbw(W) ~= (W - 1) * link_GBps * efficiency``.
* **Per-call cost.**  ``t(B) = 2 (W - 1) * alpha + (2 (W - 1) / W) * B / busbw``: 2 (W - 1) ring steps of fixed
  latency ``alpha`` (kernel launch, proxy hand-off, flag round trip) plus the bytes each rank moves.
* **Bucket size.**  A bucket is worth sending once its bandwidth term dominates: efficiency
  ``e = t_bw / (t_bw + t_lat) >= target`` gives ``B >= target / (1 - target) * alpha * W * busbw``.  Because the
  link bandwidth grows with W, so does the bucket (a 2-rank gang wants ~10 MB, 8 ranks ~300 MB).  The size is
  clamped so the backward still overlaps at least ``min_buckets`` collectives (the last bucket, the first layers'
  gradients, is the exposed one) and to at least ``min_mb``.
* **Measured at start-up.**  With ``bucket_mb="auto"`` at world > 1, :class:`~polyaxon_amd.parallel.ddp.FlatDDP`
  first times a few all-reduces on the trial's own communicator (:func:`calibrate`: 1-64 MB on the GPU, ~0.1 s),
  averages the times over the ranks (so every rank fits the same numbers and cuts the same buckets) and plans with
  that fit (``source: "measured"``).
* **Measured table.**  ``python -m torch.distributed.run --nproc-per-node W -m polyaxon_amd.parallel.rccl``
  prints the node's all-reduce algbw per message size; :func:`fit_table` turns those rows into (alpha, busbw) by a
  least-squares fit of ``t(B) = a + b B``, and ``PLX_COMM_TABLE=<that JSON>`` makes :func:`plan` use the fit for
  its world size instead of the analytic link model.

``FlatDDP(bucket_mb="auto")`` (the LM trainer's default, ``--bucket_mb auto``) sizes its buckets with :func:`plan`.
"""
from __future__ import annotations

import argparse
import json
import math
import os
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional, Sequence

MB = 2 ** 20


@dataclass
class LinkModel:
    """xGMI cost model of one node.  ``link_GBps`` per link and direction, ``efficiency`` the share of it a ring
    step sustains, ``alpha_us`` the fixed cost of one ring step, ``links`` per GPU (peers of a full mesh)."""

    link_GBps: float = 153.0
    efficiency: float = 0.75
    alpha_us: float = 6.0
    links: int = 7

    def busbw_GBps(self, world: int) -> float:
        if world <= 1:
            return float("inf")
        return min(world - 1, self.links) * self.link_GBps * self.efficiency

    def alpha_s(self, world: int) -> float:
        return self.alpha_us * 1e-6


@dataclass
class FittedModel:
    """(alpha, busbw) of one world size from measured all-reduce rows."""

    world: int
    alpha_s_: float
    busbw: float
    measured: bool = False  # timed at start-up on the trial's communicator (calibrate), not read from a table

    def busbw_GBps(self, world: int) -> float:
        return self.busbw

    def alpha_s(self, world: int) -> float:
        return self.alpha_s_


def allreduce_seconds(nbytes: float, world: int, model=None) -> float:
    """Modelled time of one ring all-reduce of ``nbytes`` over ``world`` ranks."""
    if world <= 1:
        return 0.0
    m = model or LinkModel()
    steps = 2 * (world - 1)
    return steps * m.alpha_s(world) + (steps / world) * nbytes / (m.busbw_GBps(world) * 1e9)


def fit_table(rows: Sequence[Dict], world: int) -> FittedModel:
    """Least-squares ``t(B) = a + b B`` over rows ``{"bytes", "algbw_GBps"}`` (``t = bytes / algbw``, the
    parallel.rccl probe's output) -> alpha = a / (2 (W - 1)), busbw = (2 (W - 1) / W) / b."""
    pts = [(float(r["bytes"]), float(r["bytes"]) / (float(r["algbw_GBps"]) * 1e9)) for r in rows
           if float(r.get("algbw_GBps", 0)) > 0]
    if len(pts) < 2 or world <= 1:
        raise ValueError("need >= 2 rows with positive algbw and world > 1")
    n = len(pts)
    mx = sum(b for b, _ in pts) / n
    my = sum(t for _, t in pts) / n
    sxx = sum((b - mx) ** 2 for b, _ in pts)
    if sxx <= 0:
        raise ValueError("rows need distinct message sizes")
    slope = sum((b - mx) * (t - my) for b, t in pts) / sxx
    icept = max(0.0, my - slope * mx)
    if slope <= 0:
        raise ValueError("time does not grow with the message size: not an all-reduce table")
    steps = 2 * (world - 1)
    return FittedModel(world=world, alpha_s_=icept / steps, busbw=(steps / world) / slope / 1e9)


def load_table(path: str, world: int) -> Optional[FittedModel]:
    """The fit for ``world`` from a probe JSON (one object or JSON lines, each ``{"world", "all_reduce": [...]}``)."""
    with open(path) as f:
        text = f.read().strip()
    docs = [json.loads(line) for line in text.splitlines() if line.strip()] if not text.startswith("[") else json.loads(text)
    for d in docs:
        if int(d.get("world", 0)) == world:
            return fit_table(d["all_reduce"], world)
    return None


def calibrate(comm, world: int, device, sizes: Optional[Sequence[int]] = None, reps: int = 5,
              retry: bool = True) -> Optional[FittedModel]:
    """Fit (alpha, busbw) from all-reduces of ``sizes`` bytes timed on ``comm`` (a parallel/comm.py communicator:
    RCCL on the GPU, the gloo shim on the CPU).  Collective: every rank of the group calls it with the same
    arguments.  Each size runs once untimed, then ``reps`` timed single calls (median); the per-rank times are averaged over the ranks
    with one more all-reduce, so the fit -- and every plan made from it -- is the same on every rank.  None when the
    rows do not fit a line (e.g. a noisy CPU run); the caller keeps the link model then."""
    import time

    import torch

    if world <= 1:
        return None
    cuda = getattr(device, "type", str(device)) == "cuda"
    if sizes is None:
        sizes = [1 * MB, 4 * MB, 16 * MB, 64 * MB] if cuda else [256 * 1024, 1 * MB, 4 * MB]
    buf = torch.zeros(max(sizes) // 4, dtype=torch.float32, device=device)
    times = []
    for nbytes in sizes:
        view = buf[: nbytes // 4]
        comm.all_reduce(view, op="sum")  # warm: algorithm / channel set-up for this size
        if cuda:
            torch.cuda.synchronize(device)
        samples = []
        for _ in range(reps):  # the median of single calls: robust to a descheduled rank on a busy host
            t0 = time.perf_counter()
            comm.all_reduce(view, op="sum")
            if cuda:
                torch.cuda.synchronize(device)
            samples.append(time.perf_counter() - t0)
        times.append(sorted(samples)[len(samples) // 2])
    t = torch.tensor(times, dtype=torch.float64 if not cuda else torch.float32, device=device)
    comm.all_reduce(t, op="sum")
    if cuda:
        torch.cuda.synchronize(device)
    mean = [float(v) / world for v in t.cpu().tolist()]
    rows = [{"bytes": b, "algbw_GBps": b / max(tt, 1e-9) / 1e9} for b, tt in zip(sizes, mean)]
    try:
        fit = fit_table(rows, world)
    except ValueError:  # noise swamped the size dependence: once more with 4x larger messages
        if retry:
            return calibrate(comm, world, device, [4 * b for b in sizes], reps, retry=False)
        return None
    fit.measured = True
    return fit


def plan(grad_bytes: float, world: int, target: float = 0.9, min_buckets: int = 4, min_mb: float = 4.0,
         model=None) -> Dict:
    """Bucket size (bytes) for ``grad_bytes`` of gradients all-reduced over ``world`` ranks, with the numbers that
    chose it.  ``PLX_COMM_TABLE`` (a parallel.rccl probe JSON) overrides the analytic link model for its world."""
    if model is None:
        table = os.environ.get("PLX_COMM_TABLE", "")
        if table and os.path.exists(table) and world > 1:
            model = load_table(table, world)
    source = ("measured" if getattr(model, "measured", False) else "table") if isinstance(model, FittedModel) \
        else "link-model"
    m = model or LinkModel()
    if world <= 1:
        b = max(min_mb * MB, grad_bytes / max(1, min_buckets))
        return {"bucket_bytes": int(b), "world": world, "source": "world-1", "reason": "no collectives"}
    alpha, bw = m.alpha_s(world), m.busbw_GBps(world) * 1e9
    want = target / (1.0 - target) * alpha * world * bw  # efficiency >= target
    cap = grad_bytes / max(1, min_buckets)  # >= min_buckets overlapped collectives
    b = max(min_mb * MB, min(want, cap))
    t = allreduce_seconds(b, world, m)
    eff = (2 * (world - 1) / world) * b / bw / t if t > 0 else 1.0
    n = max(1, math.ceil(grad_bytes / b))
    return {"bucket_bytes": int(b), "world": world, "source": source, "target_efficiency": target,
            "efficiency": round(eff, 3), "buckets": n, "alpha_us": round(alpha * 1e6, 2),
            "busbw_GBps": round(bw / 1e9, 1), "per_bucket_ms": round(t * 1e3, 3),
            "total_ms": round(n * t * 1e3, 2),
            "reason": (f"floor of {min_mb:g} MB" if b > min(want, cap) else "efficiency target" if want <= cap
                       else f"capped for >= {min_buckets} overlapped buckets")}


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="polyaxon_amd.parallel.comm_plan",
                                 description="gradient-bucket plan for DP over MI355X xGMI")
    ap.add_argument("--params", type=float, required=True, help="parameter count (e.g. 8.03e9)")
    ap.add_argument("--bytes_per_grad", type=int, default=2, help="2 for bf16 gradients, 4 for fp32")
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--table", default="", help="parallel.rccl probe JSON (overrides the link model)")
    ap.add_argument("--target", type=float, default=0.9)
    args = ap.parse_args(argv)
    for w in args.world:
        model = load_table(args.table, w) if args.table else None
        p = plan(args.params * args.bytes_per_grad, w, target=args.target, model=model)
        p["bucket_MB"] = round(p["bucket_bytes"] / MB, 1)
        p["link_model"] = asdict(LinkModel()) if model is None else asdict(model)
        print(json.dumps(p))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
