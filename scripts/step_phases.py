#!/usr/bin/env python3
"""Forward / backward split of the ResNet training step from a rocprofv3 kernel trace (CSV).

For each of the last ``--steps`` steps (bracketed by the optimizer kernel): the forward is everything up to the end of
the loss kernel, the backward the rest.  Per phase: wall, busy time per stream and the union, and per class the kernel
time on each stream -- so a run with the weight gradients on the side stream can be compared with a serialised run
(``PLX_WGRAD_STREAM=0``) to price the overlap and the CU contention it causes.

    python scripts/step_phases.py run_kernel_trace.csv [--steps 20] [--markdown]
"""
import argparse
import collections
import csv
import sys


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def kind(name):
    n = name
    if "gemm_tn_kernel" in n or "wgrad_kernel" in n or "slab_" in n or "stem_unpack_wgrad" in n:
        return "wgrad"
    if "gemm_nt_kernel" in n:
        return "nt(fwd/dgrad)"
    if "bn_" in n or "stem_" in n:
        return "bn/stem"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--marker", default="sgd_flat_kernel")
    # the loss kernel ends the forward: torch's NLL, or the fused class cross entropy (ops/lm.py class_xent)
    ap.add_argument("--loss", default="nll_loss_forward,xent_fwd_kernel")
    ap.add_argument("--markdown", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < 2:
        sys.exit("not enough step markers")
    marks = marks[-(a.steps + 1):]
    agg = collections.defaultdict(float)
    n = 0
    for k in range(len(marks) - 1):
        step = rows[marks[k] + 1:marks[k + 1] + 1]
        li = [i for i, r in enumerate(step) if any(x in r["Kernel_Name"] for x in a.loss.split(","))]
        if not li:
            continue
        cut = int(step[li[0]]["End_Timestamp"])
        t0 = int(step[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in step)
        n += 1
        for phase, lo, hi in (("fwd", t0, cut), ("bwd", cut, t1)):
            agg[(phase, "wall")] += hi - lo
            ivs = collections.defaultdict(list)
            for r in step:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                s, e = max(s, lo), min(e, hi)
                if e <= s:
                    continue
                st = r.get("Stream_Id", "0")
                ivs[st].append((s, e))
                ivs["union"].append((s, e))
                agg[(phase, "kern", st, kind(r["Kernel_Name"]))] += e - s
            for st, iv in ivs.items():
                agg[(phase, "busy", st)] += union(iv)
    if not n:
        sys.exit("no step with a loss kernel")
    ms = lambda v: v / n / 1e6  # noqa: E731
    out = [f"steps averaged: {n}", ""]
    out.append("| phase | wall ms | union busy ms | " + " | ".join(f"stream {s} busy ms" for s in sorted(
        {k[2] for k in agg if k[1] == "busy" and k[2] != "union"})) + " |")
    streams = sorted({k[2] for k in agg if k[1] == "busy" and k[2] != "union"})
    out.append("|---" * (3 + len(streams)) + "|")
    for ph in ("fwd", "bwd"):
        out.append(f"| {ph} | {ms(agg[(ph, 'wall')]):.3f} | {ms(agg[(ph, 'busy', 'union')]):.3f} | " +
                   " | ".join(f"{ms(agg[(ph, 'busy', s)]):.3f}" for s in streams) + " |")
    out.append("")
    out.append("| phase | stream | kind | kernel ms |")
    out.append("|---|---|---|---|")
    for k in sorted(k for k in agg if k[1] == "kern"):
        out.append(f"| {k[0]} | {k[2]} | {k[3]} | {ms(agg[k]):.3f} |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
