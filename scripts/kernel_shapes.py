"""Per-launch-shape kernel time from a rocprofv3 kernel trace: groups dispatches by (kernel, grid, workgroup) so one
kernel's calls on different problem shapes separate (the LM GEMMs: grid = tiles x K splits).

    python scripts/kernel_shapes.py run_kernel_trace.csv [--match gemm256] [--top 40] [--skip-first 0.2]

``--skip-first``: fraction of the trace (by dispatch order) dropped as warm-up.  One JSON line per group, sorted by
total time: calls, mean / min / total microseconds.
"""
import argparse
import csv
import json
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--skip-first", type=float, default=0.2)
    a = ap.parse_args()
    with open(a.trace) as f:
        rows = list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * a.skip_first):]
    groups = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if a.match and a.match not in name:
            continue
        grid = tuple(int(r.get(f"Grid_Size_{d}", 0) or 0) for d in "XYZ")
        wg = int(r.get("Workgroup_Size_X", 0) or 0)
        groups[(name[:90], grid, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = sorted(groups.items(), key=lambda kv: -sum(kv[1]))[: a.top]
    for (name, grid, wg), ds in out:
        print(json.dumps({"kernel": name, "grid": grid, "wg": wg, "calls": len(ds), "mean_us": round(sum(ds) / len(ds), 1),
                          "min_us": round(min(ds), 1), "total_us": round(sum(ds), 1)}))


if __name__ == "__main__":
    main()
