"""Where the GPU idles: every interval in a rocprofv3 kernel trace during which no kernel runs on ANY stream, longer
than a threshold, grouped by the (kernel before, kernel after) pair, sorted by total idle time.

    python scripts/gap_report.py run_kernel_trace.csv [--min-us 10] [--skip-first 0.2] [--top 25]
"""
import argparse
import csv
import json
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:70]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-us", type=float, default=10.0)
    ap.add_argument("--skip-first", type=float, default=0.2)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    with open(a.trace) as f:
        rows = list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * a.skip_first):]
    groups = defaultdict(lambda: [0, 0.0])
    total = 0.0
    busy_until, prev = None, None
    t_first, t_last = int(rows[0]["Start_Timestamp"]), 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if busy_until is not None and s > busy_until:
            gap = (s - busy_until) / 1e3
            if gap >= a.min_us:
                g = groups[(short(prev), short(r["Kernel_Name"]))]
                g[0] += 1
                g[1] += gap
                total += gap
        if busy_until is None or e > busy_until:
            busy_until, prev = e, r["Kernel_Name"]
        t_last = max(t_last, e)
    span = (t_last - t_first) / 1e3
    print(json.dumps({"span_ms": round(span / 1e3, 2), "idle_ms_over_threshold": round(total / 1e3, 2),
                      "idle_share": round(total / span, 4)}))
    for (p, n), (cnt, us) in sorted(groups.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(json.dumps({"before": p, "after": n, "count": cnt, "total_ms": round(us / 1e3, 2),
                          "mean_us": round(us / cnt, 1)}))


if __name__ == "__main__":
    main()
