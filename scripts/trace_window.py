"""Print the kernel sequence of a rocprofv3 kernel trace around the k-th occurrence of a kernel, with the idle gap
before each launch (per stream) -- e.g. the forward -> backward hand-off of the training step.

    python scripts/trace_window.py run_kernel_trace.csv --match nll_loss --occurrence -3 --before 15 --after 25
        [--api run_hip_api_trace.csv]

``--api``: the HIP API trace of the same run (rocprofv3 --hip-trace); each kernel then also shows how long after the
host's launch call returned it started (``lag``: ~0 when the host was the bottleneck, large when the GPU was).
"""
import argparse
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", required=True)
    ap.add_argument("--occurrence", type=int, default=-2, help="which match (python index; -2 = second to last)")
    ap.add_argument("--before", type=int, default=15)
    ap.add_argument("--after", type=int, default=25)
    ap.add_argument("--api", default="")
    a = ap.parse_args()
    launch_end = {}
    if a.api:
        with open(a.api) as f:
            for r in csv.DictReader(f):
                if "Launch" in r.get("Function", ""):
                    launch_end[r["Correlation_Id"]] = int(r["End_Timestamp"])
    with open(a.trace) as f:
        rows = list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    hits = [i for i, r in enumerate(rows) if a.match in r["Kernel_Name"]]
    if not hits:
        raise SystemExit(f"no kernel matching {a.match!r}")
    c = hits[a.occurrence]
    lo, hi = max(0, c - a.before), min(len(rows), c + a.after)
    t0 = int(rows[lo]["Start_Timestamp"])
    last_end = {}
    for r in rows[:lo]:
        last_end[r.get("Stream_Id", "0")] = int(r["End_Timestamp"])
    for r in rows[lo:hi]:
        s, e, sid = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", "0")
        gap = (s - last_end[sid]) / 1e3 if sid in last_end else 0.0
        last_end[sid] = e
        le = launch_end.get(r.get("Correlation_Id", ""))
        lag = f"  lag {(s - le) / 1e3:8.1f}" if le is not None else ""
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}{lag}  s{sid}  {r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
