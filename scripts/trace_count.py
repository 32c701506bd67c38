"""Count the kernels of a rocprofv3 kernel trace whose name contains a substring.

    python scripts/trace_count.py run_kernel_trace.csv Cijk
"""
import csv
import json
import sys


def main() -> None:
    path, sub = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    hits = [r["Kernel_Name"] for r in rows if sub in r["Kernel_Name"]]
    print(json.dumps({"kernels": len(rows), "match": sub, "count": len(hits), "names": sorted(set(hits))[:20]}))


if __name__ == "__main__":
    main()
