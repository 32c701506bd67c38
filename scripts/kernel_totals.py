#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 SQLite output (``rocprofv3 --kernel-trace``): calls, total ms, mean us.

    python scripts/kernel_totals.py gpurun_out/<dir>/run_results.db [--top 20] [--grep attn]
"""
import argparse
import collections
import sqlite3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, start, end in c.execute("select name, start, end from kernels"):
        if a.grep and a.grep not in name:
            continue
        agg[name][0] += 1
        agg[name][1] += (end - start) / 1e6
    print("| kernel | calls | total ms | mean us |")
    print("|---|---|---|---|")
    for name, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{name[:90]}` | {n} | {ms:.3f} | {1e3 * ms / n:.1f} |")


if __name__ == "__main__":
    main()
