#!/usr/bin/env python3
"""Per-step kernel summary of a rocprofv3 SQLite output (``rocprofv3 --kernel-trace`` default format).

The steady-state window is bracketed by launches of the optimizer kernel (``--marker``, default adamw): the
last ``--steps`` intervals between consecutive markers.  Prints wall and busy ms per step and the top kernels.
"""
import argparse
import collections
import sqlite3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adamw")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--md", action="store_true", help="markdown table")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, (n, _, _) in enumerate(rows) if a.marker in n.lower()]
    marks = sorted(set(idx))
    # the optimizer may be several launches per step (lp mode: mixed + tail); keep the first of each burst
    firsts = [i for k, i in enumerate(marks) if k == 0 or i - marks[k - 1] > 4]
    steps = min(a.steps, len(firsts) - 1)
    lo, hi = firsts[-steps - 1], firsts[-1]
    win = rows[lo:hi]
    wall = (win[-1][2] - win[0][1]) / 1e6 / steps
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in win:
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e6
    busy = sum(v[1] for v in agg.values()) / steps
    print(f"steady-state window: {steps} steps, wall {wall:.2f} ms/step, kernel-busy {busy:.2f} ms/step, "
          f"{len(win) / steps:.0f} launches/step\n")
    if a.md:
        print("| ms/step | calls/step | kernel |\n|---|---|---|")
    for n, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1])[: a.top]:
        name = n[:140].replace("|", "/")
        if a.md:
            print(f"| {t / steps:.2f} | {k / steps:.0f} | `{name}` |")
        else:
            print(f"{t / steps:8.2f} ms {k / steps:6.0f}x  {name}")


if __name__ == "__main__":
    main()
