#!/usr/bin/env python3
"""Per-step stream overlap of an LM training trace (rocprofv3 SQLite): for the last ``--steps`` steps (delimited by
the loss kernel ``--marker``), wall time, union busy time, and per stream its busy time and its top kernels -- to
see whether the optimizer launches on their own stream overlap the backward.

    python scripts/lm_step_streams.py run_results.db [--marker cunn_SoftMaxForward] [--steps 3]
"""
import argparse
import collections
import sqlite3


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="cunn_SoftMaxForward")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    marks = marks[-(a.steps + 1):]
    for k in range(len(marks) - 1):
        step = rows[marks[k]:marks[k + 1]]
        t0, t1 = step[0][1], max(r[2] for r in step)
        per = collections.defaultdict(list)
        names = collections.defaultdict(collections.Counter)
        for n, s, e, st in step:
            per[st].append((s, e))
            names[st][n[:60]] += e - s
        print(f"step {k}: wall {(t1 - t0) / 1e6:.2f} ms, union busy {union([x for v in per.values() for x in v]) / 1e6:.2f} ms")
        for st, iv in sorted(per.items()):
            top = ", ".join(f"{n} {d / 1e6:.1f}" for n, d in names[st].most_common(3))
            print(f"  stream {st}: {len(iv)} kernels, busy {union(iv) / 1e6:.2f} ms, sum {sum(e - s for s, e in iv) / 1e6:.2f} ms; {top}")


if __name__ == "__main__":
    main()
