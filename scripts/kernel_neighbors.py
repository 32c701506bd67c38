#!/usr/bin/env python3
"""Print the kernels launched around each of the first ``--n`` launches matching a pattern in a rocprofv3 SQLite trace
(to find which op issues an unexpected kernel).

    python scripts/kernel_neighbors.py run_results.db FillFunctor [--n 2] [--ctx 4]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("pattern")
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--ctx", type=int, default=4)
    ap.add_argument("--skip", type=int, default=0, help="skip this many matches first (warm-up steps)")
    ap.add_argument("--tail", action="store_true", help="the last --n matches (steady state) instead")
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name, start, end, stream_id from kernels order by start").fetchall()
    hits = [i for i, r in enumerate(rows) if a.pattern in r[0]]
    hits = hits[-a.n:] if a.tail else hits[a.skip:a.skip + a.n]
    for i in hits:
        print(f"--- match at #{i}")
        for j in range(max(0, i - a.ctx), min(len(rows), i + a.ctx + 1)):
            n, s, e, st = rows[j]
            print(f"{'>>' if j == i else '  '} s{st} {(e - s) / 1e3:8.1f} us  {n[:110]}")


if __name__ == "__main__":
    main()
