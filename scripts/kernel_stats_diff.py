"""Per-kernel difference of two rocprofv3 ``*_kernel_stats.csv`` files of the same workload (e.g. the ResNet-50 bench
with and without a live RCCL communicator): calls, mean duration and total per step for the kernels whose total
changed most.

    python scripts/kernel_stats_diff.py base.csv other.csv [--steps-base N] [--steps-other N] [--top 25]
"""
import argparse
import csv


def load(path):
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Name"]
        e = out.setdefault(name, [0, 0.0])
        e[0] += int(r["Calls"])
        e[1] += float(r["TotalDurationNs"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("base")
    ap.add_argument("other")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    a, b = load(args.base), load(args.other)
    # per training step: normalised by the launches of the optimizer kernel (one per step), else of the most
    # frequent kernel common to both
    common = [k for k in a if k in b]
    opt = [k for k in common if "sgd_flat_kernel" in k or "adamw" in k.lower()]
    ref = opt[0] if opt else (max(common, key=lambda k: a[k][0]) if common else None)
    sa = a[ref][0] if ref else 1
    sb = b[ref][0] if ref else 1
    rows = []
    for k in set(a) | set(b):
        ca, ta = a.get(k, (0, 0.0))
        cb, tb = b.get(k, (0, 0.0))
        rows.append((tb / sb - ta / sa, k, ca / sa, cb / sb, ta / max(ca, 1) / 1e3, tb / max(cb, 1) / 1e3,
                     ta / sa / 1e3, tb / sb / 1e3))
    rows.sort(key=lambda r: -abs(r[0]))
    tot_a = sum(t for _, t in a.values()) / sa / 1e3
    tot_b = sum(t for _, t in b.values()) / sb / 1e3
    print(f"normalised per launch of `{ref[:60] if ref else '-'}`: base {sa} / other {sb} launches")
    print(f"kernel time per step: base {tot_a:.1f} us, other {tot_b:.1f} us ({tot_b - tot_a:+.1f})\n")
    print("| kernel | calls base | calls other | mean us base | mean us other | us/step base | us/step other | delta |")
    print("|---|---|---|---|---|---|---|---|")
    for d, k, ca, cb, ma, mb, ua, ub in rows[:args.top]:
        print(f"| `{k[:70]}` | {ca:.2f} | {cb:.2f} | {ma:.1f} | {mb:.1f} | {ua:.1f} | {ub:.1f} | {d:+.1f} |")


if __name__ == "__main__":
    main()
