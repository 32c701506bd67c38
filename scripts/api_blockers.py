"""Which HIP API calls hold the host back: a rocprofv3 run with --hip-trace --kernel-trace, summarised.

    python scripts/api_blockers.py run_hip_api_trace.csv run_kernel_trace.csv [--skip-first 0.3] [--top 20]

Prints (JSON lines):
- per API function: calls, total / max host ms (a synchronising call -- hipMalloc, hipFree, hipStreamSynchronize,
  hipEventSynchronize, a pageable hipMemcpy -- shows up as a few long calls);
- the host lead over the GPU: for every kernel, start - end of its launch call (``lead_us``), as percentiles over the
  steady-state window -- ~5 us means the GPU waited for the host, milliseconds mean the host ran ahead;
- the API calls longer than 100 us, with what the GPU was doing (the lead just before them), so a call that drains
  the host's lead can be named.
"""
import argparse
import csv
import json
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("api")
    ap.add_argument("kernels")
    ap.add_argument("--skip-first", type=float, default=0.3)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    with open(a.kernels) as f:
        kr = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Correlation_Id"], r["Kernel_Name"])
              for r in csv.DictReader(f)]
    kr.sort()
    t_lo = kr[int(len(kr) * a.skip_first)][0]
    t_hi = kr[-1][1]
    calls = []
    launch_end = {}
    with open(a.api) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            fn = r["Function"]
            if "Launch" in fn:
                launch_end[r["Correlation_Id"]] = e
            if t_lo <= s <= t_hi:
                calls.append((s, e, fn))
    by = defaultdict(lambda: [0, 0, 0])
    for s, e, fn in calls:
        d = e - s
        b = by[fn]
        b[0] += 1
        b[1] += d
        b[2] = max(b[2], d)
    span = (t_hi - t_lo) / 1e6
    print(json.dumps({"window_ms": round(span, 2), "kernels": sum(1 for k in kr if k[0] >= t_lo),
                      "api_calls": len(calls)}))
    for fn, (n, tot, mx) in sorted(by.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(json.dumps({"api": fn, "calls": n, "total_ms": round(tot / 1e6, 3), "max_us": round(mx / 1e3, 1)}))
    leads = []
    lead_at = []
    for s, e, cid, name in kr:
        if s < t_lo or cid not in launch_end:
            continue
        le = launch_end[cid]
        leads.append((s - le) / 1e3)
        lead_at.append((le, (s - le) / 1e3, name))
    leads_sorted = sorted(leads)
    if leads_sorted:
        q = lambda p: round(leads_sorted[min(len(leads_sorted) - 1, int(p * len(leads_sorted)))], 1)  # noqa: E731
        print(json.dumps({"lead_us": {"p05": q(0.05), "p25": q(0.25), "p50": q(0.5), "p75": q(0.75), "p95": q(0.95)},
                          "under_20us_share": round(sum(1 for v in leads if v < 20) / len(leads), 3)}))
    lead_at.sort()
    import bisect
    keys = [t for t, _, _ in lead_at]
    long_calls = [(s, e, fn) for s, e, fn in calls if e - s > 100_000]
    for s, e, fn in long_calls[: a.top]:
        i = bisect.bisect_left(keys, s) - 1
        prev = lead_at[i] if i >= 0 else (0, float("nan"), "")
        print(json.dumps({"long_call": fn, "us": round((e - s) / 1e3, 1), "at_ms": round((s - t_lo) / 1e6, 3),
                          "lead_before_us": round(prev[1], 1), "kernel_before": prev[2][:70]}))


if __name__ == "__main__":
    main()
