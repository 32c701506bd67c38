"""Sum rocprofv3 --pmc counter_collection CSV rows per (kernel, counter) and print one JSON line per kernel with the
derived ratios used in the round-3 GEMM analysis (MFMA busy share, wait / active shares, LDS conflict rate).

    python scripts/pmc_summary.py <counter_collection.csv> [--match substr]
"""
import csv
import json
import sys
from collections import defaultdict


def main() -> None:
    path = sys.argv[1]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name") or row.get("KernelName") or ""
            if match and match not in k:
                continue
            c = row.get("Counter_Name") or row.get("CounterName")
            v = float(row.get("Counter_Value") or row.get("CounterValue") or 0)
            acc[k][c] += v
            disp[k].add(row.get("Dispatch_Id") or row.get("DispatchId"))
    for k, cs in acc.items():
        out = {"kernel": k[:120], "dispatches": len(disp[k])}
        out.update({c: v for c, v in sorted(cs.items())})
        wc = cs.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in cs:
                    out[c + "_share"] = round(cs[c] / wc, 3)
        if cs.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
            # MFMA busy cycles are per SIMD-cycle; busy cycles per SE: normalise by 4 SIMDs x CUs later if needed
            out["mfma_busy_per_busy"] = round(cs["SQ_VALU_MFMA_BUSY_CYCLES"] / cs["SQ_BUSY_CYCLES"], 3)
        if cs.get("SQ_INSTS_LDS"):
            out["lds_conflict_per_inst"] = round(cs.get("SQ_LDS_BANK_CONFLICT", 0) / cs["SQ_INSTS_LDS"], 3)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
