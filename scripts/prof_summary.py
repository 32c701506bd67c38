#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace over the steady-state training window.

The window is the span of the last ``--steps`` optimizer launches (``sgd_flat_kernel`` / ``adamw_flat``
mark one training step each), so MIOpen's first-use Find / compile kernels and the warm-up are excluded.
Prints per-step time by kernel class and the top kernels, optionally as markdown for profiles/.
"""
import argparse
import collections
import csv
import sys

CLASSES = [
    ("conv GEMM (plx MFMA: 1x1, 3x3 implicit, wgrad slabs)", ("gemm_nt_kernel", "gemm_tn_kernel", "wgrad_kernel",
                                                           "slab_partial", "slab_final", "weight_prep",
                                                           "stem_pack", "stem_unpack")),
    ("fused BN+add+ReLU (plx)", ("bn_stats", "bn_apply", "bn_bwd", "bn_fwd", "bn_partial", "stem_apply_pool",
                                 "stem_pool_bn")),
    ("pool (plx)", ("maxpool_fwd", "maxpool_bwd", "gap_fwd", "gap_bwd")),
    ("loss (plx class cross entropy)", ("xent_fwd", "xent_bwd")),
    ("data (plx synthetic batch)", ("synth_images", "counter_add")),
    ("conv (MIOpen igemm/CK/naive)", ("igemm", "conv", "ck::tensor_operation", "naive_conv", "gtcx")),
    ("BN (MIOpen)", ("MIOpenBatchNorm",)),
    ("optimizer / trial kernels (plx)", ("sgd_flat", "adamw_flat", "adamw_mixed", "record_metric", "commit_metric",
                                         "init_flat", "zero_kernel")),
    ("LM GEMM (plx MFMA gemm256: 8-wave, 4-wave, stream-K, split-K reduce)", ("gemm256",)),
    ("attention (plx flash fwd / dq / dkdv)", ("attn_fwd", "attn_bwd")),
    ("LM fused elementwise (plx LayerNorm / RMSNorm, RoPE, SwiGLU, GELU + column sums)",
     ("ln_fwd", "ln_bwd", "rms_", "qkv_rope", "swiglu", "colsum", "partial_colsum")),
    ("GEMM (hipBLASLt/rocBLAS)", ("Cijk", "gemm", "Gemm")),
    ("pool", ("pool",)),
    ("elementwise/other torch", ("at::native",)),
]


def classify(name: str) -> str:
    for cls, keys in CLASSES:
        if any(k in name for k in keys):
            return cls
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--marker", default="sgd_flat_kernel")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--markdown", action="store_true")
    ap.add_argument("--context", type=int, default=1, help="list the kernels around the last step's largest gap")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < 2:
        sys.exit("not enough step markers")
    marks = marks[-(a.steps + 1):]
    lo, hi = marks[0] + 1, marks[-1] + 1
    n_steps = len(marks) - 1
    win = rows[lo:hi]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    busy = collections.Counter()
    calls = collections.Counter()
    per_class = collections.Counter()
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy[r["Kernel_Name"]] += d
        calls[r["Kernel_Name"]] += 1
        per_class[classify(r["Kernel_Name"])] += d
    total = sum(busy.values())
    wall = (t1 - t0) / n_steps / 1e6
    out = []
    out.append(f"steady-state window: {n_steps} steps, wall {wall:.3f} ms/step, kernel-busy {total / n_steps / 1e6:.3f} "
               f"ms/step, {len(win) / n_steps:.0f} launches/step")
    out.append("")
    out.append("| class | ms/step | share |")
    out.append("|---|---|---|")
    for cls, d in per_class.most_common():
        out.append(f"| {cls} | {d / n_steps / 1e6:.3f} | {100 * d / total:.1f}% |")
    # GPU idle time: the union of kernel intervals over all streams vs the window, and per stream the gaps between
    # consecutive kernels (launch / drain boundaries inside the replayed graph)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in win)
    union, cur_s, cur_e, prev = 0, iv[0][0], iv[0][1], iv[0][2]
    idle = []                                               # (gap ns, kernel before, kernel after)
    for s, e, name in iv[1:]:
        if s > cur_e:
            union += cur_e - cur_s
            idle.append((s - cur_e, prev, name))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            prev = name
    union += cur_e - cur_s
    idle.sort(reverse=True)
    big = [g for g in idle if g[0] > 20_000]
    skey = "Stream_Id" if "Stream_Id" in win[0] else ("Queue_Id" if "Queue_Id" in win[0] else None)
    out.append("")
    out.append(f"GPU busy (union over streams) {union / n_steps / 1e6:.3f} ms/step, idle "
               f"{(t1 - t0 - union) / n_steps / 1e6:.3f} ms/step ({len(idle)} gaps; {len(big)} over 20 us hold "
               f"{sum(g[0] for g in big) / n_steps / 1e6:.3f} ms/step)")
    for g, before, after in idle[:8]:
        out.append(f"- idle {g / 1e3:.1f} us after `{before[:60]}` before `{after[:60]}`")
    # kernel sequence around the largest idle gap inside one step (offsets from the step's first kernel)
    if a.context and big:
        step_rows = rows[marks[-2] + 1: marks[-1] + 1]
        t_s = int(step_rows[0]["Start_Timestamp"])
        ks = sorted(step_rows, key=lambda r: int(r["Start_Timestamp"]))
        worst, wi = 0, None
        for i in range(1, len(ks)):
            g = int(ks[i]["Start_Timestamp"]) - max(int(k["End_Timestamp"]) for k in ks[:i])
            if g > worst:
                worst, wi = g, i
        out.append("")
        run_end = 0
        for i, k in enumerate(ks):
            if i and int(k["Start_Timestamp"]) - run_end > 20_000:
                p_ = ks[i - 1]
                out.append(f"- step gap {(int(k['Start_Timestamp']) - run_end) / 1e3:.1f} us at +"
                           f"{(run_end - t_s) / 1e3:.1f}: `{p_['Kernel_Name'][:50]}` (stream {p_.get(skey, '?')}) -> "
                           f"`{k['Kernel_Name'][:50]}` (stream {k.get(skey, '?')})")
            run_end = max(run_end, int(k["End_Timestamp"]))
        ends = collections.defaultdict(int)
        for k in ks:
            ends[k.get(skey, "?")] = max(ends[k.get(skey, "?")], int(k["End_Timestamp"]) - t_s)
        out.append("last step: last kernel end per stream " + ", ".join(f"stream {sid}: +{e / 1e3:.1f} us"
                                                                 for sid, e in sorted(ends.items())))
        out.append("last step: final kernels:")
        for k in sorted(ks, key=lambda r: int(r["End_Timestamp"]))[-10:]:
            out.append(f"- +{(int(k['Start_Timestamp']) - t_s) / 1e3:9.1f} .. +{(int(k['End_Timestamp']) - t_s) / 1e3:9.1f} us"
                       f"  stream {k.get(skey, '?')}  `{k['Kernel_Name'][:70]}`")
        out.append(f"last step: largest idle {worst / 1e3:.1f} us before kernel #{wi}; neighbourhood:")
        for k in ks[max(0, (wi or 0) - 6): (wi or 0) + 4]:
            out.append(f"- +{(int(k['Start_Timestamp']) - t_s) / 1e3:9.1f} .. +{(int(k['End_Timestamp']) - t_s) / 1e3:9.1f} us"
                       f"  stream {k.get(skey, '?') if skey else '?'}  `{k['Kernel_Name'][:70]}`")
    if skey is not None:
        streams = collections.defaultdict(list)
        for r in win:
            streams[r[skey]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        out.append("")
        out.append(f"| {skey} | launches/step | busy ms/step | gaps ms/step | median gap us |")
        out.append("|---|---|---|---|---|")
        for sid, ks in sorted(streams.items(), key=lambda kv: -len(kv[1])):
            ks.sort()
            gaps = sorted(max(0, ks[i + 1][0] - ks[i][1]) for i in range(len(ks) - 1))
            med = gaps[len(gaps) // 2] / 1e3 if gaps else 0.0
            out.append(f"| {sid} | {len(ks) / n_steps:.0f} | {sum(e - s for s, e in ks) / n_steps / 1e6:.3f} | "
                       f"{sum(gaps) / n_steps / 1e6:.3f} | {med:.1f} |")
    out.append("")
    out.append("| kernel | calls/step | us/call | ms/step | share |")
    out.append("|---|---|---|---|---|")
    for name, d in busy.most_common(a.top):
        out.append(f"| `{name[:90]}` | {calls[name] / n_steps:.1f} | {d / calls[name] / 1e3:.1f} | "
                   f"{d / n_steps / 1e6:.3f} | {100 * d / total:.1f}% |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
