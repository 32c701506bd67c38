"""Time the 256x256 MFMA GEMM (csrc/gemm256.hip) against torch (hipBLASLt) on the LM linears' shapes.

    python scripts/gemm_bench.py [--models gpt2,llama] [--reps 20] [--waves 8,4]

One JSON line per (model, linear, pass): ms and TFLOP/s of both, and the max |diff| relative to the output scale.
``--waves 8,4`` times both kernel schedules (ops/gemm.py FORCE_SCHEDULE) in the same process, interleaved per shape;
``--waves table`` times the per-shape table (ops/gemm.py SCHEDULE).
Passes: fwd (x . W^T), dgrad (dy . W), wgrad (dy^T . x, K = tokens).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from polyaxon_amd.ops import gemm  # noqa: E402

# (model, tokens, [(linear, in, out)])
MODELS = {
    "gpt2": (16 * 1024, [("qkv", 768, 2304), ("proj", 768, 768), ("up", 768, 3072), ("down", 3072, 768),
                        ("head", 768, 50432)]),
    "llama": (4096, [("qkv", 4096, 6144), ("proj", 4096, 4096), ("up", 4096, 28672), ("down", 14336, 4096)]),
}


def timed(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="gpt2,llama")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--waves", default="8")
    ap.add_argument("--groups", default="", help="tile-group sizes to A/B (plx_gemm256_set_group), e.g. 1,4,8")
    ap.add_argument("--cold", type=int, default=0,
                    help="rotate each call through this many operand copies (>= 1 GB in total defeats the 256 MB "
                         "infinity cache: the operands stream from HBM as in a training step)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    tot = {"torch": 0.0}
    waves = [0 if w == "table" else int(w) for w in args.waves.split(",")]
    groups = [int(g) for g in args.groups.split(",")] if args.groups else [0]
    lib = gemm._native.lib("plx_gemm")
    for model in args.models.split(","):
        T, linears = MODELS[model]
        for name, fin, fout in linears:
            x = torch.randn(T, fin, device=dev).to(torch.bfloat16)
            w = (torch.randn(fout, fin, device=dev) * 0.02).to(torch.bfloat16)
            dy = torch.randn(T, fout, device=dev).to(torch.bfloat16)
            n = max(1, args.cold)
            xs, ws, dys = [x] + [x.clone() for _ in range(n - 1)], [w] + [w.clone() for _ in range(n - 1)], \
                [dy] + [dy.clone() for _ in range(n - 1)]
            it = {"i": 0}

            def nxt():  # the operand copy of this call (round robin)
                it["i"] = (it["i"] + 1) % n
                return xs[it["i"]], ws[it["i"]], dys[it["i"]]

            def op(f):
                def run():
                    a_, b_, c_ = nxt()
                    return f(a_, b_, c_)
                return run
            # the kernel itself (gemm.gemm), not gemm.forward / dgrad / wgrad: those dispatch through ``auto``, which
            # sends the shapes outside ops/gemm.py's table to hipBLASLt (round 4's per-shape numbers for the forward
            # and most data gradients were hipBLASLt against itself)
            cases = [
                ("fwd", T, fout, fin, op(lambda x, w, dy: gemm.gemm(x, w, T, fout, fin, True, True)),
                 op(lambda x, w, dy: x @ w.t())),
                ("dgrad", T, fin, fout, op(lambda x, w, dy: gemm.gemm(dy, w, T, fin, fout, True, False)),
                 op(lambda x, w, dy: dy @ w)),
                ("wgrad", fout, fin, T, op(lambda x, w, dy: gemm.gemm(dy, x, fout, fin, T, False, False)),
                 op(lambda x, w, dy: dy.t() @ x)),
            ]
            for pas, M, N, K, nat, ref in cases:
                b = ref()
                fl = 2.0 * M * N * K
                tt = timed(ref, args.reps)
                tot["torch"] += tt
                rec = {"model": model, "linear": name, "pass": pas, "M": M, "N": N, "K": K,
                       "splits": gemm._native.size("plx_gemm", "plx_gemm256_splits", M, N, K),
                       "torch_ms": round(tt, 4), "torch_tflops": round(fl / tt / 1e9, 1)}
                for wv, grp in [(w_, g_) for g_ in groups for w_ in waves]:
                    gemm.FORCE_SCHEDULE = wv
                    if grp:
                        lib.plx_gemm256_set_group(grp)
                    a = nat()
                    err = ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()
                    tn = timed(nat, args.reps)
                    sfx = ("" if len(waves) == 1 else f"_w{wv}") + (f"_g{grp}" if grp else "")
                    tot["native" + sfx] = tot.get("native" + sfx, 0.0) + tn
                    rec.update({f"native{sfx}_ms": round(tn, 4), f"native{sfx}_tflops": round(fl / tn / 1e9, 1),
                                f"speedup{sfx}": round(tt / tn, 3), f"rel_err{sfx}": round(err, 5)})
                print(json.dumps(rec), flush=True)
            del x, w, dy, xs, ws, dys
    gemm.FORCE_SCHEDULE = 0
    print(json.dumps({f"total_{k}_ms": round(v, 3) for k, v in tot.items()}))


if __name__ == "__main__":
    main()
