"""Interleaved A/B of the implicit-GEMM convolution kernels on the ResNet-50 3x3 shapes (bs 256), one process.

Each variant is a set of knob calls on libplx_conv (``plx_set_*``); every round runs every variant once per
(shape, pass) in a rotating order, so clock / thermal drift hits all of them alike (cdna_hip_programming.md §5.4
rule 24).  The first run of every variant is checked against an fp32 ``F.conv2d`` reference (forward) or
``conv_transpose2d`` (data gradient).  Prints one JSON line per (shape, pass) with the median and min µs and the
TFLOP/s of each variant.

    python scripts/conv_ab.py [variants=base,tap_inner] [rounds=7] [passes=fwd,dgrad] [shapes=all|s1|s2]

CONV_AB_DATA=relu (default: the input is post-ReLU, half zeros, as in training -- the chip holds a higher clock on
such data, cdna_hip_programming.md §5.4 rule 25) or randn.
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from polyaxon_amd.ops import _native  # noqa: E402
from polyaxon_amd.ops.conv import weight_prep_k  # noqa: E402
from polyaxon_amd.ops.conv1x1 import _zero_page  # noqa: E402

# (batch, c_in, c_out, input side, stride): the ResNet-50 3x3 convolutions
S1 = [(256, 64, 64, 56, 1), (256, 128, 128, 28, 1), (256, 256, 256, 14, 1), (256, 512, 512, 7, 1)]
S2 = [(256, 128, 128, 56, 2), (256, 256, 256, 28, 2), (256, 512, 512, 14, 2)]

VARIANTS = {
    "r3": {},  # the round-3 kernels (libplx_conv_r3ref.so, built from git history into _native/ when present)
    "base": {"plx_set_tap_inner": 0},
    "tap_inner": {"plx_set_tap_inner": 1},
}


def arg(i, default):
    return sys.argv[i] if len(sys.argv) > i and sys.argv[i] else default


def main():
    variants = arg(1, "base,tap_inner").split(",")
    rounds = int(arg(2, "7"))
    passes = arg(3, "fwd,dgrad").split(",")
    which = arg(4, "all")
    shapes = (S1 if which in ("all", "s1") else []) + (S2 if which in ("all", "s2") else [])
    dev = torch.device("cuda", 0)
    lib = _native.lib("plx_conv")
    libs = {v: lib for v in variants}
    if "r3" in variants:
        import ctypes

        r3 = ctypes.CDLL(str(_native.OUT / "libplx_conv_r3ref.so"))
        for fn, argtypes in _native.SIGNATURES["plx_conv"].items():
            if hasattr(r3, fn):
                f = getattr(r3, fn)
                f.argtypes = argtypes
                f.restype = _native.RESTYPES.get(fn, ctypes.c_int)
        libs["r3"] = r3
    relu = os.environ.get("CONV_AB_DATA", "relu") == "relu"  # post-ReLU activations, as in training
    st = torch.cuda.current_stream().cuda_stream
    zero = _zero_page(dev).data_ptr()

    cur = {"lib": lib}

    def apply(v):
        cur["lib"] = libs[v]
        for fn, val in VARIANTS[v].items():
            getattr(lib, fn)(*(val if isinstance(val, tuple) else (val,)))

    torch.manual_seed(0)
    for n, ci, co, h, s in shapes:
        ho = (h + 2 - 3) // s + 1
        x = torch.randn(n, h, h, ci, device=dev)
        x = (x.clamp_min(0) if relu else x).to(torch.bfloat16)
        w = torch.randn(co, ci, 3, 3, device=dev) * (1.0 / (9 * ci) ** 0.5)
        wf, wd = weight_prep_k(w)
        y = torch.empty(n, ho, ho, co, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(n, ho, ho, co, device=dev).to(torch.bfloat16)
        dx = torch.empty(n, h, h, ci, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * n * ho * ho * co * ci * 9
        ref = {}
        if "fwd" in passes:
            ref["fwd"] = F.conv2d(x.permute(0, 3, 1, 2).float(), w, None, s, 1).permute(0, 2, 3, 1)
        if "dgrad" in passes:
            ref["dgrad"] = torch.nn.grad.conv2d_input((n, ci, h, h), w, dy.permute(0, 3, 1, 2).float(), s, 1).permute(
                0, 2, 3, 1)

        def run(p):
            lib = cur["lib"]
            if p == "fwd":
                rc = lib.plx_conv_fwd(x.data_ptr(), wf.data_ptr(), y.data_ptr(), n, h, h, ci, co, 3, s, zero, None, st)
            else:
                rc = lib.plx_conv_dgrad(dy.data_ptr(), wd.data_ptr(), dx.data_ptr(), n, h, h, ci, co, 3, s, zero, None,
                                        None, st)
            assert rc == 0, rc

        for p in passes:
            out = y if p == "fwd" else dx
            err = {}
            for v in variants:
                apply(v)
                out.fill_(float("nan"))
                run(p)
                torch.cuda.synchronize()
                r = ref[p]
                e = ((out.float() - r).abs().max() / r.abs().max()).item()
                err[v] = e
                assert e < 2e-2, (v, p, e)
            times = {v: [] for v in variants}
            reps = 10
            for rd in range(rounds):
                order = variants[rd % len(variants):] + variants[:rd % len(variants)]
                for v in order:
                    apply(v)
                    run(p)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(reps):
                        run(p)
                    b.record()
                    torch.cuda.synchronize()
                    times[v].append(a.elapsed_time(b) * 1e3 / reps)
            rec = {"shape": f"{ci}->{co}@{h}s{s}", "pass": p, "gflop": round(flops / 1e9, 1)}
            for v in variants:
                t = sorted(times[v])
                med = t[len(t) // 2]
                rec[v] = {"us": round(med, 1), "min": round(t[0], 1), "tflops": round(flops / med / 1e6, 0),
                          "err": float(f"{err[v]:.2e}")}
            print(json.dumps(rec), flush=True)
    apply(variants[0])


if __name__ == "__main__":
    main()
