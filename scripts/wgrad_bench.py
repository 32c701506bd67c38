"""Weight-gradient (TN GEMM) kernels in isolation on every ResNet-50 wgrad shape, v1 (gemm_tn_kernel) against v2
(wgrad_kernel), each checked against an fp32 reference.  One process, CUDA events, median over rounds; prints one
JSON line per (shape, variant) and a step-weighted summary.

    python scripts/wgrad_bench.py [--variants v1,v2,v2w] [--rounds 5] [--reps 10] [--check 1]

Variants: v1 = the round-4 kernel and plan, v2 = wgrad_kernel with a 128 KB LDS ring (one block per CU), v2s = the
same with a 64 KB ring (two blocks per CU, or room for other kernels' blocks beside it).
"""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

from polyaxon_amd.ops import _native
from polyaxon_amd.ops.conv1x1 import _num_cus, _zero_page

# (n, cin, h, w, cout, k, s) -- input image h x w; COUNT = how many of each one ResNet-50 step runs
SHAPES = [(256, 64, 56, 56, 256, 1, 1), (256, 256, 56, 56, 64, 1, 1), (256, 64, 56, 56, 64, 1, 1),
          (256, 256, 56, 56, 128, 1, 1), (256, 512, 28, 28, 128, 1, 1), (256, 128, 28, 28, 512, 1, 1),
          (256, 512, 28, 28, 256, 1, 1), (256, 1024, 14, 14, 256, 1, 1), (256, 256, 14, 14, 1024, 1, 1),
          (256, 1024, 14, 14, 512, 1, 1), (256, 2048, 7, 7, 512, 1, 1), (256, 512, 7, 7, 2048, 1, 1),
          (256, 256, 56, 56, 512, 1, 2), (256, 512, 28, 28, 1024, 1, 2), (256, 1024, 14, 14, 2048, 1, 2),
          (256, 64, 56, 56, 64, 3, 1), (256, 128, 28, 28, 128, 3, 1), (256, 256, 14, 14, 256, 3, 1),
          (256, 512, 7, 7, 512, 3, 1), (256, 128, 56, 56, 128, 3, 2), (256, 256, 28, 28, 256, 3, 2),
          (256, 512, 14, 14, 512, 3, 2)]
COUNT = [4, 2, 1, 1, 3, 4, 1, 5, 6, 1, 2, 3, 1, 1, 1, 3, 3, 5, 2, 1, 1, 1]
VARIANTS = {"v1": (0, -1), "v2": (1, 128), "v2s": (1, 64)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="v1,v2,v2s")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--shapes", default="")
    args = ap.parse_args()
    variants = args.variants.split(",")
    dev = torch.device("cuda", 0)
    lib = _native.lib("plx_conv")
    cus = _num_cus(dev)
    zero = _zero_page(dev).data_ptr()
    stream = torch.cuda.current_stream().cuda_stream
    idx = [int(i) for i in args.shapes.split(",")] if args.shapes else list(range(len(SHAPES)))
    cases = []
    g = torch.Generator(device=dev).manual_seed(0)
    for ci in idx:
        n, cin, h, w, cout, k, s = SHAPES[ci]
        ho, wo = (h + 2 * (k // 2) - k) // s + 1, (w + 2 * (k // 2) - k) // s + 1
        x = torch.randn(n * h * w, cin, device=dev, generator=g).to(torch.bfloat16)
        dy = torch.randn(n * ho * wo, cout, device=dev, generator=g).to(torch.bfloat16)
        out = torch.empty(cout, k * k * cin, device=dev)
        ws = torch.empty(int(lib.plx_conv_wgrad_workspace(n, h, w, cin, cout, k, s, cus)) + 64, device=dev)
        if k == 1 and s == 1:
            ws2 = int(lib.plx_gemm_tn_workspace(n * h * w, cout, cin, cus))
            if ws2 + 64 > ws.numel():
                ws = torch.empty(ws2 + 64, device=dev)
        ref = None
        if args.check:
            xf = x.float().view(n, h, w, cin).permute(0, 3, 1, 2)
            dyf = dy.float().view(n, ho, wo, cout).permute(0, 3, 1, 2)
            ref = torch.nn.grad.conv2d_weight(xf, (cout, cin, k, k), dyf, stride=s, padding=k // 2)
            ref = ref.permute(0, 2, 3, 1).reshape(cout, k * k * cin)
            del xf, dyf
        cases.append((ci, (n, cin, h, w, cout, k, s, ho, wo), x, dy, out, ws, ref))

    def runner(case):
        ci, (n, cin, h, w, cout, k, s, ho, wo), x, dy, out, ws, _ = case
        if k == 1 and s == 1:
            m = n * h * w

            def run():
                _native.check(lib.plx_gemm_tn(dy.data_ptr(), x.data_ptr(), out.data_ptr(), ws.data_ptr(), m, cout, cin,
                                              cout, cin, cin, zero, cus, 0, stream), "plx_gemm_tn")
        else:
            def run():
                _native.check(lib.plx_conv_wgrad(dy.data_ptr(), x.data_ptr(), out.data_ptr(), ws.data_ptr(), n, h, w,
                                                 cin, cout, k, s, zero, cus, 0, stream), "plx_conv_wgrad")
        return run

    res = {v: {c[0]: [] for c in cases} for v in variants}
    err = {v: {} for v in variants}
    for rnd in range(args.rounds):
        for v in variants:
            lib.plx_set_tn_v2(*VARIANTS[v])
            for case in cases:
                run = runner(case)
                ci, ref = case[0], case[6]
                run()
                if rnd == 0 and ref is not None:
                    torch.cuda.synchronize()
                    e = ((case[4] - ref).abs().max() / ref.abs().max()).item()
                    err[v][ci] = e
                    assert e < 2e-2, (v, SHAPES[ci], e)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(args.reps):
                    run()
                en.record()
                torch.cuda.synchronize()
                res[v][ci].append(st.elapsed_time(en) / args.reps)
        print(f"# round {rnd} done", file=sys.stderr, flush=True)
    lib.plx_set_tn_v2(1, 128)
    tot = {v: 0.0 for v in variants}
    flops_tot = 0.0
    for case in cases:
        ci = case[0]
        n, cin, h, w, cout, k, s, ho, wo = case[1]
        fl = 2.0 * n * ho * wo * cout * cin * k * k
        flops_tot += fl * COUNT[ci]
        for v in variants:
            t = sorted(res[v][ci])[len(res[v][ci]) // 2]
            tot[v] += t * COUNT[ci]
            print(json.dumps({"shape": SHAPES[ci], "variant": v, "us": round(t * 1000, 1),
                              "tflops": round(fl / (t * 1e-3) / 1e12, 1), "rel_err": err[v].get(ci),
                              "count": COUNT[ci]}), flush=True)
    for v in variants:
        print(json.dumps({"summary": v, "step_weighted_ms": round(tot[v], 3),
                          "tflops": round(flops_tot / (tot[v] * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
