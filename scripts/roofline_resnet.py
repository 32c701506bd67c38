"""Per-kernel roofline of the ResNet-50 training step (bs 256, 224^2, bf16 NHWC) on MI355X.

Every native pass of every layer shape is timed in isolation (10 calls captured in one hipGraph, median of 5 replays, per call) with the exact
arguments the model uses (dgrad epilogues with the fused BatchNorm-backward partials / residual add, wgrad into
the fp32 flat slot, BatchNorm from the GEMM-epilogue partials).  Bytes are the compulsory HBM traffic from the
shapes (each operand read once, each output written once; a 3x3 gather counts its source image once) and FLOPs
the GEMM work; the roofline time is max(bytes / 8 TB/s, flops / 2.5 PFLOP/s) (MI355X dense bf16, HBM3E peak).

    python scripts/roofline_resnet.py [--bs 256] [--md profiles/r2_resnet50_roofline.md]

Prints one JSON line per (layer pass) and, with --md, writes the per-kernel table plus per-class totals
(multiplied by how often each shape occurs in the network) for comparison with the steady-state profile.
"""
import argparse
import ctypes
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM = 8.0e12
MFMA = 2.5e15


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bs", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--md", default="")
    ap.add_argument("--only", default="", help="comma-separated substrings: time only matching layers")
    ap.add_argument("--bn-apply-only", type=int, default=0, help="also time the apply pass alone")
    ap.add_argument("--bn-counters", type=int, default=1, help="A/B knob: 1 = fused BN reduce+finalize (ticket "
                    "counters), 0 = the two-launch path")
    a = ap.parse_args()
    import torch

    from polyaxon_amd.ops import _native
    from polyaxon_amd.ops.conv1x1 import _num_cus, _zero_page, nt_stats_rows

    dev = torch.device("cuda")
    conv = _native.lib("plx_conv")
    bn = _native.lib("plx_bn")
    cus = _num_cus(dev)
    zero = _zero_page(dev).data_ptr()
    st = torch.cuda.current_stream().cuda_stream
    cnt = torch.zeros(64, dtype=torch.int32, device=dev)  # BatchNorm reduce + finalize tickets
    cptr = cnt.data_ptr() if a.bn_counters else None
    bf = dict(dtype=torch.bfloat16, device=dev)
    f32 = dict(dtype=torch.float32, device=dev)
    rows = []

    def timeit(fn):
        """GPU time per call: ``a.reps`` calls captured in one hipGraph, replayed back to back (as in the training
        step), so host launch latency never shows up in a small kernel's number; median of 5 replays."""
        nonlocal st
        base = st
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            st = s.cuda_stream
            for _ in range(2):
                fn()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(a.reps):
                    fn()
        st = base
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for e0, e1 in ev:
            e0.record()
            g.replay()
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        return ts[len(ts) // 2] * 1e3 / a.reps  # us

    def emit(layer, kind, count, us, nbytes, flops):
        roof = max(nbytes / HBM, flops / MFMA) * 1e6
        r = {"layer": layer, "pass": kind, "count": count, "us": round(us, 1), "MB": round(nbytes / 1e6, 1),
             "GFLOP": round(flops / 1e9, 2), "TBps": round(nbytes / us / 1e6, 2),
             "TFLOPs": round(flops / us / 1e6, 1), "roof_us": round(roof, 1), "pct_roof": round(100 * roof / us, 1),
             "bound": "HBM" if nbytes / HBM >= flops / MFMA else "MFMA"}
        rows.append(r)
        print(json.dumps(r), flush=True)

    def rnd(shape, dtype=torch.bfloat16):
        return torch.randn(*shape, dtype=dtype, device=dev)

    def bn_args(m, c):
        x = rnd((m, c))
        mean = x.float().mean(0).contiguous()
        invstd = torch.rsqrt(x.float().var(0) + 1e-5).contiguous()
        mask = torch.randint(0, 255, (m * c // 8,), dtype=torch.uint8, device=dev)
        return x, mask, mean, invstd

    def wanted(name):
        return not a.only or any(t in name for t in a.only.split(","))

    def conv_layer(name, count, nb, h, w, cin, cout, k, s, dgrad_mode):
        """dgrad_mode: 'bnr' (fused BN-backward partials), 'add+bnr', 'add' (residual / deferred gradient), ''"""
        if not wanted(name):
            return
        ho, wo = (h + 2 * (k // 2) - k) // s + 1, (w + 2 * (k // 2) - k) // s + 1
        m_in, m_out = nb * h * w, nb * ho * wo
        x = rnd((m_in, cin))
        y = torch.empty(m_out, cout, **bf)
        dy = rnd((m_out, cout))
        dx = torch.empty(m_in, cin, **bf)
        flops = 2.0 * m_out * cout * cin * k * k
        wbytes = 2.0 * cout * cin * k * k
        gemm = k == 1 and s == 1
        rpb = nt_stats_rows(cout)
        stats = torch.empty(2 * (-(-m_out // rpb)) * cout, **f32)
        wb = rnd((cout, k * k * cin))
        wt = rnd((cin, k * k * cout))
        if gemm:
            fwd = lambda: conv.plx_gemm_nt(x.data_ptr(), wb.data_ptr(), y.data_ptr(), m_out, cout, cin, cin, cin,  # noqa
                                           cout, zero, stats.data_ptr(), None, 0, None, None, st)
        else:
            fwd = lambda: conv.plx_conv_fwd(x.data_ptr(), wb.data_ptr(), y.data_ptr(), nb, h, w, cin, cout, k, s,  # noqa
                                            zero, stats.data_ptr(), st)
        emit(name, "fwd", count, timeit(fwd), 2.0 * (m_in * cin + m_out * cout) + wbytes + stats.numel() * 4, flops)
        # data gradient
        extra = 0.0
        add = rnd((m_in, cin)) if "add" in dgrad_mode else None
        amask = None
        if add is not None:
            extra += 2.0 * m_in * cin
            if gemm and "bnr" in dgrad_mode:  # identity block: bn3's incoming gradient + its ReLU mask (no dres)
                amask = torch.randint(0, 255, (m_in * cin // 8,), dtype=torch.uint8, device=dev)
                extra += m_in * cin / 8
        bnr = None
        if "bnr" in dgrad_mode:
            bx, mask, mean, invstd = bn_args(m_in, cin)
            nblk = (-(-m_in // nt_stats_rows(cin))) if gemm else int(conv.plx_conv_dgrad_blocks(nb, h, w, cin, cout, k, s))
            part = torch.empty(2 * nblk * cin, **f32)
            bnr = _native.BnBwdArgs(bx.data_ptr(), mask.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                                    part.data_ptr(), nblk, 0)
            extra += 2.0 * m_in * cin + m_in * cin / 8 + part.numel() * 4
        bp = ctypes.addressof(bnr) if bnr is not None else None
        if gemm:
            dg = lambda: conv.plx_gemm_nt(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), m_in, cin, cout, cout, cout,  # noqa
                                          cin, zero, None, add.data_ptr() if add is not None else None,
                                          cin if add is not None else 0,
                                          amask.data_ptr() if amask is not None else None, bp, st)
        else:
            target = add if (add is not None and k == 1 and s == 2) else dx  # strided 1x1: in place on the deferred grad
            dg = lambda: conv.plx_conv_dgrad(dy.data_ptr(), wt.data_ptr(), target.data_ptr(), nb, h, w, cin, cout,  # noqa
                                             k, s, zero, add.data_ptr() if add is not None else None, bp, st)
        emit(name, "dgrad", count, timeit(dg), 2.0 * (m_out * cout + m_in * cin) + wbytes + extra, flops)
        # weight gradient into the fp32 flat slot (+=), slab reduction included
        g = torch.zeros(cout, k * k * cin, **f32)
        if gemm:
            ws = torch.empty(int(conv.plx_gemm_tn_workspace(m_out, cout, cin, cus)), **f32)
            wg = lambda: conv.plx_gemm_tn(dy.data_ptr(), x.data_ptr(), g.data_ptr(), ws.data_ptr(), m_out, cout, cin,  # noqa
                                          cout, cin, cin, zero, cus, 1, st)
        else:
            ws = torch.empty(int(conv.plx_conv_wgrad_workspace(nb, h, w, cin, cout, k, s, cus)), **f32)
            wg = lambda: conv.plx_conv_wgrad(dy.data_ptr(), x.data_ptr(), g.data_ptr(), ws.data_ptr(), nb, h, w, cin,  # noqa
                                             cout, k, s, zero, cus, 1, st)
        emit(name, "wgrad", count, timeit(wg), 2.0 * (m_out * cout + m_in * cin) + 8.0 * cout * cin * k * k, flops)

    def bn_layer(name, count, m, c, relu, res, partials_bwd):
        if not wanted(name):
            return
        x, mask, mean, invstd = bn_args(m, c)
        y = torch.empty(m, c, **bf)
        r = rnd((m, c)) if res else None
        weight, bias = torch.ones(c, **f32), torch.zeros(c, **f32)
        rm, rv = torch.zeros(c, **f32), torch.ones(c, **f32)
        stats = torch.empty(4 * c, **f32)
        nblk = -(-m // 128)
        part = torch.rand(2 * nblk * c, **f32)
        l2 = torch.empty(int(bn.plx_bn_l2_workspace(nblk, c)), **f32)
        mo = torch.empty(m * c // 8, dtype=torch.uint8, device=dev) if relu else None
        fwd = lambda: bn.plx_bn_forward_from_partials(  # noqa
            x.data_ptr(), r.data_ptr() if r is not None else None, y.data_ptr(), m, c, weight.data_ptr(),
            bias.data_ptr(), 1e-5, 0.1, rm.data_ptr(), rv.data_ptr(), stats.data_ptr(), stats[c:].data_ptr(),
            stats[2 * c:].data_ptr(), part.data_ptr(), nblk, l2.data_ptr(),
            mo.data_ptr() if mo is not None else None, int(relu), None, cptr, st)
        nbytes = 2.0 * m * c * (2 + (1 if res else 0)) + (m * c / 8 if relu else 0)
        emit(name, "bn_fwd", count, timeit(fwd), nbytes, 0.0)
        if a.bn_apply_only:
            app = lambda: bn.plx_bn_apply(x.data_ptr(), r.data_ptr() if r is not None else None, y.data_ptr(), m, c,  # noqa
                                          stats[2 * c:].data_ptr(), int(relu), st)
            emit(name, "bn_apply", count, timeit(app), nbytes, 0.0)
        dy = rnd((m, c))
        dx = torch.empty(m, c, **bf)
        dres = torch.empty(m, c, **bf) if res else None
        dg, db, coef = torch.zeros(c, **f32), torch.zeros(c, **f32), torch.empty(3 * c, **f32)
        mp = mask.data_ptr() if relu else None
        if partials_bwd:
            bwd = lambda: bn.plx_bn_backward_from_partials(  # noqa
                x.data_ptr(), mp, dy.data_ptr(), dx.data_ptr(), dres.data_ptr() if dres is not None else None, m, c,
                weight.data_ptr(), mean.data_ptr(), invstd.data_ptr(), dg.data_ptr(), db.data_ptr(), coef.data_ptr(),
                part.data_ptr(), nblk, l2.data_ptr(), int(relu), 1, None, cptr, st)
        else:
            pw = torch.empty(int(bn.plx_bn_workspace(m, c)), **f32)
            bwd = lambda: bn.plx_bn_backward(  # noqa
                x.data_ptr(), mp, dy.data_ptr(), dx.data_ptr(), dres.data_ptr() if dres is not None else None, m, c,
                weight.data_ptr(), mean.data_ptr(), invstd.data_ptr(), dg.data_ptr(), db.data_ptr(), coef.data_ptr(),
                pw.data_ptr(), int(relu), 1, None, cptr, st)
        nbytes = 2.0 * m * c * (3 + (1 if res else 0)) + (m * c / 8 if relu else 0)
        emit(name, "bn_bwd" + ("" if partials_bwd else "+reduce"), count, timeit(bwd), nbytes, 0.0)

    def stem_pool(name):
        """stem BN + ReLU + max-pool: fused (ops/stem.py) vs BN (stats, apply + mask) followed by the pool."""
        if not wanted(name):
            return
        n, c, h, w = a.bs, 64, 112, 112
        m = n * h * w
        pool = _native.lib("plx_pool")
        x, mask, mean, invstd = bn_args(m, c)
        weight, bias = torch.ones(c, **f32), torch.zeros(c, **f32)
        rm, rv = torch.zeros(c, **f32), torch.ones(c, **f32)
        stats = torch.empty(4 * c, **f32)
        ws = torch.empty(int(bn.plx_bn_workspace(m, c)), **f32)
        y = torch.empty(m, c, **bf)
        p = torch.empty(n * 56 * 56, c, **bf)
        idx = torch.empty(n * 56 * 56 * c, dtype=torch.uint8, device=dev)
        ff = lambda: bn.plx_stem_bn_pool_forward(  # noqa
            x.data_ptr(), p.data_ptr(), idx.data_ptr(), n, h, w, c, weight.data_ptr(), bias.data_ptr(), 1e-5, 0.1,
            rm.data_ptr(), rv.data_ptr(), stats.data_ptr(), stats[c:].data_ptr(), stats[2 * c:].data_ptr(),
            ws.data_ptr(), None, 0, cptr, st)

        def fu():
            bn.plx_bn_forward(x.data_ptr(), None, y.data_ptr(), m, c, weight.data_ptr(), bias.data_ptr(), 1e-5, 0.1,
                              rm.data_ptr(), rv.data_ptr(), stats.data_ptr(), stats[c:].data_ptr(),
                              stats[2 * c:].data_ptr(), ws.data_ptr(), mask.data_ptr(), 1, None, cptr, st)
            pool.plx_maxpool3s2_forward(y.data_ptr(), p.data_ptr(), idx.data_ptr(), n, h, w, c, st)
        nbytes = 2.0 * m * c * 2 + 3.0 * n * 56 * 56 * c
        emit(name + " fused", "fwd", 1, timeit(ff), nbytes, 0.0)
        emit(name + " unfused", "fwd", 1, timeit(fu), nbytes, 0.0)
        dp = rnd((n * 56 * 56, c))
        dx = torch.empty(m, c, **bf)
        dy1 = torch.empty(m, c, **bf)
        dg, db, coef = torch.zeros(c, **f32), torch.zeros(c, **f32), torch.empty(3 * c, **f32)
        wsb = torch.empty(int(bn.plx_stem_bn_pool_bwd_workspace(n, h, w, c)), **f32)
        bf_ = lambda: bn.plx_stem_bn_pool_backward(  # noqa
            dp.data_ptr(), idx.data_ptr(), x.data_ptr(), dx.data_ptr(), n, h, w, c, weight.data_ptr(),
            mean.data_ptr(), invstd.data_ptr(), stats[2 * c:].data_ptr(), dg.data_ptr(), db.data_ptr(),
            coef.data_ptr(), wsb.data_ptr(), 1, cptr, st)

        def bu():
            pool.plx_maxpool3s2_backward(dp.data_ptr(), idx.data_ptr(), dy1.data_ptr(), n, h, w, c, st)
            bn.plx_bn_backward(x.data_ptr(), mask.data_ptr(), dy1.data_ptr(), dx.data_ptr(), None, m, c,
                               weight.data_ptr(), mean.data_ptr(), invstd.data_ptr(), dg.data_ptr(), db.data_ptr(),
                               coef.data_ptr(), ws.data_ptr(), 1, 1, None, cptr, st)
        nbytes = 2.0 * m * c * 2 + 3.0 * n * 56 * 56 * c
        emit(name + " fused", "bwd", 1, timeit(bf_), nbytes, 0.0)
        emit(name + " unfused", "bwd", 1, timeit(bu), nbytes, 0.0)

    nb = a.bs
    stem_pool("stem_pool 64@112")
    bn_layer("stem_bn 64@112", 1, nb * 112 * 112, 64, True, False, False)
    cfg = [(3, 64, 56, 1), (4, 128, 56, 2), (6, 256, 28, 2), (3, 512, 14, 2)]
    in_ch = 64
    for si, (blocks, wd, hin, s) in enumerate(cfg):
        out = wd * 4
        hout = hin // s
        tag = f"s{si + 1}"
        # first block (downsampling)
        conv_layer(f"{tag}.0.conv1 1x1 {in_ch}->{wd}@{hin}", 1, nb, hin, hin, in_ch, wd, 1, 1, "")
        conv_layer(f"{tag}.0.conv2 3x3/{s} {wd}@{hin}", 1, nb, hin, hin, wd, wd, 3, s, "bnr")
        conv_layer(f"{tag}.0.conv3 1x1 {wd}->{out}@{hout}", 1, nb, hout, hout, wd, out, 1, 1, "bnr")
        conv_layer(f"{tag}.0.down 1x1/{s} {in_ch}->{out}@{hin}", 1, nb, hin, hin, in_ch, out, 1, s, "add")
        bn_layer(f"{tag}.0.bn1 {wd}@{hin}", 1, nb * hin * hin, wd, True, False, True)
        bn_layer(f"{tag}.bn2 {wd}@{hout}", blocks, nb * hout * hout, wd, True, False, True)
        bn_layer(f"{tag}.bn3 {out}@{hout}", blocks, nb * hout * hout, out, True, True, True)
        bn_layer(f"{tag}.0.down_bn {out}@{hout}", 1, nb * hout * hout, out, False, False, False)
        if blocks > 1:
            conv_layer(f"{tag}.j.conv1 1x1 {out}->{wd}@{hout}", blocks - 1, nb, hout, hout, out, wd, 1, 1, "add+bnr")
            conv_layer(f"{tag}.j.conv2 3x3 {wd}@{hout}", blocks - 1, nb, hout, hout, wd, wd, 3, 1, "bnr")
            conv_layer(f"{tag}.j.conv3 1x1 {wd}->{out}@{hout}", blocks - 1, nb, hout, hout, wd, out, 1, 1, "bnr")
            bn_layer(f"{tag}.j.bn1 {wd}@{hout}", blocks - 1, nb * hout * hout, wd, True, False, True)
        in_ch = out

    if a.md:
        cls = defaultdict(lambda: [0.0, 0.0, 0.0, 0.0])
        for r in rows:
            c = cls[r["pass"]]
            c[0] += r["us"] * r["count"] / 1e3
            c[1] += r["roof_us"] * r["count"] / 1e3
            c[2] += r["MB"] * r["count"]
            c[3] += r["GFLOP"] * r["count"]
        tot = [sum(v[i] for v in cls.values()) for i in range(4)]
        lines = [
            f"# ResNet-50 training step roofline (bs {nb}, 224^2, bf16 NHWC, MI355X) -- per-kernel, shapes from the model",
            "",
            "`scripts/roofline_resnet.py`: each native pass of each layer shape timed in isolation "
            f"({a.reps} calls captured in one hipGraph, median of 5 replays, per call) with the model's arguments.  Bytes = compulsory HBM traffic from the shapes; roofline = "
            "max(bytes / 8 TB/s, FLOPs / 2.5 PFLOP/s).  `count` = occurrences of the shape per step.",
            "",
            "## Per class (sum over the network)",
            "",
            "| pass | ms/step | roofline ms/step | % of roofline | GB/step | TFLOP/step | achieved TB/s |",
            "|---|---|---|---|---|---|---|"]
        for k, (ms, roof, mb, gf) in sorted(cls.items(), key=lambda kv: -kv[1][0]):
            lines.append(f"| {k} | {ms:.2f} | {roof:.2f} | {100 * roof / ms:.0f}% | {mb / 1e3:.2f} | {gf / 1e3:.3f} | "
                         f"{mb / 1e3 / ms:.2f} |")
        lines.append(f"| **total** | {tot[0]:.2f} | {tot[1]:.2f} | {100 * tot[1] / tot[0]:.0f}% | {tot[2] / 1e3:.2f} | "
                     f"{tot[3] / 1e3:.3f} | {tot[2] / 1e3 / tot[0]:.2f} |")
        lines += ["", "## Per kernel call", "",
                  "| layer | pass | count | us | MB | GFLOP | TB/s | TFLOP/s | roofline us | % roofline | bound |",
                  "|---|---|---|---|---|---|---|---|---|---|---|"]
        for r in rows:
            lines.append(f"| {r['layer']} | {r['pass']} | {r['count']} | {r['us']} | {r['MB']} | {r['GFLOP']} | "
                         f"{r['TBps']} | {r['TFLOPs']} | {r['roof_us']} | {r['pct_roof']}% | {r['bound']} |")
        with open(a.md, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
