"""Sweep the weight-gradient slicing knobs (plx_set_tn_plan: blocks per CU, slab byte cap) over the
ResNet-50 wgrad shapes (1x1 and 3x3, stride 1 and 2).  One process, CUDA events, median of interleaved rounds;
prints ms per shape per plan and the total."""
import itertools
import sys

import torch

from polyaxon_amd.ops import _native
from polyaxon_amd.ops.conv1x1 import _num_cus, _zero_page

dev = torch.device("cuda", 0)
# (n, cin, h, w, cout, k, s)  -- the input image is h x w
SHAPES = [(256, 64, 56, 56, 256, 1, 1), (256, 256, 56, 56, 64, 1, 1), (256, 64, 56, 56, 64, 1, 1),
          (256, 256, 56, 56, 128, 1, 1), (256, 512, 28, 28, 128, 1, 1), (256, 128, 28, 28, 512, 1, 1),
          (256, 512, 28, 28, 256, 1, 1), (256, 1024, 14, 14, 256, 1, 1), (256, 256, 14, 14, 1024, 1, 1),
          (256, 1024, 14, 14, 512, 1, 1), (256, 2048, 7, 7, 512, 1, 1), (256, 512, 7, 7, 2048, 1, 1),
          (256, 256, 56, 56, 512, 1, 2), (256, 512, 28, 28, 1024, 1, 2), (256, 1024, 14, 14, 2048, 1, 2),
          (256, 64, 56, 56, 64, 3, 1), (256, 128, 28, 28, 128, 3, 1), (256, 256, 14, 14, 256, 3, 1),
          (256, 512, 7, 7, 512, 3, 1), (256, 128, 56, 56, 128, 3, 2), (256, 256, 28, 28, 256, 3, 2),
          (256, 512, 14, 14, 512, 3, 2)]
# how many of each shape one ResNet-50 step runs (layer blocks)
COUNT = [4, 2, 1, 1, 3, 4, 1, 5, 6, 1, 2, 3, 1, 1, 1, 3, 3, 5, 2, 1, 1, 1]
PLANS = [(3, 32), (4, 32), (2, 32), (6, 128)]


def main():
    lib = _native.lib("plx_conv")
    cus = _num_cus(dev)
    zero = _zero_page(dev).data_ptr()
    stream = torch.cuda.current_stream().cuda_stream
    cases = []
    for (n, cin, h, w, cout, k, s) in SHAPES:
        ho, wo = (h + 2 * (k // 2) - k) // s + 1, (w + 2 * (k // 2) - k) // s + 1
        x = torch.randn(n * h * w, cin, device=dev).to(torch.bfloat16)
        dy = torch.randn(n * ho * wo, cout, device=dev).to(torch.bfloat16)
        g = torch.empty(cout, k, k, cin, device=dev)
        cases.append((n, cin, h, w, cout, k, s, x, dy, g))
    res = {p: [[] for _ in cases] for p in PLANS}
    ref = {}
    for rnd in range(5):
        for plan in PLANS:
            lib.plx_set_tn_plan(*plan)
            for ci, (n, cin, h, w, cout, k, s, x, dy, g) in enumerate(cases):
                ws = torch.empty(int(lib.plx_conv_wgrad_workspace(n, h, w, cin, cout, k, s, cus)), device=dev)

                def run():
                    _native.check(lib.plx_conv_wgrad(dy.data_ptr(), x.data_ptr(), g.data_ptr(), ws.data_ptr(), n, h,
                                                     w, cin, cout, k, s, zero, cus, 0, stream), "plx_conv_wgrad")
                run()
                if rnd == 0:
                    if ci not in ref:
                        ref[ci] = g.clone()
                    else:
                        err = (g - ref[ci]).abs().max().item() / (ref[ci].abs().max().item() + 1e-9)
                        assert err < 1e-3, (plan, ci, err)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(5):
                    run()
                en.record()
                torch.cuda.synchronize()
                res[plan][ci].append(st.elapsed_time(en) / 5)
    lib.plx_set_tn_plan(3, 32)
    med = {p: [sorted(v)[len(v) // 2] for v in res[p]] for p in PLANS}
    hdr = "shape".ljust(34) + "".join(f"{str(p):>12}" for p in PLANS)
    print(hdr)
    for ci, sh in enumerate(SHAPES):
        print(str(sh).ljust(34) + "".join(f"{med[p][ci] * 1000:12.1f}" for p in PLANS))
    print("step-weighted total (us)".ljust(34) + "".join(
        f"{sum(c * t for c, t in zip(COUNT, med[p])) * 1000:12.1f}" for p in PLANS))
    best = [min(PLANS, key=lambda p: med[p][ci]) for ci in range(len(SHAPES))]
    print("best per shape:", best)
    print("step-weighted best-per-shape total (us): %.1f" % (sum(c * med[b][ci] for ci, (c, b) in
                                                                   enumerate(zip(COUNT, best))) * 1000))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
