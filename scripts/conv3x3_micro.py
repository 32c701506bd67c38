"""3x3 stride-1 implicit-GEMM convolutions of ResNet-50 (bs 256): forward (plx_conv_fwd) and data gradient
(plx_conv_dgrad) timed alone, TFLOP/s per pass -- the kernel-level view behind the roofline table, and the program
that rocprofv3 --pmc passes run (scripts/gpu_conv_pmc.sh).

    python scripts/conv3x3_micro.py [fwd|dgrad|both] [iters]
"""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

from polyaxon_amd.ops import _native  # noqa: E402
from polyaxon_amd.ops.conv import weight_prep_k  # noqa: E402
from polyaxon_amd.ops.conv1x1 import _zero_page  # noqa: E402

SHAPES = [(256, 64, 56), (256, 128, 28), (256, 256, 14), (256, 512, 7)]  # (batch, channels in = out, side)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    lib = _native.lib("plx_conv")
    st = torch.cuda.current_stream().cuda_stream
    zero = _zero_page(dev).data_ptr()
    for n, c, h in SHAPES:
        x = torch.randn(n, h, h, c, device=dev).to(torch.bfloat16)
        w = torch.randn(c, c, 3, 3, device=dev) * 0.05
        wf, wd = weight_prep_k(w)
        y = torch.empty(n, h, h, c, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * n * h * h * c * c * 9
        rec = {"shape": f"3x3 {c}@{h}", "gflop": round(flops / 1e9, 1)}
        for p in (["fwd", "dgrad"] if which == "both" else [which]):
            def run():
                if p == "fwd":
                    rc = lib.plx_conv_fwd(x.data_ptr(), wf.data_ptr(), y.data_ptr(), n, h, h, c, c, 3, 1, zero, None, st)
                else:
                    rc = lib.plx_conv_dgrad(y.data_ptr(), wd.data_ptr(), x.data_ptr(), n, h, h, c, c, 3, 1, zero, None,
                                            None, st)
                assert rc == 0
            run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                run()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / iters
            rec[p + "_us"] = round(ms * 1e3, 1)
            rec[p + "_tflops"] = round(flops / ms / 1e9, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
