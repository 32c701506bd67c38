"""Stem convolution forward: MIOpen (F.conv2d, bf16 NHWC) vs the packed-super-pixel MFMA GEMM (ops/stem.py), each
timed as 10 calls captured in one hipGraph (median of 5 replays); prints one JSON line per variant."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def timeit(fn, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[2] * 1e3 / reps


def main():
    from polyaxon_amd.ops import _native
    from polyaxon_amd.ops.conv1x1 import _zero_page
    from polyaxon_amd.ops.stem import StemConv

    dev = torch.device("cuda")
    n = int(os.environ.get("BS", "256"))
    x = torch.randn(n, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    conv = StemConv().to(dev)
    wb = conv.weight.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    lib = _native.lib("plx_conv")
    xp = torch.empty(n * 224 * 112 * 8, dtype=torch.bfloat16, device=dev)
    wp = torch.empty(64, 256, dtype=torch.bfloat16, device=dev)
    y = torch.empty(n, 64, 112, 112, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    nblk = -(-n * 112 * 112 // 256)
    stats = torch.empty(2 * nblk * 64, dtype=torch.float32, device=dev)
    w = conv.weight.detach()
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa
    z = _zero_page(dev).data_ptr()
    res = {
        "miopen_fwd": timeit(lambda: F.conv2d(x, wb, None, 2, 3)),
        "pack_input": timeit(lambda: lib.plx_stem_pack_input(x.data_ptr(), xp.data_ptr(), n, 224, 224, st())),
        "pack_weight": timeit(lambda: lib.plx_stem_pack_weight(w.data_ptr(), *w.stride(), wp.data_ptr(), 64, st())),
        "stem_gemm": timeit(lambda: lib.plx_stem_conv_fwd(xp.data_ptr(), wp.data_ptr(), y.data_ptr(), n, 224, 224, z,
                                                          stats.data_ptr(), st())),
    }
    dy = torch.randn(n, 64, 112, 112, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    from polyaxon_amd.ops.conv1x1 import _num_cus
    cus = _num_cus(dev)
    ws = torch.empty(int(lib.plx_stem_conv_wgrad_workspace(n, 224, 224, cus)), dtype=torch.float32, device=dev)
    gw = torch.zeros(64, 3, 7, 7, device=dev)
    res["miopen_wgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]))
    res["stem_wgrad"] = timeit(lambda: lib.plx_stem_conv_wgrad(dy.data_ptr(), xp.data_ptr(), gw.data_ptr(), *gw.stride(),
                                                               ws.data_ptr(), n, 224, 224, z, cus, 1, st()))
    for k, v in res.items():
        print(json.dumps({"pass": k, "us": round(v, 1)}))


if __name__ == "__main__":
    main()
