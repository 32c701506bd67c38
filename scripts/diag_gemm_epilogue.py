"""Cost of plx_gemm_nt's fused epilogues (BatchNorm channel stats, BatchNorm-backward partials, residual add)
on ResNet-50 1x1 shapes: the same GEMM timed with each epilogue on and off (HIP events, median of 20).

    python scripts/diag_gemm_epilogue.py
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from polyaxon_amd.ops import _native
    from polyaxon_amd.ops.conv1x1 import _zero_page, nt_stats_rows

    conv = _native.lib("plx_conv")
    dev = torch.device("cuda")
    zero = _zero_page(dev).data_ptr()
    st = torch.cuda.current_stream().cuda_stream

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        return round(ts[len(ts) // 2] * 1e3, 1)

    nb = 256
    for (h, k, n) in [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024), (14, 1024, 256),
                      (7, 512, 2048)]:
        m = nb * h * h
        a = torch.randn(m, k, dtype=torch.bfloat16, device=dev)
        b = torch.randn(n, k, dtype=torch.bfloat16, device=dev)
        c = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
        d = torch.randn(m, n, dtype=torch.bfloat16, device=dev)
        nblk = -(-m // nt_stats_rows(n))
        stats = torch.empty(2 * nblk * n, dtype=torch.float32, device=dev)
        x = torch.randn(m, n, dtype=torch.bfloat16, device=dev)
        mask = torch.randint(0, 255, (m * n // 8,), dtype=torch.uint8, device=dev)
        mean = torch.zeros(n, dtype=torch.float32, device=dev)
        inv = torch.ones(n, dtype=torch.float32, device=dev)
        part = torch.empty(2 * nblk * n, dtype=torch.float32, device=dev)
        bnr = _native.BnBwdArgs(x.data_ptr(), mask.data_ptr(), mean.data_ptr(), inv.data_ptr(), part.data_ptr(), nblk, 0)

        def run(stats_on=False, add=False, bn=False):
            return lambda: conv.plx_gemm_nt(a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, k, k, n, zero,
                                            stats.data_ptr() if stats_on else None, d.data_ptr() if add else None,
                                            n if add else 0, None, ctypes.addressof(bnr) if bn else None, st)
        plain = timeit(run())
        rec = {"M": m, "N": n, "K": k, "plain_us": plain, "stats_us": timeit(run(stats_on=True)),
               "add_us": timeit(run(add=True)), "bnr_us": timeit(run(bn=True)),
               "add_bnr_us": timeit(run(add=True, bn=True)),
               "plain_TBps": round(2.0 * (m * k + m * n + n * k) / plain / 1e6, 2)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
