"""Clock / power of the GPU while one GEMM runs back to back: the MFMA kernel (each schedule) vs hipBLASLt on a
Llama-3 8B shape, sampled with rocm-smi every 0.25 s (is the kernel's box-to-box spread a clock effect?).

    python scripts/gemm_clock_probe.py [seconds=4] [M N K]
One JSON line per variant: TFLOP/s and the median sclk (MHz) / socket power (W) over the samples.
"""
import json
import os
import re
import subprocess
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from polyaxon_amd.ops import gemm  # noqa: E402


def sample(stop, out):
    while not stop.is_set():
        try:
            r = subprocess.run(["rocm-smi", "--showclocks", "--showpower"], capture_output=True, text=True, timeout=5)
            s = re.search(r"sclk clock level: \d+: \((\d+)Mhz\)", r.stdout)
            p = re.search(r"Power \(W\): ([0-9.]+)", r.stdout)
            if s:
                out.append((float(s.group(1)), float(p.group(1)) if p else float("nan")))
        except Exception:
            pass
        time.sleep(0.25)


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    M, N, K = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (4096, 28672, 4096)
    dev = torch.device("cuda", 0)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    variants = [("hipblaslt", None), ("k8", 8), ("k5", 5), ("k7", 7), ("hipblaslt", None)]
    for name, v in variants:
        fn = (lambda: x @ w.t()) if v is None else (lambda: gemm.gemm(x, w, M, N, K, True, True))
        gemm.FORCE_SCHEDULE = v or 0
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        stop, smp = threading.Event(), []
        th = threading.Thread(target=sample, args=(stop, smp), daemon=True)
        th.start()
        n, t0 = 0, time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        while time.perf_counter() - t0 < secs:
            for _ in range(20):
                fn()
            n += 20
            torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        stop.set()
        th.join()
        ms = e0.elapsed_time(e1) / n
        sc = sorted(s for s, _ in smp)
        pw = sorted(p for _, p in smp)
        print(json.dumps({"variant": name, "M": M, "N": N, "K": K, "tflops": round(2.0 * M * N * K / ms / 1e9, 1),
                          "sclk_mhz_median": sc[len(sc) // 2] if sc else None,
                          "sclk_mhz_min": sc[0] if sc else None, "power_w_median": pw[len(pw) // 2] if pw else None,
                          "samples": len(sc)}), flush=True)
    gemm.FORCE_SCHEDULE = 0


if __name__ == "__main__":
    main()
