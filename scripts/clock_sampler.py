"""Run a command and sample the GPU's shader clock and socket power with rocm-smi every 0.5 s while it runs; print
one JSON line with the median / quartiles (is a workload power-capped?).

    python scripts/clock_sampler.py -- python bench.py --steps 3 --warmup 1
"""
import json
import re
import subprocess
import sys
import time


def main():
    cmd = sys.argv[sys.argv.index("--") + 1:]
    p = subprocess.Popen(cmd)
    clk, pw = [], []
    while p.poll() is None:
        try:
            r = subprocess.run(["rocm-smi", "--showclocks", "--showpower", "--showuse"], capture_output=True, text=True,
                               timeout=5)
            s = re.search(r"sclk clock level: \d+: \((\d+)Mhz\)", r.stdout)
            w = re.search(r"Power \(W\): ([0-9.]+)", r.stdout)
            u = re.search(r"GPU use \(%\): (\d+)", r.stdout)
            if s and u and int(u.group(1)) > 50:  # only while the GPU is busy
                clk.append(float(s.group(1)))
                if w:
                    pw.append(float(w.group(1)))
        except Exception:
            pass
        time.sleep(0.5)

    def q(v, f):
        v = sorted(v)
        return v[min(len(v) - 1, int(f * len(v)))] if v else None

    print(json.dumps({"cmd": " ".join(cmd)[:120], "rc": p.returncode, "samples": len(clk),
                      "sclk_mhz": {"p25": q(clk, 0.25), "p50": q(clk, 0.5), "p75": q(clk, 0.75)},
                      "power_w": {"p25": q(pw, 0.25), "p50": q(pw, 0.5), "p75": q(pw, 0.75)}}), flush=True)
    sys.exit(p.returncode)


if __name__ == "__main__":
    main()
