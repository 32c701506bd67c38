"""Host (Python) cost of the LM trainer's step: cProfile over ``train_lm`` (GPT-2 125M by default), top functions by
own time.  The trainer's JSON line reports host_ms_per_step against ms_per_step; equal values mean the GPU waited for
the host's launches.

    python scripts/lm_host_profile.py [--top 40] [-- trainer args]
"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    argv = sys.argv[1:]
    top = 40
    if argv[:1] == ["--top"]:
        top, argv = int(argv[1]), argv[2:]
    if argv[:1] == ["--"]:
        argv = argv[1:]
    if not argv:
        argv = ["--model", "gpt2_125m", "--bs", "16", "--seq", "1024", "--steps", "20"]
    from polyaxon_amd.trainers import train_lm

    pr = cProfile.Profile()
    pr.enable()
    train_lm(argv)
    pr.disable()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(top)
    print(buf.getvalue())


if __name__ == "__main__":
    main()
