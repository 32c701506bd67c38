"""Calibrate the synthetic ResNet-50 task: loss after N fresh-batch steps for a few learning rates.

    python scripts/calib_synth.py --steps 36 --signal 0.5
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from polyaxon_amd.models.resnet import resnet50  # noqa: E402
from polyaxon_amd.ops.synth import SyntheticImages  # noqa: E402
from polyaxon_amd.polyflow.executor import ResidentTrialExecutor  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=36)
    ap.add_argument("--signal", type=float, nargs="+", default=[0.5])
    ap.add_argument("--lr", type=float, nargs="+", default=[0.05, 0.2, 0.8])
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for sig in args.signal:
        data = SyntheticImages(args.batch, 224, dev, signal=sig, seed=1234)
        ex = ResidentTrialExecutor(resnet50(), data, dev, use_graph=False)
        for lr in args.lr:
            ex.reset(seed=1)
            ex.set_hparams(lr=lr, momentum=0.9, weight_decay=1e-4)
            torch.cuda.synchronize()
            t = time.time()
            ex.run(args.steps)
            torch.cuda.synchronize()
            dt = (time.time() - t) / args.steps
            l = ex.losses()
            print(json.dumps({"signal": sig, "lr": lr, "ms_per_step": round(dt * 1000, 2),
                              "loss": [round(float(v), 3) for v in l[:: max(1, len(l) // 12)]],
                              "last4": round(float(l[-4:].mean()), 3)}), flush=True)


if __name__ == "__main__":
    main()
