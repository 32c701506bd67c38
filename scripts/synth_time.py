"""Time the device batch generator (plx_synth_images) at the bench's batch shape: bs 256, 224^2, bf16 NHWC."""
import json
import sys

import torch

from polyaxon_amd.ops.synth import SyntheticImages

dev = torch.device("cuda", 0)
d = SyntheticImages(256, 224, dev, classes=1000, active_classes=100, grid=7, signal=0.5, seed=0)
for _ in range(3):
    d.next()
torch.cuda.synchronize()
n = 20
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(n):
    d.next()
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) * 1000 / n
print(json.dumps({"kernel": "plx_synth_images", "batch": 256, "image": 224, "us_per_batch": round(us, 1),
                  "GB_per_s_written": round(d.x.numel() * 2 / us / 1e3, 1), "tag": sys.argv[1] if len(sys.argv) > 1 else ""}))
