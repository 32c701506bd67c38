"""How far the host runs ahead of the GPU inside the resident ResNet-50 step, without a profiler attached.

The host time at which a point of the step is *issued* is compared with the GPU time at which the GPU *reaches* it.
GPU times come from events, mapped to the host clock through a reference event recorded on an idle, synchronised
device.  A lead near zero at a point means the GPU waited there for the host's launches.

Points: forward issued (the loss is computed), backward issued (loss.backward() returned), step issued (optimizer
queued).  The script also prints the host time per step against the GPU time per step.

    python scripts/host_lead.py [--steps 40] [--trial-steps 0]

``--trial-steps N`` re-arms a trial every N steps (reset + hyper-parameters), as the Hyperband bench does.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--trial-steps", type=int, default=0)
    a = ap.parse_args()
    from polyaxon_amd.polyflow.programs import build_program

    dev = torch.device("cuda", 0)
    prog = build_program("resnet50", {"batch": 256, "image": 224, "unit_steps": 4, "signal": 0.5, "data_seed": 1234},
                         dev)
    prog.warm()
    ex = prog.executor
    hp = {"lr": 0.1, "momentum": 0.9, "weight_decay": 1e-4}
    ex.reset(seed=1)
    ex.set_hparams(**hp)
    ex.run(3)
    marks = []  # (label, host_s, event)
    loss_fn, step_fn = ex.loss_fn, ex.opt.step_

    def mark(label):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((label, time.perf_counter(), ev))

    def loss_hook(out, y):
        loss = loss_fn(out, y)
        mark("fwd")
        return loss

    def step_hook():
        mark("bwd")
        step_fn()
        mark("step")

    ex.loss_fn, ex.opt.step_ = loss_hook, step_hook
    torch.cuda.synchronize()
    ref = torch.cuda.Event(enable_timing=True)
    time.sleep(0.01)
    h0 = time.perf_counter()
    ref.record()
    for i in range(a.steps):
        if a.trial_steps and i and i % a.trial_steps == 0:
            ex.reset(seed=i)
            ex.set_hparams(**hp)
        ex.run(1)
    h1 = time.perf_counter()
    torch.cuda.synchronize()
    h2 = time.perf_counter()
    leads = {}
    for label, h, ev in marks:
        g = h0 + ref.elapsed_time(ev) / 1e3  # when the GPU reached the point, on the host clock
        leads.setdefault(label, []).append((g - h) * 1e3)
    out = {"steps": a.steps, "trial_steps": a.trial_steps,
           "host_ms_per_step": round((h1 - h0) / a.steps * 1e3, 3),
           "gpu_ms_per_step": round((h2 - h0) / a.steps * 1e3, 3)}
    for label, v in leads.items():
        s = sorted(v[len(v) // 4:])  # skip the first quarter (the lead builds up)
        out[f"lead_ms_{label}"] = {"min": round(s[0], 3), "p50": round(s[len(s) // 2], 3), "max": round(s[-1], 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
