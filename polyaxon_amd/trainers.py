"""Trial entry points for the BASELINE.json configs (run under polyflow; read hyper-parameters from
POLYAXON_DECLARATIONS / CLI flags, report metrics through the tracking client).

    python -m polyaxon_amd.trainers mlp     --lr 0.01 --bs 256 --steps 200          (config 2)
    python -m polyaxon_amd.trainers resnet  --lr 0.1 --steps 80                     (config 3, process mode)
    python -m polyaxon_amd.trainers lm --model gpt2_125m --steps 50                  (config 4, DP=N ranks)
    python -m polyaxon_amd.trainers lm --model llama3_8b --seq 4096 --bs 1 --zero1   (config 5, DP=8)

Every trainer: flat fp32 master weights + fused HIP optimizer, bf16 autocast, synthetic data of the real
shape, metrics streamed from the GPU (tracking client MetricStream), DP through FlatDDP (RCCL) when
WORLD_SIZE > 1, rank 0 reports.  ``--ckpt`` saves/loads ``model.pt`` under POLYAXON_RUN_OUTPUTS_PATH so
Hyperband RESUME promotions continue training.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


def _declared(args: argparse.Namespace) -> argparse.Namespace:
    decl = json.loads(os.environ.get("POLYAXON_DECLARATIONS", "{}") or "{}")
    for k, v in decl.items():
        k = k.replace("-", "_")
        if hasattr(args, k) and getattr(args, k) == args._defaults.get(k):
            setattr(args, k, type(args._defaults[k])(v) if args._defaults.get(k) is not None else v)
    return args


def _parser(name: str) -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog=f"polyaxon_amd.trainers {name}")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--weight_decay", type=float, default=0.0)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--bs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--log_every", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--ckpt", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    return ap


def _parse(ap: argparse.ArgumentParser, argv):
    args = ap.parse_args(argv)
    args._defaults = {a.dest: a.default for a in ap._actions}
    return _declared(args)


def _device(args):
    if args.cpu or not torch.cuda.is_available() or os.environ.get("PLX_CPU_ONLY") == "1":
        return torch.device("cpu")
    from polyaxon_amd.client.budget import apply_hbm_budget

    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) if torch.cuda.device_count() > 1 else 0)
    apply_hbm_budget(dev)  # the replica's HBM reservation (PLX_HBM_GB / PLX_HBM_FRACTION from polyflow)
    return dev


def _tracker():
    from polyaxon_amd.client import Experiment

    return Experiment() if (os.environ.get("POLYAXON_EXPERIMENT_ID") or os.environ.get("POLYAXON_STORE_PATH")) \
        else None


def _ckpt_path():
    out = os.environ.get("POLYAXON_RUN_OUTPUTS_PATH")
    return os.path.join(out, "model.pt") if out else None


# ------------------------------------------------------------------ config 2: 2-layer MLP
class MLP(nn.Module):
    def __init__(self, d_in=784, hidden=1024, classes=10):
        super().__init__()
        self.fc1 = nn.Linear(d_in, hidden)
        self.fc2 = nn.Linear(hidden, classes)

    def forward(self, x):
        return self.fc2(F.relu(self.fc1(x)))

    def init_spec(self):
        return [(self.fc1.weight, "uniform", 1 / math.sqrt(self.fc1.in_features)),
                (self.fc1.bias, "const", 0.0),
                (self.fc2.weight, "uniform", 1 / math.sqrt(self.fc2.in_features)),
                (self.fc2.bias, "const", 0.0)]


def train_mlp(argv=None) -> float:
    """Grid-search lr x bs over a 2-layer MLP; the whole step is a replayed hipGraph (launch-bound model)."""
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    args = _parse(_parser("mlp"), argv)
    dev = _device(args)
    g = torch.Generator().manual_seed(args.seed)
    x = torch.randn(args.bs, 784, generator=g)
    w_true = torch.randn(784, 10, generator=g)
    y = (x @ w_true).argmax(1)
    ex = ResidentTrialExecutor(MLP(), (x, y), dev, optimizer="sgd", use_graph=dev.type == "cuda",
                               channels_last=False)
    ex.capture(warmup=2)
    ex.reset(seed=args.seed)
    ex.set_hparams(lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    xp = _tracker()
    steps_done = 0
    while steps_done < args.steps:
        n = min(args.log_every, args.steps - steps_done)
        ex.run(n)
        steps_done += n
        if xp is not None:  # GPU tensor -> pinned side-stream copy, no sync on the training stream
            xp.log_metrics(step=steps_done, loss=ex.ring[(int(steps_done) - 1) % ex.ring_size])
    loss = float(ex.losses()[-1])
    if xp is not None:
        xp.log_metrics(step=steps_done, loss=loss)
        xp.close()
    print(json.dumps({"loss": loss, "steps": steps_done}))
    return loss


# ------------------------------------------------------------------ config 3 (process mode): ResNet-50 trial
def train_resnet(argv=None) -> float:
    from polyaxon_amd.models.resnet import resnet50
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    ap = _parser("resnet")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--units", type=int, default=1)
    ap.add_argument("--unit_steps", type=int, default=8)
    args = _parse(ap, argv)
    dev = _device(args)
    g = torch.Generator().manual_seed(args.seed)
    x = torch.randn(args.bs, 3, args.image, args.image, generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.bs,), generator=g)
    ex = ResidentTrialExecutor(resnet50(), (x, y), dev, use_graph=False)
    ckpt = _ckpt_path() if args.ckpt else None
    done_units = 0
    ex.reset(seed=args.seed)
    if ckpt and os.path.exists(ckpt):  # Hyperband RESUME: continue from the previous rung
        st = torch.load(ckpt, map_location=dev, weights_only=True)
        ex.flat.params.copy_(st["params"])
        ex.opt.momentum_buf.copy_(st["momentum"])
        ex.buffers.copy_(st["buffers"])
        ex.step.fill_(int(st["step"]))
        done_units = int(st["units"])
    ex.set_hparams(lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    ex.run(max(0, args.units - done_units) * args.unit_steps)
    out = torch.full((1,), float("nan"), device=dev)
    ex.commit(out, 0, window=4)
    loss = float(out[0])
    if ckpt:
        torch.save({"params": ex.flat.params, "momentum": ex.opt.momentum_buf, "buffers": ex.buffers,
                    "step": int(ex.step.item()), "units": args.units}, ckpt)
    xp = _tracker()
    if xp is not None:
        xp.log_metrics(step=int(ex.step.item()), loss=loss)
        xp.close()
    print(json.dumps({"loss": loss, "units": args.units}))
    return loss


# ------------------------------------------------------------------ configs 4 & 5: language models, DP over RCCL
def train_lm(argv=None) -> float:
    from polyaxon_amd.models.transformer import Transformer, gpt2_125m, llama3_8b, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW
    from polyaxon_amd.parallel.ddp import FlatDDP, MetricReducer, init_from_env

    ap = _parser("lm")
    ap.add_argument("--model", default="gpt2_125m", choices=["gpt2_125m", "llama3_8b", "tiny"])
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--warmup_steps", type=int, default=0)
    ap.add_argument("--bucket_mb", type=lambda v: v if v == "auto" else float(v), default="auto",
                    help="gradient bucket size in MB, or 'auto': planned for the world size over xGMI "
                         "(parallel/comm_plan.py)")
    ap.add_argument("--checkpoint_activations", action="store_true")
    ap.add_argument("--beta2", type=float, default=0.95)
    ap.add_argument("--fp32_weights", action="store_true",
                    help="model computes from fp32 weights under autocast (default on GPU: bf16 weights/grads with "
                         "an fp32 master copy in the optimizer)")
    ap.add_argument("--fixed_batch", action="store_true", help="reuse one synthetic batch every step")
    ap.add_argument("--data", choices=["random", "copy"], default="random",
                    help="synthetic tokens: uniform random (loss stays ln V), or the copy task of the resident GPT-2 "
                         "program (ops/synth.py SyntheticTokens: learnable, hyper-parameter sensitive)")
    ap.add_argument("--period", type=int, default=64, help="copy task: phrase length (seq must be a multiple)")
    ap.add_argument("--world1_collectives", nargs="?", const="all", default="", choices=["", "all", "metric"],
                    help="world 1 on the GPU: still create the gloo rendezvous and the trial's RCCL communicator (metric "
                         "mean); 'all' (the bare flag) also runs every gradient bucket's collective on it (the DP path's "
                         "overheads measured on one GPU)")
    ap.add_argument("--zero1", action="store_true",
                    help="ZeRO-1: reduce-scatter each gradient bucket, AdamW on this rank's 1/W slice inside the "
                         "backward, all-gather the bf16 weights (parallel/ddp.py); also PLX_ZERO1=1")
    args = _parse(ap, argv)
    # the process group is the gloo rendezvous; every device collective of the trial (gradient buckets, ZeRO-1,
    # the parameter broadcast, the metric mean) runs on ONE framework RCCL communicator (parallel/comm.py)
    cuda = not args.cpu and torch.cuda.is_available()
    info = init_from_env("gloo", device=torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0"))) if cuda
                         else torch.device("cpu"))
    dev = info["device"]
    force = bool(args.world1_collectives) and dev.type == "cuda" and info["world"] == 1
    force_buckets = force and args.world1_collectives == "all"
    if force:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        dist.init_process_group("gloo", rank=0, world_size=1)
    if dev.type == "cuda":
        from polyaxon_amd.client.budget import apply_hbm_budget

        apply_hbm_budget(dev)
    cfg = {"gpt2_125m": gpt2_125m, "llama3_8b": llama3_8b, "tiny": tiny_llama}[args.model](
        checkpoint=args.checkpoint_activations)
    seq = min(args.seq, cfg.max_seq_len)
    torch.manual_seed(args.seed)
    model = Transformer(cfg) if dev.type == "cpu" else _build_on_device(Transformer, cfg, dev)
    lp = torch.bfloat16 if (dev.type == "cuda" and not args.fp32_weights) else None
    flat = FlatParams(model, dev, channels_last=False, lp_dtype=lp)
    if lp is not None:
        flat.enable_direct_grads(True)  # weight-gradient GEMMs write into the flat bf16 grads (ops/lm.py)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    opt = FusedAdamW(flat, lr=args.lr, betas=(0.9, args.beta2), weight_decay=args.weight_decay, step_counter=step)
    # PLX_OPT_IN_BACKWARD=1: the AdamW update of each gradient bucket runs inside the backward as the bucket completes
    # (parallel/ddp.py).  Off by default: bitwise the same trajectory, but on one MI355X the HBM-bound update only
    # moved time from itself to the backward's memory-bound kernels (Llama-3 8B 18.17k vs 18.03k tokens/s with a
    # full-chip grid, slower with a capped one; profiles/r3_negative_results.md)
    zero1 = args.zero1 or os.environ.get("PLX_ZERO1", "0") == "1"
    in_bwd = zero1 or (dev.type == "cuda" and os.environ.get("PLX_OPT_IN_BACKWARD", "0") == "1")
    ddp = FlatDDP(flat, bucket_mb=args.bucket_mb, optimizer=opt if in_bwd else None, shard_optimizer=zero1,
                  force_collectives=force_buckets)
    ddp.broadcast_params()
    metrics = MetricReducer(dev, force_comm=force)  # cross-rank mean of the logged loss (RCCL communicator, GPU)
    g = torch.Generator(device=dev).manual_seed(args.seed + 1000 * info["rank"])

    def batch():  # synthetic tokens drawn on the device: a fresh batch per step costs one tiny kernel
        return torch.randint(0, cfg.vocab_size, (args.bs, seq), generator=g, device=dev)

    if args.data == "copy":
        from polyaxon_amd.ops.synth import SyntheticTokens

        src = SyntheticTokens(args.bs, seq, cfg.vocab_size, dev, period=args.period,
                              seed=args.seed + 1000 * info["rank"])

        def batch():  # noqa: F811 -- the copy task, refilled in place on the device
            src.next()
            return src.x

    tokens = batch()
    xp = _tracker() if info["rank"] == 0 else None
    amp = dev.type == "cuda"
    t0 = time.time()
    loss_val = float("nan")
    skip = 2 if args.steps > 4 else 0  # exclude allocator / kernel-selection warmup from tokens/s
    for it in range(args.steps):
        if it == skip and skip:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t0 = time.time()
        lr = args.lr * min(1.0, (it + 1) / args.warmup_steps) if args.warmup_steps else args.lr
        opt.set_hparams(lr=lr)
        if it and not args.fixed_batch:
            tokens = batch()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            loss = lm_loss(model(tokens), tokens)
        loss.backward()
        ddp.finish()
        opt.step_()
        step += 1
        if (it + 1) % args.log_every == 0 or it == args.steps - 1:
            loss_mean = metrics.mean(loss)  # every rank joins the collective; rank 0 logs it
            if xp is not None and (it + 1) % args.log_every == 0:
                xp.log_metrics(step=it + 1, loss=loss_mean[0])
            if it == args.steps - 1:
                loss_val = float(loss_mean[0])
    t_host = time.time() - t0  # the host has queued every step (a host time ~ dt: the GPU waited for launches)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = time.time() - t0
    tok_s = (args.steps - skip) * args.bs * seq * info["world"] / dt
    if xp is not None:
        xp.log_metrics(step=args.steps, loss=loss_val, tokens_per_s=tok_s)
        xp.close()
    if info["rank"] == 0:
        from polyaxon_amd.ops import gemm as _gemm

        dec = _gemm.decisions()
        print(json.dumps({"loss": loss_val, "tokens_per_s": round(tok_s, 1), "world": info["world"],
                          "ms_per_step": round(dt / max(1, args.steps - skip) * 1e3, 3),
                          "host_ms_per_step": round(t_host / max(1, args.steps - skip) * 1e3, 3),
                          "world1_collectives": args.world1_collectives if force else "", "zero1": zero1, "bucket_launches": ddp.launched,
                          "buckets": len(ddp.buckets), "bucket_plan": ddp.plan,
                          "params_m": round(sum(s.numel for s in flat.segments) / 1e6, 1),
                          "lm_gemm": {"mode": _gemm.mode(), "native_shapes": sum(1 for d in dec.values() if d["native"]),
                                      "shapes": len(dec), "decisions": dec}}))
    ddp.close()
    metrics.close()
    if info["world"] > 1 or force:
        import torch.distributed as dist

        dist.destroy_process_group()
    return loss_val


def _build_on_device(cls, cfg, dev):
    with torch.device(dev):
        return cls(cfg)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    which, rest = argv[0], argv[1:]
    {"mlp": train_mlp, "resnet": train_resnet, "lm": train_lm}[which](rest)
    return 0


if __name__ == "__main__":
    sys.exit(main())
