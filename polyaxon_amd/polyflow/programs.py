"""Trial programs for resident executors: what a warm worker builds once and then trains trial after trial.

A *program* is the trial-invariant part of an experiment -- model architecture, batch shape, data stream,
optimizer kind, the step (eager or captured as a hipGraph) -- and is named in the Polyaxonfile as
``environment.executor: {kind: resident, program: <name>, params: {...}}``.  Everything that varies between
trials (hyper-parameters, random init seed, Hyperband resource) is device data the executor rewrites in place
(polyflow/executor.py).  In the reference every trial is a pod running ``run.cmd`` from scratch
(polyaxon/scheduler/spawners/experiment_spawner.py:108-179); the program is what stays warm instead.

Registry: ``resnet50`` (BASELINE.json config 3), ``resnet_tiny`` (same code path, CPU-test sized), ``mlp``
(config 2), ``gpt2`` (config 4's GPT-2 125M trial), ``gpt2_tiny`` (same code path, CPU-test sized).  ``module:callable`` names any user factory with the same signature ``(params, device) -> TrialProgram``.
"""
from __future__ import annotations

import importlib
import math
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Optional, Tuple

# torch is imported inside the builders: the scheduler imports this module for program_key / bracket_units, and the
# scheduler process never loads torch or the HIP runtime (tests/test_gpu_free_scheduler.py)


@dataclass
class TrialProgram:
    executor: Any                     # ResidentTrialExecutor
    unit_steps: int = 1               # training steps per Hyperband / ASHA resource unit
    metric: str = "loss"              # the metric the executor commits (mean loss over the last `window` steps)
    window: int = 4
    hp_keys: Tuple[str, ...] = ()     # hyper-parameters the program understands
    info: Dict[str, Any] = field(default_factory=dict)

    def warm(self, steps: int = 2) -> None:
        """Pay one-time costs (kernel selection, allocator growth, library page-in) before the first trial."""
        import torch

        ex = self.executor
        if ex.use_graph:
            ex.capture(warmup=steps)
        else:
            ex.reset(seed=0)
            ex.set_hparams(**{k: v for k, v in self.info.get("warm_hparams", {}).items()})
            ex.run(steps)
            ex.snapshot("__warm__")
            ex.restore("__warm__")
            ex.drop("__warm__")
        if ex.is_cuda:
            torch.cuda.synchronize(ex.device)


def _resnet(params: Dict[str, Any], device, tiny: bool) -> TrialProgram:
    import torch

    from polyaxon_amd.models.resnet import resnet18ish, resnet50
    from polyaxon_amd.ops.synth import SyntheticImages
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    dev = torch.device(device)
    batch = int(params.get("batch", 8 if tiny else 256))
    image = int(params.get("image", 32 if tiny else 224))
    classes = int(params.get("classes", 10 if tiny else 1000))
    data = SyntheticImages(batch, image, dev, classes=classes,
                           active_classes=int(params.get("active_classes", min(classes, 100))),
                           grid=int(params.get("grid", 4 if tiny else 7)), signal=float(params.get("signal", 0.5)),
                           seed=int(params.get("data_seed", 0)))
    model = resnet18ish(num_classes=classes) if tiny else resnet50(num_classes=classes)
    ex = ResidentTrialExecutor(model, data, dev, optimizer="sgd", use_graph=bool(params.get("graph", False)))
    return TrialProgram(ex, unit_steps=int(params.get("unit_steps", 1 if tiny else 4)),
                        window=int(params.get("window", 4)), hp_keys=("lr", "momentum", "weight_decay", "nesterov"),
                        info={"model": "resnet18ish" if tiny else "resnet50", "batch": batch, "image": image,
                              "classes": classes, "data": "synthetic, fresh per step (ops/synth.py)",
                              "warm_hparams": {"lr": 0.01, "momentum": 0.9, "weight_decay": 1e-4},
                              "images_per_step": batch})


def _mlp(params: Dict[str, Any], device) -> TrialProgram:
    import torch

    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor
    from polyaxon_amd.trainers import MLP

    dev = torch.device(device)
    bs = int(params.get("batch", 256))
    g = torch.Generator().manual_seed(int(params.get("data_seed", 0)))
    x = torch.randn(bs, 784, generator=g)
    y = (x @ torch.randn(784, 10, generator=g)).argmax(1)
    ex = ResidentTrialExecutor(MLP(), (x, y), dev, optimizer="sgd", use_graph=dev.type == "cuda", channels_last=False)
    return TrialProgram(ex, unit_steps=int(params.get("unit_steps", 10)), window=int(params.get("window", 4)),
                        hp_keys=("lr", "momentum", "weight_decay"),
                        info={"model": "mlp", "batch": bs, "warm_hparams": {"lr": 0.01, "momentum": 0.9},
                              "images_per_step": bs})


def _gpt2(params: Dict[str, Any], device, tiny: bool) -> TrialProgram:
    import torch

    """GPT-2 125M (BASELINE.json config 4's trial) on the synthetic copy-task token stream (ops/synth.py
    SyntheticTokens): bf16 weights / gradients with an fp32 master and fused AdamW (the LM trainer's numerics),
    every trial re-initialised in place (GPT-2 init via plx_init_flat), AdamW hyper-parameters as device data."""
    from polyaxon_amd.models.transformer import Transformer, gpt2_125m, lm_loss
    from polyaxon_amd.ops.synth import SyntheticChain, SyntheticTokens
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    dev = torch.device(device)
    if tiny:
        cfg = gpt2_125m(vocab_size=int(params.get("vocab", 256)), n_layers=2, d_model=64, n_heads=2, d_ff=256,
                        max_seq_len=int(params.get("seq", 32)))
    else:
        cfg = gpt2_125m(vocab_size=int(params.get("vocab", 50257)))
    batch = int(params.get("batch", 2 if tiny else 16))
    seq = int(params.get("seq", 32 if tiny else 1024))
    task = str(params.get("task", "copy"))
    if task == "chain":  # a memorised transition table: learning-rate sensitive within ~100 steps
        data = SyntheticChain(batch, seq, cfg.vocab_size, dev, p=int(params.get("chain_p", 251 if tiny else 4093)),
                              seed=int(params.get("data_seed", 0)))
    else:
        data = SyntheticTokens(batch, seq, cfg.vocab_size, dev, period=int(params.get("period", 8 if tiny else 64)),
                               seed=int(params.get("data_seed", 0)), active_vocab=int(params.get("active_vocab", 0)))
    if dev.type == "cuda":
        with torch.device(dev):
            model = Transformer(cfg)
    else:
        model = Transformer(cfg)
    ex = ResidentTrialExecutor(model, data, dev, loss_fn=lm_loss, optimizer="adamw",
                               use_graph=bool(params.get("graph", False)), channels_last=False,
                               lp_dtype=torch.bfloat16)
    return TrialProgram(ex, unit_steps=int(params.get("unit_steps", 4 if tiny else 10)),
                        window=int(params.get("window", 4)),
                        hp_keys=("lr", "beta1", "beta2", "eps", "weight_decay"),
                        info={"model": "gpt2_tiny" if tiny else "gpt2_125m", "batch": batch, "seq": seq,
                              "vocab": cfg.vocab_size, "data": f"synthetic {task} task, fresh per step (ops/synth.py)",
                              "warm_hparams": {"lr": 3e-4, "beta1": 0.9, "beta2": 0.95, "eps": 1e-8,
                                               "weight_decay": 0.1},
                              "tokens_per_step": batch * seq, "floor_loss": data.floor_loss,
                              "unigram_loss": data.unigram_loss, "chance_loss": data.chance_loss,
                              "active_vocab": data.active_vocab})


PROGRAMS: Dict[str, Callable[[Dict[str, Any], Any], TrialProgram]] = {
    "gpt2": lambda p, d: _gpt2(p, d, tiny=False),
    "gpt2_tiny": lambda p, d: _gpt2(p, d, tiny=True),
    "resnet50": lambda p, d: _resnet(p, d, tiny=False),
    "resnet_tiny": lambda p, d: _resnet(p, d, tiny=True),
    "mlp": _mlp,
}


def resolve(name: str) -> Callable[[Dict[str, Any], Any], TrialProgram]:
    if name in PROGRAMS:
        return PROGRAMS[name]
    if ":" in name:
        mod, _, attr = name.partition(":")
        return getattr(importlib.import_module(mod), attr)
    raise KeyError(f"unknown resident program {name!r}; known: {sorted(PROGRAMS)} or module:callable")


def build_program(name: str, params: Optional[Dict[str, Any]], device) -> TrialProgram:
    prog = resolve(name)(dict(params or {}), device)
    if not isinstance(prog, TrialProgram):
        raise TypeError(f"program {name} returned {type(prog).__name__}, expected TrialProgram")
    return prog


def program_key(name: str, params: Optional[Dict[str, Any]]) -> str:
    """Executors are shared by every group whose program (name + build params) is identical."""
    import json

    return f"{name}:{json.dumps(params or {}, sort_keys=True)}"


def bracket_units(max_iter: float, eta: float, iteration: int, resume: bool) -> float:
    """Training resource (in units) one Hyperband bracket costs -- the load the pool balances across executors."""
    s_max = int(math.log(max_iter) / math.log(eta))
    s = s_max - iteration
    B = (s_max + 1) * max_iter
    n0 = int(math.ceil((B / max_iter) * (eta ** s) / (s + 1)))
    r = max_iter * eta ** (-s)
    total, prev, n, i = 0.0, 0.0, n0, 0
    while n > 0:
        ri = r * eta ** i
        total += n * ((ri - prev) if (resume and i) else ri)
        prev = ri
        # the reference's create_iteration: a bracket with a successor ends at rung s (should_reschedule); the last
        # bracket (s = 0) takes one more reduction, keep = int(n0 / eta) (the reference quirk), and none after it
        # (get_n_config_to_keep_for_iteration is 0 at rung s + 1)
        n = 0 if (i >= s and iteration < s_max) or i == s + 1 else int(n0 * (eta ** -i) / eta)
        i += 1
    return total


def asha_units(n_configs: int, min_r: float, max_r: float, eta: float, resume: bool) -> float:
    """Expected training resource (in units) of an ASHA shard over ``n_configs`` configs: rung k holds about
    n / eta^k configs, each training r_k (or r_k - r_{k-1} when resumed) -- the load the pool balances."""
    n_rungs = int(math.floor(math.log(max_r / min_r) / math.log(eta) + 1e-9)) + 1
    total, prev = 0.0, 0.0
    for k in range(n_rungs):
        rk = min(min_r * eta ** k, max_r)
        total += (n_configs / eta ** k) * ((rk - prev) if (resume and k) else rk)
        prev = rk
    return total
