"""Hyperband sweep driven on a resident trial executor (the north-star workload's inner loop).

This is the reference's Hyperband task chain — ``hp_hyperband_create → start → iterate → reduce``
(polyaxon/hpsearch/tasks/hyperband.py:7-83) — collapsed into one event-driven loop on
the GPU that owns the trials:

* suggestions come from :class:`HyperbandSearchManager` (reference-exact bracket arithmetic);
* each experiment (a config at one rung) is a trial on the warm executor, with no poll interval, no
  task hop and no pod start between trials;
* rung metrics are reduced on the device into a ``BracketMetrics`` tensor and the promotion decision is
  the ``plx_topk_brackets`` kernel (the reference sorts rows pulled from Postgres);
* promotions with ``resume: true`` restore the HBM snapshot and train only the additional resource
  (reference RESUME cloning strategy, db/models/experiments.py:225-316), otherwise they restart.

Trial end times are recorded with device events so wall-clock-to-target can be computed after the run
without inserting host synchronisations into the trial stream.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

from polyaxon_amd.obs.tracing import trace_range
from polyaxon_amd.polytune.kernels import BracketMetrics
from polyaxon_amd.polytune.managers import HyperbandIterationConfig, HyperbandSearchManager


@dataclass
class TrialRecord:
    trial: int
    config_id: int
    iteration: int
    bracket_iteration: int
    resource: float
    steps: int
    params: Dict
    end_event: Optional[object] = None
    slot: int = 0
    metric: Optional[float] = None


@dataclass
class SweepResult:
    trials: List[TrialRecord] = field(default_factory=list)
    best_metric: Optional[float] = None
    best_params: Optional[Dict] = None


class HyperbandSweep:
    def __init__(self, manager: HyperbandSearchManager, executor, unit_steps: int, hp_keys=None,
                 seed: int = 0, metric_window: int = 4, on_trial_end: Optional[Callable] = None):
        self.manager = manager
        self.ex = executor
        self.unit_steps = unit_steps
        self.hp_keys = hp_keys
        self.seed = seed
        self.window = metric_window
        self.on_trial_end = on_trial_end
        self.resume = manager.hptuning_config.hyperband.resume
        self.resource_name = manager.hptuning_config.hyperband.resource.name
        self.maximize = manager.hptuning_config.hyperband.metric.optimization == "maximize"
        max_configs = max(manager.get_n_configs(manager.get_bracket(i)) for i in range(manager.s_max + 1))
        self.metrics = BracketMetrics(1, max_configs, executor.device)
        self.result = SweepResult()
        self._trial = 0
        self._events = executor.is_cuda

    def _event(self):
        if not self._events:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def _run_trial(self, it: HyperbandIterationConfig, cid: int, params: Dict, slot: int,
                   prev_resource: Optional[float]) -> TrialRecord:
        with trace_range(f"trial {self._trial} it{it.iteration}.{it.bracket_iteration} cfg{cid}"):
            return self._run_trial_inner(it, cid, params, slot, prev_resource)

    def _run_trial_inner(self, it, cid, params, slot, prev_resource) -> TrialRecord:
        r = params[self.resource_name]
        if self.resume and prev_resource is not None:
            self.ex.restore(cid)
            steps = int(round((r - prev_resource) * self.unit_steps))
        else:
            self.ex.reset(seed=self.seed * 100003 + cid)
            steps = int(round(r * self.unit_steps))
        hp = {k: v for k, v in params.items() if k != self.resource_name}
        self.ex.set_hparams(**hp)
        self.ex.run(steps)
        self.ex.commit(self.metrics.values[0], slot, self.window)
        more = self.manager.get_n_config_to_keep_for_iteration(it.iteration, it.bracket_iteration) > 0
        if self.resume and more:
            self.ex.snapshot(cid)
        rec = TrialRecord(self._trial, cid, it.iteration, it.bracket_iteration, r, steps, params, self._event(), slot)
        self._trial += 1
        self.result.trials.append(rec)
        if self.on_trial_end is not None:
            self.on_trial_end(rec)
        return rec

    def run(self, max_trials: Optional[int] = None) -> SweepResult:
        """Run the full Hyperband schedule (or stop after ``max_trials`` experiments)."""
        m = self.manager
        it = m.next_iteration(None)
        configs: Dict[int, Dict] = {}
        active: List[int] = []
        prev_r: Dict[int, float] = {}
        next_cid = 0
        while True:
            if it.bracket_iteration == 0:
                for cid in active:
                    self.ex.drop(cid)
                sugg = m.get_suggestions(it)
                active = []
                for s in sugg:
                    configs[next_cid] = s
                    active.append(next_cid)
                    next_cid += 1
                prev_r = {}
            else:
                r = m.hptuning_config.hyperband.resource.cast_value(
                    m.get_n_resources_for_iteration(it.iteration, it.bracket_iteration))
                for cid in active:
                    configs[cid] = dict(configs[cid], **{self.resource_name: r})
            self.metrics.reset_bracket(0, len(active))
            it.experiment_ids = list(active)
            rung: List[TrialRecord] = []
            for slot, cid in enumerate(active):
                rung.append(self._run_trial(it, cid, configs[cid], slot, prev_r.get(cid)))
                if max_trials is not None and self._trial >= max_trials:
                    return self.result
            # rung decision on the device: one top-k launch, one small D2H read
            order = self.metrics.order(self.maximize)[0].cpu().tolist()
            vals = self.metrics.values[0, : len(active)].cpu().tolist()
            it.experiments_metrics = [(cid, vals[i]) for i, cid in enumerate(active) if not math.isnan(vals[i])]
            for rec in rung:
                rec.metric = vals[rec.slot]
            self._update_best(active, vals, configs)
            if m.is_done(it):
                break
            nxt = m.next_iteration(it)
            if nxt.iteration == it.iteration:  # reduce: promote top-k (device order, NaN last)
                keep = m.get_n_config_to_keep_for_iteration(it.iteration, it.bracket_iteration)
                ranked = [active[i] for i in order if i >= 0 and not math.isnan(vals[i])]
                promoted = ranked[:keep]
                for cid in active:
                    if cid not in promoted:
                        self.ex.drop(cid)
                prev_r = {cid: configs[cid][self.resource_name] for cid in promoted}
                active = promoted
            it = nxt
        return self.result

    def _update_best(self, active, vals, configs) -> None:
        for i, cid in enumerate(active):
            v = vals[i]
            if math.isnan(v):
                continue
            b = self.result.best_metric
            if b is None or (v > b if self.maximize else v < b):
                self.result.best_metric = v
                self.result.best_params = configs[cid]
