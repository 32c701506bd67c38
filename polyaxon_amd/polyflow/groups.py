"""Experiment-group drivers: grid, random, Hyperband (synchronous, reference-exact), BO, ASHA.

Reference: polyaxon/hpsearch/tasks/{base,grid,random,hyperband,bo}.py and iteration_managers/*.py — a
chain of Celery tasks that create experiments, start them up to ``concurrency`` and then *poll* every 30 s
(``self.retry(countdown=Intervals.EXPERIMENTS_SCHEDULER)``) until the iteration is done.  Here each group
is a driver object living on the polyflow thread; ``on_experiment_done`` is called the moment a trial
finishes, so the next trial is enqueued in the same loop iteration (no poll interval, no task hop).

Semantics kept from the reference:
* all grid/random experiments are created up front (status ``created``) and started ≤ concurrency;
* Hyperband iterations/brackets/rungs and promotions follow HyperbandSearchManager exactly; promoted
  configs become new experiments cloned with RESUME (``hyperband.resume: true``) or RESTART, with the
  resource declaration patched (iteration_managers/hyperband.py:79-113);
* BO proposes ``n_initial_trials`` random configs, then one suggestion per iteration (``n_suggestions``
  > 1 is the batch extension) until ``n_iterations``;
* early stopping checks every rule against ``last_metric`` and stops the *pending* experiments
  (hpsearch/tasks/base.py:36-42; ``early_stopping_stop_running: true`` in ``settings`` extends it to
  running ones);
* the group is RUNNING while it has work and SUCCEEDED when everything is done (FAILED if nothing
  succeeded is not a reference behaviour — a group with failed trials still succeeds).
"""
from __future__ import annotations

import logging
import math
from typing import Any, Dict, List, Optional

from polyaxon_amd.fsm import ExperimentLifeCycle
from polyaxon_amd.polytune.managers import (AshaSearchManager, HyperbandIterationConfig, HyperbandSearchManager,
                                            get_search_algorithm_manager)
from polyaxon_amd.spec.hptuning import Optimization, SearchAlgorithms
from polyaxon_amd.spec.specification import GroupSpecification

log = logging.getLogger("polyaxon_amd.groups")


class GroupDriver:
    def __init__(self, flow, gid: int, spec: GroupSpecification, project: Dict, user: str, cwd: str):
        self.flow = flow
        self.store = flow.store
        self.gid = gid
        self.spec = spec
        self.project = project
        self.user = user
        self.cwd = cwd
        self.hp = spec.hptuning
        self.manager = get_search_algorithm_manager(self.hp)
        self.concurrency = max(1, self.hp.concurrency)
        self.queue: List[int] = []        # created, not yet started (in order)
        self.active: set = set()          # started, not done
        self.finished: Dict[int, str] = {}
        self.done = False
        self.stopped = False
        settings = spec.raw_data.get("settings") or {}
        self.stop_running_on_early_stop = bool(settings.get("early_stopping_stop_running", False))

    # ------------------------------------------------------------------ helpers
    def create_experiment(self, params: Dict[str, Any], enqueue: bool = False, original_id: Optional[int] = None,
                          strategy: Optional[str] = None) -> int:
        if original_id is not None:
            return self.flow._clone(original_id, strategy, params, None, group_id=self.gid)
        xspec = self.spec.get_experiment_spec(params)
        return self.flow._create_experiment(xspec, self.project, self.user, self.cwd, group_id=self.gid,
                                            enqueue=enqueue)

    def _start_more(self) -> None:
        while self.queue and len(self.active) < self.concurrency and not self.stopped:
            xid = self.queue.pop(0)
            run = self.flow.runs.get(f"experiment:{xid}")
            if run is None or run.final_status is not None:
                continue
            self.active.add(xid)
            self.flow._enqueue(run)

    def start(self) -> None:
        self.store.set_group_status(self.gid, "running")
        self.flow.auditor.record(f"experiment_group.{self.hp.search_algorithm.replace('_search', '')}",
                                 "experiment_group", self.gid)
        self.begin()
        self._start_more()
        self._check_finished()

    def begin(self) -> None:
        raise NotImplementedError

    def on_experiment_done(self, xid: int, status: str) -> None:
        self.active.discard(xid)
        self.finished[xid] = status
        if self.done:
            return
        if self.stopped:  # teardown in progress (stop() itself finishes pending trials)
            self._check_finished()
            return
        if self._should_stop_early():
            self.flow.auditor.record("experiment_group.stopped", "experiment_group", self.gid, reason="early_stopping")
            self.stop(pending_only=not self.stop_running_on_early_stop, message="Early stopping")
            return
        self.advance(xid, status)
        self._start_more()
        self._check_finished()

    def advance(self, xid: int, status: str) -> None:
        """Algorithm-specific reaction to a finished trial (may create/queue more experiments)."""

    def has_more_work(self) -> bool:
        return False

    def _check_finished(self) -> None:
        if self.done or self.queue or self.active or self.has_more_work():
            return
        self.done = True
        status = "stopped" if self.stopped else "succeeded"
        if self.store.get_group(self.gid)["status"] != "stopped":
            self.store.set_group_status(self.gid, status)
        self.flow.auditor.record(f"experiment_group.{'done' if status == 'stopped' else 'succeeded'}",
                                 "experiment_group", self.gid)

    def _should_stop_early(self) -> bool:
        rules = self.hp.early_stopping
        if not rules:
            return False
        xps = self.store.list_experiments(group_id=self.gid)
        for r in rules:
            for x in xps:
                v = (x.get("last_metric") or {}).get(r.metric)
                if v is None:
                    continue
                if (Optimization.maximize(r.optimization) and v >= r.value) or (
                        Optimization.minimize(r.optimization) and v <= r.value):
                    return True
        return False

    def stop(self, pending_only: bool = False, message: str = "Stopped") -> None:
        self.stopped = True
        for xid in list(self.queue):
            run = self.flow.runs.get(f"experiment:{xid}")
            if run is not None:
                self.flow._finish_unstarted(run, "stopped", message)
        self.queue.clear()
        for xid in list(self.active):
            run = self.flow.runs.get(f"experiment:{xid}")
            if run is None:
                continue
            if not run.replicas:  # queued in polyflow but not placed yet: pending
                self.flow._finish_unstarted(run, "stopped", message)
            elif not pending_only:
                self.flow._stop("experiment", xid, message)
        if pending_only:
            self.active = {x for x in self.active
                           if self.flow.runs.get(f"experiment:{x}") and self.flow.runs[f"experiment:{x}"].active}
        if not self.store.get_group(self.gid)["status"] in ("stopped", "succeeded", "failed"):
            self.store.set_group_status(self.gid, "stopped", message)
        self._check_finished()

    def metric_of(self, xid: int, name: str) -> Optional[float]:
        x = self.store.get_experiment(xid)
        v = (x.get("last_metric") or {}).get(name)
        return None if v is None else float(v)


class GridRandomDriver(GroupDriver):
    def begin(self) -> None:
        for params in self.manager.get_suggestions():
            self.queue.append(self.create_experiment(params))


class HyperbandDriver(GroupDriver):
    """Synchronous rung barrier per bracket, exactly like the reference — but event-driven."""

    def begin(self) -> None:
        self.m: HyperbandSearchManager = self.manager
        self.it = self.m.next_iteration(None)
        self.iteration_id: Optional[int] = None
        self._launch_iteration(self.m.get_suggestions(self.it), None)

    def _launch_iteration(self, params_list: List[Dict], originals: Optional[List[int]]) -> None:
        ids = []
        strategy = "resume" if self.hp.hyperband.resume else "restart"
        for i, params in enumerate(params_list):
            if originals is None:
                ids.append(self.create_experiment(params))
            else:
                ids.append(self.create_experiment(params, original_id=originals[i], strategy=strategy))
        self.it.experiment_ids = ids
        self.iteration_id = self.store.create_iteration(self.gid, self.it.to_dict())
        self.queue.extend(ids)

    def advance(self, xid: int, status: str) -> None:
        if any(x not in self.finished for x in self.it.experiment_ids):
            return  # rung barrier: wait for the whole iteration
        metric = self.hp.hyperband.metric.name
        self.it.experiments_metrics = [(x, v) for x, v in ((x, self.metric_of(x, metric))
                                                           for x in self.it.experiment_ids) if v is not None]
        self.store.update_iteration(self.iteration_id, self.it.to_dict())
        if self.m.is_done(self.it):
            return
        nxt = self.m.next_iteration(self.it)
        if nxt.iteration == self.it.iteration:  # reduce: promote the top-k
            keep_ids = self.m.reduce(self.it)
            r = self.hp.hyperband.resource.cast_value(
                self.m.get_n_resources_for_iteration(nxt.iteration, nxt.bracket_iteration))
            params = []
            for x in keep_ids:
                decl = dict(self.store.get_experiment(x)["declarations"])
                decl[self.hp.hyperband.resource.name] = r
                params.append(decl)
            self.it = nxt
            self._launch_iteration(params, keep_ids)
        else:
            self.it = nxt
            self._launch_iteration(self.m.get_suggestions(self.it), None)


class BODriver(GroupDriver):
    def begin(self) -> None:
        from polyaxon_amd.polytune.bo import BOIterationConfig

        self.iteration = 0
        self.old_configs: List = []
        self.old_metrics: List = []
        self.cur_ids: List[int] = []
        self.BOIterationConfig = BOIterationConfig
        for params in self.manager.get_suggestions(None):
            xid = self.create_experiment(params)
            self.cur_ids.append(xid)
            self.queue.append(xid)
        self.iteration_id = self.store.create_iteration(self.gid, {"iteration": 0, "experiment_ids": self.cur_ids})

    def has_more_work(self) -> bool:
        return self.manager.should_reschedule(self.iteration) and not self.stopped and bool(self.cur_ids) and False

    def advance(self, xid: int, status: str) -> None:
        if any(x not in self.finished for x in self.cur_ids):
            return
        metric = self.hp.bo.metric.name
        for x in self.cur_ids:
            v = self.metric_of(x, metric)
            if v is not None:
                self.old_configs.append((x, dict(self.store.get_experiment(x)["declarations"])))
                self.old_metrics.append((x, v))
        self.store.update_iteration(self.iteration_id, {"iteration": self.iteration, "experiment_ids": self.cur_ids,
                                                        "experiments_metrics": [list(m) for m in self.old_metrics]})
        if not self.manager.should_reschedule(self.iteration) or not self.old_metrics:
            self.cur_ids = []
            return
        self.iteration += 1
        cfg = self.BOIterationConfig(iteration=self.iteration, old_experiments_configs=list(self.old_configs),
                                     old_experiments_metrics=list(self.old_metrics))
        suggestions = self.manager.get_suggestions(cfg) or []
        self.cur_ids = []
        for params in suggestions:
            xid = self.create_experiment(params)
            self.cur_ids.append(xid)
            self.queue.append(xid)
        self.iteration_id = self.store.create_iteration(self.gid, {"iteration": self.iteration,
                                                                   "experiment_ids": self.cur_ids})


class AshaDriver(GroupDriver):
    """Asynchronous successive halving: no rung barrier; a free slot immediately gets a promotion or a new
    config (the reference has no ASHA — hpsearch/tasks/hyperband.py:57-60)."""

    def begin(self) -> None:
        self.m: AshaSearchManager = self.manager
        self.xp_info: Dict[int, tuple] = {}
        self._fill()

    def _fill(self) -> None:
        while len(self.active) + len(self.queue) < self.concurrency and not self.stopped:
            job = self.m.next_job()
            if job is None:
                return
            cid, rung, params = job
            prev = self.m.__dict__.setdefault("_last_xp", {}).get(cid)
            if rung > 0 and prev is not None and self.hp.asha.resume:
                xid = self.create_experiment(params, original_id=prev, strategy="resume")
            else:
                xid = self.create_experiment(params)
            self.m._last_xp[cid] = xid
            self.xp_info[xid] = (cid, rung)
            self.queue.append(xid)

    def has_more_work(self) -> bool:
        return not self.stopped and (bool(self.m._pending) or self._promotable())

    def _promotable(self) -> bool:
        for rung in range(self.m.n_rungs - 1):
            if any(c not in self.m.promoted[rung] for c in self.m._top(rung)):
                return True
        return False

    def advance(self, xid: int, status: str) -> None:
        cid, rung = self.xp_info[xid]
        v = self.metric_of(xid, self.hp.asha.metric.name)
        if v is not None and status == "succeeded":
            self.m.report(cid, rung, v)
        self._fill()


def make_group_driver(flow, gid: int, spec: GroupSpecification, project: Dict, user: str, cwd: str) -> GroupDriver:
    algo = spec.search_algorithm
    cls = {SearchAlgorithms.GRID: GridRandomDriver, SearchAlgorithms.RANDOM: GridRandomDriver,
           SearchAlgorithms.HYPERBAND: HyperbandDriver, SearchAlgorithms.BO: BODriver,
           SearchAlgorithms.ASHA: AshaDriver}[algo]
    return cls(flow, gid, spec, project, user, cwd)
