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

import json
import logging
import math
import time
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
        """Reference ExperimentGroup.should_stop_early (db/models/experiment_groups.py:211-221): any experiment whose
        ``last_metric`` crosses any rule.  The group's metrics are pulled in one query into an [experiments x
        metrics] matrix and every rule is evaluated in one ``early_stop_any`` call (HIP kernel for device tensors,
        the same vectorised reduction on the host otherwise)."""
        rules = self.hp.early_stopping
        if not rules:
            return False
        import numpy as np
        import torch

        from polyaxon_amd.polytune.kernels import early_stop_any

        names = sorted({r.metric for r in rules})
        rows = self.store.execute("SELECT last_metric FROM experiments WHERE group_id = ?", (self.gid,)).fetchall()
        mat = np.full((max(len(rows), 1), len(names)), np.nan, dtype=np.float32)
        for i, r in enumerate(rows):
            last = json.loads(r["last_metric"] or "{}")
            for j, n in enumerate(names):
                v = last.get(n)
                if isinstance(v, (int, float)):
                    mat[i, j] = v
        flags = early_stop_any(torch.from_numpy(mat), [(names.index(r.metric), float(r.value),
                                                        Optimization.maximize(r.optimization)) for r in rules])
        return any(flags)

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


class ResidentHyperbandDriver(GroupDriver):
    """Hyperband on resident executors (``environment.executor: resident``; polyflow/resident.py, pool.py).

    The reference runs the brackets one after another with a synchronous rung barrier and a 30 s poll
    (polyaxon/hpsearch/tasks/hyperband.py:7-83), every trial a pod.  Here all ``s_max + 1`` brackets are created
    up front (same suggestions as the reference: ``get_suggestions`` per iteration, same seed) and handed to the
    group's executors -- at most ``concurrency`` of them, balanced by training units -- which run them
    concurrently; each executor decides its rungs on the device.  This driver mirrors what the executors report
    into the store, so every trial is an experiment row with its FSM history, metrics and ``last_metric``;
    promotions are RESUME (or RESTART) clones of the previous rung's experiment with the resource declaration
    patched (iteration_managers/hyperband.py:79-113); every finished rung is an iteration row.
    """

    def begin(self) -> None:
        from polyaxon_amd.polyflow.programs import bracket_units, program_key

        self.m: HyperbandSearchManager = self.manager
        self.hb = self.hp.hyperband
        self.ex = self.spec.environment.executor
        self.program_key = program_key(self.ex.program, self.ex.params)
        res = self.spec.environment.resources
        g = res.gpu.value if (res is not None and res.gpu is not None) else 1.0
        self.gpu = g if g > 0 else 1.0
        if self.gpu > 1:
            raise ValueError("a resident executor runs on one device (resources.gpu <= 1)")
        self.hbm = res.hbm_gb if res is not None else 0.0
        self.brackets: Dict[str, Dict[str, Any]] = {}
        self.pending_keys: List[str] = []
        self.used_workers: set = set()
        self._xspec_cache: Dict[str, Any] = {}
        rname = self.hb.resource.name
        for it in range(self.m.s_max + 1):
            sugg = self.m.get_suggestions(HyperbandIterationConfig(iteration=it))
            key = f"{self.gid}.{it}"
            configs = [{"cid": i, "params": {k: v for k, v in s.items() if k != rname}} for i, s in enumerate(sugg)]
            self.brackets[key] = {"iteration": it, "configs": configs, "status": None, "wid": None, "xids": {},
                                  "root": {}, "open": set(),
                                  "units": bracket_units(self.hb.max_iter, self.hb.eta, it, self.hb.resume)}
            self.pending_keys.append(key)
        self._dispatch()

    # ------------------------------------------------------------------ placement
    def _dispatch(self) -> None:
        if self.stopped or self.done or not self.pending_keys:
            return
        pool = self.flow.resident_pool()
        pool.ensure(self.program_key, self.ex.program, self.ex.params, want=self.concurrency, gpu=self.gpu,
                    hbm_gb=self.hbm, max_active=self.ex.max_active_brackets)
        early = [{"metric": r.metric, "value": r.value, "optimization": r.optimization}
                 for r in self.hp.early_stopping]
        while self.pending_keys:
            key = self.pending_keys[0]
            br = self.brackets[key]
            msg = {"op": "bracket", "key": key, "hptuning": self.hp.to_dict(), "iteration": br["iteration"],
                   "configs": br["configs"], "seed": int(self.hp.seed or 0) + 7919 * self.gid,
                   "early_stopping": early}
            allowed = sorted(self.used_workers) if len(self.used_workers) >= self.concurrency else None
            w = pool.assign(self, msg, br["units"], allowed=allowed, key=self.program_key)
            if w is None:
                break
            self.used_workers.add(w.wid)
            br["wid"] = w.wid
            self.pending_keys.pop(0)
        if self.pending_keys:  # every device is busy: try again shortly (an executor or device will free up)
            self.flow.after(0.5, self._dispatch)

    def has_more_work(self) -> bool:
        return any(b["status"] is None for b in self.brackets.values())

    # ------------------------------------------------------------------ executor events (scheduler thread)
    def on_resident_event(self, h, msg: Dict[str, Any]) -> None:
        br = self.brackets.get(msg.get("key"))
        if br is None:
            return
        ev = msg["ev"]
        if ev == "trial_start":
            self._trial_start(h, br, msg)
        elif ev == "trial_end":
            self._trial_end(br, msg)
        elif ev == "rung_done":
            self._rung_done(br, msg)
        elif ev == "bracket_done":
            self._close_open(br, "failed" if msg.get("status") == "failed" else "stopped",
                             f"bracket {msg.get('status')}")
            br["status"] = msg.get("status") or "succeeded"
            self._dispatch()
            self._check_finished()
        elif ev == "error":
            log.warning("group %s bracket %s: %s", self.gid, msg.get("key"), msg.get("message"))

    def on_bracket_lost(self, h, key: str, reason: str) -> None:
        br = self.brackets.get(key)
        if br is None or br["status"] is not None:
            return
        self._close_open(br, "failed", f"resident executor {h.wid} lost: {reason}")
        br["status"] = "failed"
        self._check_finished()

    def _close_open(self, br, status: str, message: str) -> None:
        for xid in list(br["open"]):
            self.store.set_experiment_status(xid, status, message)
            jid = br.get("jobs", {}).pop(xid, None)
            if jid is not None:
                self.store.set_experiment_job_status(jid, status, message)
            self.finished[xid] = status
            self.active.discard(xid)
        br["open"].clear()

    def _experiment_data(self, params: Dict[str, Any]) -> Dict[str, Any]:
        return self.spec.experiment_data(params)

    def _trial_start(self, h, br, msg) -> None:
        rung, cid, params = int(msg["rung"]), int(msg["cid"]), msg["params"]
        prev = br["xids"].get((rung - 1, cid)) if rung > 0 else None
        strategy = ("resume" if self.hb.resume else "restart") if prev is not None else None
        xid = self.store.create_experiment(
            self.project["id"], self._experiment_data(params), group_id=self.gid, user=self.user,
            declarations=params, original_experiment_id=prev, cloning_strategy=strategy,
            code_reference_id=self.flow._group_code_ref(self.gid), resources={"gpu": self.gpu})
        root = br["root"].get(cid) if strategy == "resume" else None
        if root is None:
            br["root"][cid] = xid
            outputs = self.flow.paths.experiment_outputs(self.user, self.project["name"], xid, self.gid)
        else:
            outputs = self.store.get_experiment(root)["outputs_path"]
        logs = self.flow.paths.experiment_logs(self.user, self.project["name"], xid, self.gid)
        self.store.update_experiment(xid, outputs_path=outputs, logs_path=logs)
        br["xids"][(rung, cid)] = xid
        br["open"].add(xid)
        for st in ("scheduled", "starting", "running"):
            self.store.set_experiment_status(xid, st)
        jid = self.store.create_experiment_job(xid, "master", 0, definition={"executor": f"resident:{h.wid}"},
                                               resources={"gpu": self.gpu}, devices=h.devices)
        self.store.set_experiment_job_status(jid, "running")
        br.setdefault("jobs", {})[xid] = jid
        self.flow.auditor.record("experiment.created", "experiment", xid, self.user, group=self.gid)
        self.active.add(xid)

    def _trial_end(self, br, msg) -> None:
        xid = br["xids"].get((int(msg["rung"]), int(msg["cid"])))
        if xid is None:
            return
        v = msg.get("metric")
        name = self.hb.metric.name
        if v is not None:
            self.store.add_metrics(xid, {name: v}, step=int(msg.get("steps", 0)), created_at=msg.get("t_end"))
            status, message = "succeeded", None
        else:
            status, message = "failed", f"{name} is not finite (diverged)"
        self.store.set_experiment_status(xid, status, message)
        self.store.update_experiment(xid, started_at=msg.get("t_start"), finished_at=msg.get("t_end"))
        jid = br.get("jobs", {}).pop(xid, None)
        if jid is not None:
            self.store.set_experiment_job_status(jid, status, message)
        br["open"].discard(xid)
        self.active.discard(xid)
        self.finished[xid] = status
        self.flow.auditor.record(f"experiment.{status}", "experiment", xid, status=status)
        if self.hp.early_stopping and not self.stopped and self._should_stop_early():
            self.flow.auditor.record("experiment_group.stopped", "experiment_group", self.gid, reason="early_stopping")
            self.stop(pending_only=not self.stop_running_on_early_stop, message="Early stopping")

    def _rung_done(self, br, msg) -> None:
        rung = int(msg["rung"])
        ids = [x for (r, _c), x in sorted(br["xids"].items()) if r == rung]
        metrics = [[br["xids"][(rung, int(c))], float(v)] for c, v in msg.get("metrics") or []
                   if (rung, int(c)) in br["xids"]]
        promoted = [br["xids"][(rung, int(c))] for c in msg.get("promoted") or [] if (rung, int(c)) in br["xids"]]
        self.store.create_iteration(self.gid, {"iteration": br["iteration"], "bracket_iteration": rung,
                                               "experiment_ids": ids, "experiments_metrics": metrics,
                                               "promoted": promoted, "executor": br["wid"]})
        if msg.get("early_stop") and not self.stopped:
            self.flow.auditor.record("experiment_group.stopped", "experiment_group", self.gid, reason="early_stopping")
            self.stop(pending_only=not self.stop_running_on_early_stop, message="Early stopping")

    def stop(self, pending_only: bool = False, message: str = "Stopped") -> None:
        self.stopped = True
        pool = self.flow.resident_pool()
        for key in list(self.pending_keys):
            self.brackets[key]["status"] = "stopped"
        self.pending_keys.clear()
        for key, br in self.brackets.items():
            if br["status"] is None and br["wid"] is not None:
                if not pool.send(br["wid"], {"op": "stop_bracket", "key": key}):
                    self._close_open(br, "stopped", message)
                    br["status"] = "stopped"
        if self.store.get_group(self.gid)["status"] not in ("stopped", "succeeded", "failed"):
            self.store.set_group_status(self.gid, "stopped", message)
        self._check_finished()


def make_group_driver(flow, gid: int, spec: GroupSpecification, project: Dict, user: str, cwd: str) -> GroupDriver:
    algo = spec.search_algorithm
    ex = spec.environment.executor if spec.environment is not None else None
    if ex is not None and ex.resident:
        if algo != SearchAlgorithms.HYPERBAND:
            from polyaxon_amd.spec.specification import PolyaxonfileError

            raise PolyaxonfileError(f"resident executors run hyperband groups; {algo} groups use executor: process")
        return ResidentHyperbandDriver(flow, gid, spec, project, user, cwd)
    cls = {SearchAlgorithms.GRID: GridRandomDriver, SearchAlgorithms.RANDOM: GridRandomDriver,
           SearchAlgorithms.HYPERBAND: HyperbandDriver, SearchAlgorithms.BO: BODriver,
           SearchAlgorithms.ASHA: AshaDriver}[algo]
    return cls(flow, gid, spec, project, user, cwd)
