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
            return self.flow._clone(original_id, strategy, params, None, group_id=self.gid, enqueue=enqueue)
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
        if self._should_stop_early(xid):
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
        failed = getattr(self, "failed_message", None)
        status = "failed" if failed else ("stopped" if self.stopped else "succeeded")
        if self.store.get_group(self.gid)["status"] not in ("stopped", "failed"):
            self.store.set_group_status(self.gid, status, failed)
        self.flow.auditor.record(f"experiment_group.{ {'stopped': 'done', 'failed': 'failed'}.get(status, status)}",
                                 "experiment_group", self.gid)

    def _should_stop_early(self, xid: Optional[int] = None) -> bool:
        """Reference ExperimentGroup.should_stop_early (db/models/experiment_groups.py:211-221): any experiment whose
        ``last_metric`` crosses any rule.  Incremental: the reference re-reads every experiment of the group per
        check (O(n^2) over a group); a rule can only newly trip on the experiment that just finished, so only its
        ``last_metric`` is read and tested (``xid``), the group-wide scan is the fallback for a check without one.
        A whole-group scan evaluates every rule in one ``early_stop_any`` call (HIP kernel for device tensors, the
        same vectorised reduction on the host otherwise)."""
        rules = self.hp.early_stopping
        if not rules:
            return False
        if xid is not None:
            last = (self.store.get_experiment(xid) or {}).get("last_metric") or {}
            for r in rules:
                v = last.get(r.metric)
                if isinstance(v, (int, float)) and not math.isnan(v):
                    if (v >= float(r.value)) if Optimization.maximize(r.optimization) else (v <= float(r.value)):
                        return True
            return False
        import numpy as np

        from polyaxon_amd.polytune.utils import early_stop_any_host

        names = sorted({r.metric for r in rules})
        rows = self.store.execute("SELECT last_metric FROM experiments WHERE group_id = ?", (self.gid,)).fetchall()
        mat = np.full((max(len(rows), 1), len(names)), np.nan, dtype=np.float32)
        for i, r in enumerate(rows):
            last = json.loads(r["last_metric"] or "{}")
            for j, n in enumerate(names):
                v = last.get(n)
                if isinstance(v, (int, float)):
                    mat[i, j] = v
        # the host path of the device kernel (the scheduler process stays free of torch and HIP)
        flags = early_stop_any_host(mat, [(names.index(r.metric), float(r.value),
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
    """Hyperband in process mode: the reference's arithmetic and synchronous rung barrier *within* a bracket, but the
    ``s_max + 1`` brackets are independent successive-halving runs, so they all start at once and share the group's
    ``concurrency`` slots -- the reference runs them one after another (polyaxon/hpsearch/tasks/hyperband.py:7-83),
    which leaves devices idle while a small bracket (e.g. 3 configs of ``max_iter: 9``) finishes.  Promotions go to
    the front of the queue (deeper rungs first), so a bracket's later rungs do not wait behind the other brackets'
    first rungs.  Every (bracket, rung) is an iteration row as in the reference."""

    def begin(self) -> None:
        self.m: HyperbandSearchManager = self.manager
        self.brk: Dict[int, Dict[str, Any]] = {}          # iteration (bracket index) -> {"it", "iid", "done"}
        self.xp_bracket: Dict[int, int] = {}
        for i in range(self.m.s_max + 1):
            it = HyperbandIterationConfig(iteration=i, bracket_iteration=0)
            self._launch(it, self.m.get_suggestions(it), None)

    def _launch(self, it: HyperbandIterationConfig, params_list: List[Dict], originals: Optional[List[int]]) -> None:
        ids = []
        strategy = "resume" if self.hp.hyperband.resume else "restart"
        for i, params in enumerate(params_list):
            if originals is None:
                ids.append(self.create_experiment(params))
            else:
                ids.append(self.create_experiment(params, original_id=originals[i], strategy=strategy))
        it.experiment_ids = ids
        iid = self.store.create_iteration(self.gid, it.to_dict())
        self.brk[it.iteration] = {"it": it, "iid": iid, "done": False}
        for x in ids:
            self.xp_bracket[x] = it.iteration
        if originals is None:
            self.queue.extend(ids)
        else:
            self.queue[:0] = ids

    def has_more_work(self) -> bool:
        return not self.stopped and any(not b["done"] for b in self.brk.values())

    def advance(self, xid: int, status: str) -> None:
        b = self.brk.get(self.xp_bracket.get(xid, -1))
        if b is None or b["done"]:
            return
        it = b["it"]
        if any(x not in self.finished for x in it.experiment_ids):
            return  # rung barrier of this bracket only
        metric = self.hp.hyperband.metric.name
        it.experiments_metrics = [(x, v) for x, v in ((x, self.metric_of(x, metric))
                                                      for x in it.experiment_ids) if v is not None]
        self.store.update_iteration(b["iid"], it.to_dict())
        # this bracket's last rung: the reference's create_iteration (iteration_managers/hyperband.py:25-36) moves on
        # to the next bracket as soon as should_reschedule holds, before it considers reducing; only the last bracket
        # (nothing to reschedule to) keeps reducing while configs remain to keep
        if (self.m.should_reschedule(it.iteration, it.bracket_iteration)
                or not self.m.should_reduce_configs(it.iteration, it.bracket_iteration)):
            b["done"] = True
            return
        keep_ids = self.m.reduce(it)
        nxt = HyperbandIterationConfig(iteration=it.iteration, bracket_iteration=it.bracket_iteration + 1)
        r = self.hp.hyperband.resource.cast_value(
            self.m.get_n_resources_for_iteration(nxt.iteration, nxt.bracket_iteration))
        params = []
        for x in keep_ids:
            decl = dict(self.store.get_experiment(x)["declarations"])
            decl[self.hp.hyperband.resource.name] = r
            params.append(decl)
        if not params:
            b["done"] = True
            return
        self._launch(nxt, params, keep_ids)


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


class ResidentDriver(GroupDriver):
    """Base of the drivers that run a group on resident executors (``environment.executor: resident``;
    polyflow/resident.py, pool.py).  The group's work is cut into independent *units* -- Hyperband brackets or
    ASHA shards -- that the pool spreads over the group's executors (at most ``concurrency`` of them, balanced by
    training units).  This driver mirrors what the executors report into the store, so every trial is an
    experiment row with its FSM history, metrics and ``last_metric``; promotions are RESUME (or RESTART) clones of
    the previous rung's experiment with the resource declaration patched (iteration_managers/hyperband.py:79-113);
    every rung decision is an iteration row.

    Faults: a unit whose executor is lost (process died, fatal error) is re-dispatched to a live or newly spawned
    executor with its progress (the last completed rung and its promotions, or an ASHA shard's recorded results),
    up to ``environment.max_restarts`` times (1 when unset) -- a cluster event records each re-dispatch; past the
    budget the unit fails and the group ends ``failed``.  A group none of whose executors can be placed fails
    immediately when the request can never fit, or after ``scheduler.resident_placement_timeout_s`` (300 s)."""

    OP = "bracket"

    def begin(self) -> None:
        from polyaxon_amd.polyflow.programs import program_key

        self.ex = self.spec.environment.executor
        self.program_key = program_key(self.ex.program, self.ex.params)
        res = self.spec.environment.resources
        g = res.gpu.value if (res is not None and res.gpu is not None) else 1.0
        self.gpu = g if g > 0 else 1.0
        if self.gpu > 1 and abs(self.gpu - round(self.gpu)) > 1e-9:
            raise ValueError("a resident DP gang takes whole devices (resources.gpu <= 1 or an integer)")
        self.hbm = res.hbm_gb if res is not None else 0.0
        self.brackets: Dict[str, Dict[str, Any]] = {}
        self.pending_keys: List[str] = []
        self.used_workers: set = set()
        self.failed_message: Optional[str] = None
        mr = int(getattr(self.spec.environment, "max_restarts", 0) or 0)
        self.max_retries = mr if mr > 0 else 1
        self._waiting_since: Optional[float] = None
        self._dispatch_armed = False
        timeout = self.flow.settings.get("scheduler.resident_placement_timeout_s") if self.flow.settings else None
        self.placement_timeout = float(timeout or 300.0)
        self.make_units()
        self._dispatch()

    def make_units(self) -> None:
        raise NotImplementedError

    def unit_done(self, key: str, br: Dict[str, Any]) -> None:
        """A unit ended (any status); drivers whose next units depend on results add them here."""

    def _new_unit(self, key: str, iteration: int, configs: List[Dict[str, Any]], units: float) -> None:
        self.brackets[key] = {"iteration": iteration, "configs": configs, "status": None, "wid": None, "xids": {},
                              "root": {}, "open": set(), "units": units, "retries": 0, "last_rung": None,
                              "promoted": None, "history": []}
        self.pending_keys.append(key)

    def unit_message(self, key: str, br: Dict[str, Any]) -> Dict[str, Any]:
        early = [{"metric": r.metric, "value": r.value, "optimization": r.optimization}
                 for r in self.hp.early_stopping]
        return {"op": self.OP, "key": key, "hptuning": self.hp.to_dict(), "iteration": br["iteration"],
                "configs": br["configs"], "seed": int(self.hp.seed or 0) + 7919 * self.gid, "early_stopping": early}

    # ------------------------------------------------------------------ placement
    def _fail_group(self, message: str) -> None:
        log.error("group %s: %s", self.gid, message)
        self.failed_message = message
        for key in list(self.pending_keys):
            self.brackets[key]["status"] = "failed"
        self.pending_keys.clear()
        self.flow.store.add_cluster_event("resident_executor", "error", f"group {self.gid}: {message}")
        self.stop(pending_only=False, message=message)

    def _arm_dispatch(self) -> None:
        if not self._dispatch_armed:
            self._dispatch_armed = True
            self.flow.after(0.5, self._retry_dispatch)

    def _retry_dispatch(self) -> None:
        self._dispatch_armed = False
        self._dispatch()

    def _dispatch(self) -> None:
        if self.stopped or self.done or not self.pending_keys:
            return
        pool = self.flow.resident_pool()
        live = pool.ensure(self.program_key, self.ex.program, self.ex.params, want=self.concurrency, gpu=self.gpu,
                           hbm_gb=self.hbm, max_active=self.ex.max_active_brackets)
        if not live:
            why = pool.placement_error
            if why is not None:  # the request can never be placed on this node
                self._fail_group(f"no resident executor can be placed: {why}")
                return
            now = time.time()
            self._waiting_since = self._waiting_since or now
            if now - self._waiting_since > self.placement_timeout:
                self._fail_group(f"no resident executor could be placed within {self.placement_timeout:.0f} s")
                return
            self._arm_dispatch()
            return
        self._waiting_since = None
        world = pool.dp_world(self.gpu)
        alive = {w.wid for w in pool.workers_for(self.program_key) if len(w.devices) == world}
        self.used_workers &= alive  # dead executors never count against the group's concurrency
        while self.pending_keys:
            key = self.pending_keys[0]
            br = self.brackets[key]
            msg = self.unit_message(key, br)
            allowed = sorted(self.used_workers) if len(self.used_workers) >= self.concurrency else None
            w = pool.assign(self, msg, br["units"], allowed=allowed, key=self.program_key, world=world)
            if w is None:
                break
            self.used_workers.add(w.wid)
            br["wid"] = w.wid
            self.pending_keys.pop(0)
        if self.pending_keys:  # every device is busy: try again shortly (an executor or device will free up)
            self._arm_dispatch()

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
            self.unit_done(msg.get("key"), br)  # may add units (the next BO batch) before the finish check
            self._dispatch()
            self._check_finished()
        elif ev == "error":
            log.warning("group %s unit %s: %s", self.gid, msg.get("key"), msg.get("message"))

    def on_bracket_lost(self, h, key: str, reason: str) -> None:
        br = self.brackets.get(key)
        self.used_workers.discard(h.wid)
        if br is None or br["status"] is not None:
            return
        self._close_open(br, "failed", f"resident executor {h.wid} lost: {reason}")
        br["wid"] = None
        if not self.stopped and br["retries"] < self.max_retries:
            br["retries"] += 1
            self.flow.store.add_cluster_event(
                "resident_executor", "warning",
                f"group {self.gid}: {self.OP} {key} re-dispatched after executor {h.wid} was lost ({reason}); "
                f"retry {br['retries']} of {self.max_retries}", {"key": key, "from_rung": self._resume_rung(br)})
            self.flow.auditor.record("experiment_group.unit_redispatched", "experiment_group", self.gid, key=key)
            self.pending_keys.append(key)
            self._dispatch()
            return
        br["status"] = "failed"
        self.failed_message = f"{self.OP} {key} lost with executor {h.wid} ({reason}) after {br['retries']} retries"
        self._check_finished()

    def _resume_rung(self, br) -> int:
        return 0 if br["last_rung"] is None else br["last_rung"] + 1

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

    @property
    def resume_enabled(self) -> bool:
        raise NotImplementedError

    def _trial_start(self, h, br, msg) -> None:
        rung, cid, params = int(msg["rung"]), int(msg["cid"]), msg["params"]
        prev = br["xids"].get((rung - 1, cid)) if rung > 0 else None
        # RESUME only when the executor really continued from the previous rung's snapshot; a re-dispatched unit
        # re-trains its promoted configs from scratch (RESTART of the previous rung's experiment)
        resumed = bool(msg.get("resumed", self.resume_enabled))
        strategy = ("resume" if resumed else "restart") if prev is not None else None
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
        rung, cid = int(msg["rung"]), int(msg["cid"])
        xid = br["xids"].get((rung, cid))
        if xid is None:
            return
        v = msg.get("metric")
        br["history"].append([rung, cid, v])
        name = self.metric_name
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
        if v is not None and self.hp.early_stopping and not self.stopped and self._crosses_rule(v):
            self.flow.auditor.record("experiment_group.stopped", "experiment_group", self.gid, reason="early_stopping")
            self.stop(pending_only=not self.stop_running_on_early_stop, message="Early stopping")

    def _crosses_rule(self, v: float) -> bool:
        """Incremental early stopping on the program metric: the reference re-reads every experiment of the group
        per check (db/models/experiment_groups.py:211-221); a new result can only trip a rule by itself, so only it
        is tested (rules on other metrics never see a resident trial's value).  The executors run the same rule
        set over their device metric tensors (``early_stop_any``) and stop their own units."""
        for r in self.hp.early_stopping:
            if r.metric != self.metric_name:
                continue
            if (v >= float(r.value)) if Optimization.maximize(r.optimization) else (v <= float(r.value)):
                return True
        return False

    def _rung_done(self, br, msg) -> None:
        rung = int(msg["rung"])
        ids = [x for (r, _c), x in sorted(br["xids"].items()) if r == rung]
        metrics = [[br["xids"][(rung, int(c))], float(v)] for c, v in msg.get("metrics") or []
                   if (rung, int(c)) in br["xids"]]
        promoted = [br["xids"][(rung, int(c))] for c in msg.get("promoted") or [] if (rung, int(c)) in br["xids"]]
        br["last_rung"] = rung
        br["promoted"] = [int(c) for c in msg.get("promoted") or []]
        self.store.create_iteration(self.gid, {"iteration": br["iteration"], "bracket_iteration": rung,
                                               "experiment_ids": ids, "experiments_metrics": metrics,
                                               "promoted": promoted, "executor": br["wid"], "unit": self.OP})
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
            if br["status"] is None:
                if br["wid"] is None or not pool.send(br["wid"], {"op": "stop_bracket", "key": key}):
                    self._close_open(br, "stopped", message)
                    br["status"] = "stopped"
        if self.store.get_group(self.gid)["status"] not in ("stopped", "succeeded", "failed"):
            self.store.set_group_status(self.gid, "failed" if self.failed_message else "stopped", message)
        self._check_finished()


class ResidentHyperbandDriver(ResidentDriver):
    """Hyperband on resident executors.  The reference runs the brackets one after another with a synchronous rung
    barrier and a 30 s poll (polyaxon/hpsearch/tasks/hyperband.py:7-83), every trial a pod.  Here all ``s_max + 1``
    brackets are created up front (same suggestions as the reference: ``get_suggestions`` per iteration, same seed)
    and run concurrently on the executors; each executor decides its rungs on the device."""

    OP = "bracket"

    def make_units(self) -> None:
        from polyaxon_amd.polyflow.programs import bracket_units

        self.m: HyperbandSearchManager = self.manager
        self.hb = self.hp.hyperband
        rname = self.hb.resource.name
        for it in range(self.m.s_max + 1):
            sugg = self.m.get_suggestions(HyperbandIterationConfig(iteration=it))
            configs = [{"cid": i, "params": {k: v for k, v in s.items() if k != rname}} for i, s in enumerate(sugg)]
            self._new_unit(f"{self.gid}.{it}", it, configs,
                           bracket_units(self.hb.max_iter, self.hb.eta, it, self.hb.resume))

    @property
    def metric_name(self) -> str:
        return self.hb.metric.name

    @property
    def resume_enabled(self) -> bool:
        return bool(self.hb.resume)

    def unit_message(self, key, br):
        msg = super().unit_message(key, br)
        if br["last_rung"] is not None:  # re-dispatch: continue after the last completed rung
            msg["start_rung"] = br["last_rung"] + 1
            msg["active"] = list(br["promoted"] or [])
        return msg


class ResidentAshaDriver(ResidentDriver):
    """ASHA on resident executors (BASELINE config 3's other half; the reference has only the synchronous barrier,
    polyaxon/hpsearch/tasks/hyperband.py:48-83).  The group's ``n_experiments`` configs (same random suggestions as
    process-mode ASHA) are cut into ``executor.shards`` independent shards (default 1); each shard runs on one
    executor as an asynchronous successive-halving search: every round it starts the best unpromoted config in the
    top 1/eta of the highest rung that has one -- ranked by the round's device top-k over the shard's
    [rungs × configs] metric table -- or a new config at rung 0, and promotions RESUME from HBM snapshots."""

    OP = "asha"

    def make_units(self) -> None:
        from polyaxon_amd.polyflow.programs import asha_units

        a = self.hp.asha
        rname = a.resource.name
        sugg = list(self.manager.get_suggestions())
        n = int(self.ex.shards or 1)
        n = max(1, min(n, len(sugg)))
        for s in range(n):
            part = [(i, p) for i, p in enumerate(sugg) if i % n == s]
            configs = [{"cid": j, "params": {k: v for k, v in p.items() if k != rname}} for j, (_i, p) in enumerate(part)]
            self._new_unit(f"{self.gid}.a{s}", s, configs,
                           asha_units(len(configs), a.min_resource, a.max_resource, a.eta, a.resume))

    @property
    def metric_name(self) -> str:
        return self.hp.asha.metric.name

    @property
    def resume_enabled(self) -> bool:
        return bool(self.hp.asha.resume)

    def unit_message(self, key, br):
        msg = super().unit_message(key, br)
        if br["history"]:  # re-dispatch: the results recorded before the executor was lost
            msg["history"] = [list(h) for h in br["history"]]
        return msg

    def _resume_rung(self, br) -> int:
        return max((h[0] for h in br["history"]), default=0)


class ResidentBODriver(ResidentDriver):
    """Bayesian optimisation on resident executors (BASELINE.json config 4: BO over GPT-2 hyper-parameters).  The
    reference runs one BO iteration at a time, every suggestion a pod, and fits the GP after the whole iteration
    (polyaxon/hpsearch/tasks/bo.py:7-70, search_managers/bayesian_optimization/manager.py:17-33).  Here every
    suggestion is a ``trials`` unit of ``executor.params.trial_units`` resource units (default 25) that the pool
    places on a warm executor -- weights re-initialised in place, AdamW hyper-parameters as device data, no process
    start -- and after the initial random batch each iteration asks the GP for ``max(bo.n_suggestions,
    concurrency)`` points (constant-liar batch), so every executor the group may use has a trial.  One iteration
    row per BO iteration, as in process mode (``BODriver``)."""

    OP = "trials"

    def make_units(self) -> None:
        from polyaxon_amd.polytune.bo import BOIterationConfig

        self.BOIterationConfig = BOIterationConfig
        self.iteration = 0
        self.trial_units = float(self.ex.params.get("trial_units", 25))
        self.old_configs: List = []
        self.old_metrics: List = []
        self.batch: List[str] = []
        self._launch(self.manager.get_suggestions(None) or [])

    def _launch(self, suggestions: List[Dict[str, Any]], suggest: Optional[Dict[str, Any]] = None) -> None:
        self.batch = []
        for i, params in enumerate(suggestions):
            key = f"{self.gid}.bo{self.iteration}.{i}"
            self._new_unit(key, self.iteration, [{"cid": 0, "params": dict(params)}], self.trial_units)
            self.batch.append(key)
        self.suggest_info = suggest  # where this iteration's GP ran (kept in the iteration row)
        data = {"iteration": self.iteration, "experiment_ids": [], "unit": self.OP}
        if suggest is not None:
            data["suggest"] = suggest
        self.iteration_id = self.store.create_iteration(self.gid, data)

    @property
    def metric_name(self) -> str:
        return self.hp.bo.metric.name

    @property
    def resume_enabled(self) -> bool:
        return False

    def unit_message(self, key, br):
        early = [{"metric": r.metric, "value": r.value, "optimization": r.optimization}
                 for r in self.hp.early_stopping]
        return {"op": self.OP, "key": key, "configs": br["configs"], "units": self.trial_units,
                "metric": self.metric_name, "maximize": Optimization.maximize(self.hp.bo.metric.optimization),
                "seed": int(self.hp.seed or 0) + 7919 * self.gid + 104729 * br["iteration"] +
                int(key.rsplit(".", 1)[1]), "early_stopping": early}

    def _rung_done(self, br, msg) -> None:  # one BO iteration row per batch (unit_done), not one per trial
        br["last_rung"] = int(msg["rung"])
        if msg.get("early_stop") and not self.stopped:
            self.flow.auditor.record("experiment_group.stopped", "experiment_group", self.gid, reason="early_stopping")
            self.stop(pending_only=not self.stop_running_on_early_stop, message="Early stopping")

    def unit_done(self, key: str, br: Dict[str, Any]) -> None:
        if key not in self.batch or any(self.brackets[k]["status"] is None for k in self.batch):
            return
        ids = []
        for k in self.batch:
            b = self.brackets[k]
            xid = b["xids"].get((0, 0))
            if xid is None:
                continue
            ids.append(xid)
            v = self.metric_of(xid, self.metric_name)
            if v is not None:
                self.old_configs.append((xid, dict(b["configs"][0]["params"])))
                self.old_metrics.append((xid, v))
        data = {"iteration": self.iteration, "experiment_ids": ids, "unit": self.OP,
                "experiments_metrics": [list(m) for m in self.old_metrics if m[0] in ids]}
        if getattr(self, "suggest_info", None) is not None:
            data["suggest"] = self.suggest_info
        self.store.update_iteration(self.iteration_id, data)
        if self.stopped or not self.manager.should_reschedule(self.iteration) or not self.old_metrics:
            self.batch = []
            return
        self.iteration += 1
        cfg = self.BOIterationConfig(iteration=self.iteration, old_experiments_configs=list(self.old_configs),
                                     old_experiments_metrics=list(self.old_metrics))
        self._request_suggestions(cfg, max(int(self.hp.bo.n_suggestions or 1), int(self.concurrency)))

    # ------------------------------------------------------------------ the GP runs on an executor, not here
    awaiting: Optional[str] = None  # key of the outstanding bo_suggest request

    def _observations(self, cfg):
        configs_by_id = dict(cfg.combined_experiments_configs)
        metrics_by_id = dict(cfg.combined_experiments_metrics)
        keys = list(metrics_by_id)
        return [configs_by_id[k] for k in keys], [float(metrics_by_id[k]) for k in keys]

    def _request_suggestions(self, cfg, n: int) -> None:
        """The GP fit and the acquisition search run on one of the group's executors (``bo_suggest``: the HIP kernels
        on its device), so the scheduler process never initialises HIP (the reference runs hpsearch on a CPU worker
        queue of its own, apart from the trial pods: celery_settings.py:398-419).  No executor to ask: numpy here."""
        configs, metrics = self._observations(cfg)
        key = f"{self.gid}.bo{self.iteration}.suggest"
        msg = {"op": "bo_suggest", "key": key, "hptuning": self.hp.to_dict(), "configs": configs,
               "metrics": metrics, "n": int(n)}
        pool = self.flow.resident_pool()
        allowed = sorted(self.used_workers) or None
        self.awaiting = key
        self._pending_cfg = (cfg, n)
        if pool.request(self, msg, key=self.program_key, allowed=allowed) is None:
            self._suggest_here("no live executor of the group")

    def _suggest_here(self, why: str) -> None:
        from polyaxon_amd.polytune.bo import suggest

        cfg, n = self._pending_cfg
        self.awaiting = None
        log.warning("group %s: BO iteration %d on the scheduler's numpy backend (%s)", self.gid, self.iteration, why)
        configs, metrics = self._observations(cfg)
        out = suggest(self.hp, configs, metrics, n, backend="numpy")
        self._suggested(out, {"backend": "numpy", "where": "scheduler", "reason": why})

    def _suggested(self, suggestions, info: Dict[str, Any]) -> None:
        if self.stopped:
            self._check_finished()
            return
        self._launch(suggestions or [], info)
        self._dispatch()
        self._check_finished()

    def has_more_work(self) -> bool:
        return self.awaiting is not None or super().has_more_work()

    def on_resident_event(self, h, msg: Dict[str, Any]) -> None:
        key = msg.get("key")
        if key is not None and key == self.awaiting:
            self.awaiting = None
            if msg.get("ev") == "bo_suggestions":
                self._suggested(msg.get("suggestions") or [], {"backend": msg.get("backend"), "where": f"executor {h.wid}",
                                                               "ms": msg.get("ms")})
            else:  # the executor could not compute it (error reply): do it here
                self.awaiting = key
                self._suggest_here(f"executor {h.wid}: {msg.get('message')}")
            return
        super().on_resident_event(h, msg)

    def on_bracket_lost(self, h, key: str, reason: str) -> None:
        if key == self.awaiting:
            self._suggest_here(f"executor {h.wid} lost: {reason}")
            return
        super().on_bracket_lost(h, key, reason)


def make_group_driver(flow, gid: int, spec: GroupSpecification, project: Dict, user: str, cwd: str) -> GroupDriver:
    algo = spec.search_algorithm
    ex = spec.environment.executor if spec.environment is not None else None
    if ex is not None and ex.resident:
        if algo == SearchAlgorithms.ASHA:
            return ResidentAshaDriver(flow, gid, spec, project, user, cwd)
        if algo == SearchAlgorithms.BO:
            return ResidentBODriver(flow, gid, spec, project, user, cwd)
        if algo != SearchAlgorithms.HYPERBAND:
            from polyaxon_amd.spec.specification import PolyaxonfileError

            raise PolyaxonfileError(f"resident executors run hyperband, asha and bo groups; {algo} groups use "
                                    "executor: process")
        return ResidentHyperbandDriver(flow, gid, spec, project, user, cwd)
    cls = {SearchAlgorithms.GRID: GridRandomDriver, SearchAlgorithms.RANDOM: GridRandomDriver,
           SearchAlgorithms.HYPERBAND: HyperbandDriver, SearchAlgorithms.BO: BODriver,
           SearchAlgorithms.ASHA: AshaDriver}[algo]
    return cls(flow, gid, spec, project, user, cwd)
