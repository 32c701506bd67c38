"""Pipelines: DAGs of operations with trigger policies, concurrency, retries with exponential backoff,
timeouts and schedules (reference polyaxon/pipelines/{dags,tasks,celery_task}.py, operations/, and
db/models/pipelines.py:23-611).

Each op's ``template`` is an inline Polyaxonfile (experiment, job or group) run through polyflow; op
completion is signalled by the run's ``on_done`` callback (groups: the driver finishing), so downstream ops
are evaluated the instant an upstream op finishes instead of via Celery task chaining.  Retries are
polyflow timers (``retry_delay * 2**attempt`` capped by ``max_retry_delay`` when
``retry_exponential_backoff``; reference Operation.get_countdown :233-241); ``timeout`` stops the op's
run (reference soft/hard time limits :243-258).
"""
from __future__ import annotations

import copy
from collections import deque
from typing import Any, Dict, Iterable, List, Optional, Set

from polyaxon_amd.fsm import OperationLifeCycle, TriggerPolicy
from polyaxon_amd.spec import specification_for


# ------------------------------------------------------------------ DAG helpers (reference pipelines/dags.py)
def get_dag(nodes: Iterable[Any], downstream_fn) -> tuple:
    dag, by_id = {}, {}
    for n in nodes:
        key = n if not hasattr(n, "id") else n.id
        dag[key] = set(downstream_fn(n))
        by_id[key] = n
    return dag, by_id


def get_independent_nodes(dag: Dict[Any, Set[Any]]) -> Set[Any]:
    dependents = {d for ds in dag.values() for d in ds}
    return set(dag) - dependents


def get_orphan_nodes(dag: Dict[Any, Set[Any]]) -> Set[Any]:
    return {n for n in get_independent_nodes(dag) if not dag[n]}


def has_dependencies(node, dag) -> bool:
    return any(node in ds for ds in dag.values())


def sort_topologically(dag: Dict[Any, Set[Any]]) -> List[Any]:
    """Breadth-first Kahn ordering; raises ValueError on a cycle."""
    indeg = {n: 0 for n in dag}
    for ds in dag.values():
        for d in ds:
            if d in indeg:
                indeg[d] += 1
    q = deque(sorted((n for n, k in indeg.items() if k == 0), key=str))
    out = []
    while q:
        n = q.popleft()
        out.append(n)
        for d in sorted(dag[n], key=str):
            if d in indeg:
                indeg[d] -= 1
                if indeg[d] == 0:
                    q.append(d)
    if len(out) != len(dag):
        raise ValueError("graph is not acyclic")
    return out


def trigger_satisfied(policy: str, upstream_statuses: List[str]) -> Optional[bool]:
    """True = can start, False = can never start (upstream_failed), None = wait."""
    S = OperationLifeCycle
    done = [s for s in upstream_statuses if S.is_done(s)]
    all_done = len(done) == len(upstream_statuses)
    if not upstream_statuses:
        return True
    if policy == TriggerPolicy.ONE_DONE:
        return True if done else None
    if policy == TriggerPolicy.ONE_SUCCEEDED:
        if any(s == "succeeded" for s in upstream_statuses):
            return True
        return False if all_done else None
    if policy == TriggerPolicy.ONE_FAILED:
        if any(S.failed(s) for s in upstream_statuses):
            return True
        return False if all_done else None
    if not all_done:
        return None
    if policy == TriggerPolicy.ALL_DONE:
        return True
    if policy == TriggerPolicy.ALL_SUCCEEDED:
        return all(s == "succeeded" for s in upstream_statuses)
    if policy == TriggerPolicy.ALL_FAILED:
        return all(S.failed(s) for s in upstream_statuses)
    raise ValueError(f"unknown trigger policy {policy}")


class PipelineRunner:
    def __init__(self, flow, pipeline_id: int, spec, project: Dict, user: str, cwd: str):
        self.flow = flow
        self.store = flow.store
        self.pipeline_id = pipeline_id
        self.spec = spec
        self.project = project
        self.user = user
        self.cwd = cwd
        self.ops = {op["name"]: op for op in spec.ops}
        self.dag = {name: set() for name in self.ops}
        for name, op in self.ops.items():
            for u in op["upstream"]:
                self.dag[u].add(name)
        sort_topologically(self.dag)  # validates acyclicity
        self.concurrency = spec.concurrency
        self.on_finished: List[Any] = []  # callbacks(runner) when the run is finished / stopped (schedules)
        self.finished = False
        self.succeeded = False
        self.run_id: Optional[int] = None

    def start(self) -> int:
        self.run_id = self.store.create_pipeline_run(self.pipeline_id)
        self.op_runs: Dict[str, int] = {}
        self.attempts: Dict[str, int] = {}
        self.entity: Dict[str, tuple] = {}
        for name in sort_topologically(self.dag):
            self.op_runs[name] = self.store.create_operation_run(self.run_id, name, self.ops[name])
        self.store.set_pipeline_run_status(self.run_id, "scheduled")
        self.store.set_pipeline_run_status(self.run_id, "running")
        self.flow.auditor.record("pipeline.started", "pipeline", self.pipeline_id, run=self.run_id)
        self._evaluate()
        return self.run_id

    def status(self, name: str) -> str:
        return self.store.get("operation_runs", self.op_runs[name])["status"]

    def _running_count(self) -> int:
        return sum(1 for n in self.ops if OperationLifeCycle.is_running(self.status(n)))

    def _evaluate(self) -> None:
        progressed = True
        while progressed:
            progressed = False
            for name in sort_topologically(self.dag):
                if self.status(name) != "created":
                    continue
                ups = [self.status(u) for u in self.ops[name]["upstream"]]
                ok = trigger_satisfied(self.ops[name]["trigger"], ups)
                if ok is False:
                    self.store.set_operation_run_status(self.op_runs[name], "upstream_failed",
                                                        "upstream trigger can no longer be met")
                    self.flow.auditor.record("operation.upstream_failed", "operation", self.op_runs[name])
                    progressed = True
                elif ok:
                    if self.concurrency and self._running_count() >= self.concurrency:
                        continue
                    self._launch(name)
                    progressed = True
        self._check_done()

    def _launch(self, name: str) -> None:
        oid = self.op_runs[name]
        op = self.ops[name]
        self.store.set_operation_run_status(oid, "scheduled")
        tmpl = op.get("template")
        if tmpl is None:  # a no-op marker node
            self.store.set_operation_run_status(oid, "running")
            self.store.set_operation_run_status(oid, "succeeded")
            return
        spec = specification_for(copy.deepcopy(tmpl))
        res = self.flow._submit(spec, self.project["name"], self.user, self.cwd, f"{name}", None)
        kind, eid = res["kind"], res["id"]
        self.entity[name] = (kind, eid)
        self.store.update_operation_run(oid, entity_kind=kind, entity_id=eid)
        self.store.set_operation_run_status(oid, "running")
        self.flow.auditor.record("operation.started", "operation", oid, entity=kind, entity_id=eid)
        if kind == "group":
            driver = self.flow.groups[eid]
            orig = driver._check_finished

            def hooked(orig=orig, driver=driver, name=name):
                was = driver.done
                orig()
                if driver.done and not was:
                    st = self.store.get_group(driver.gid)["status"]
                    self._on_op_done(name, "succeeded" if st == "succeeded" else "failed")

            driver._check_finished = hooked
            hooked()
        else:
            owner = f"{'experiment' if kind == 'experiment' else 'job'}:{eid}"
            self.flow.runs[owner].on_done.append(lambda st, name=name: self._on_op_done(name, st))
        timeout = op.get("timeout")
        if timeout:
            self.flow.after(float(timeout), lambda name=name, att=self.attempts.get(name, 0): self._timeout(name, att))

    def _timeout(self, name: str, attempt: int) -> None:
        if self.attempts.get(name, 0) != attempt or self.status(name) != "running":
            return
        kind, eid = self.entity[name]
        if kind == "group":
            self.flow._stop_group(eid, False, "operation timeout")
        else:
            self.flow._stop("experiment" if kind == "experiment" else "job", eid, "operation timeout")

    def _on_op_done(self, name: str, run_status: str) -> None:
        oid = self.op_runs[name]
        op = self.ops[name]
        if run_status == "succeeded":
            self.store.set_operation_run_status(oid, "succeeded")
            self.flow.auditor.record("operation.succeeded", "operation", oid)
        else:
            attempt = self.attempts.get(name, 0)
            if attempt < int(op.get("max_retries", 0) or 0):
                self.attempts[name] = attempt + 1
                self.store.set_operation_run_status(oid, "retrying", f"{run_status}; retry {attempt + 1}")
                self.store.update_operation_run(oid, retries=attempt + 1)
                self.flow.auditor.record("operation.retrying", "operation", oid)
                delay = float(op.get("retry_delay", 0) or 0)
                if op.get("retry_exponential_backoff"):
                    delay = delay * (2 ** attempt)
                    if op.get("max_retry_delay"):
                        delay = min(delay, float(op["max_retry_delay"]))
                self.flow.after(delay, lambda name=name: self._retry(name))
                return
            self.store.set_operation_run_status(oid, "failed" if run_status == "failed" else "stopped",
                                                f"run {run_status}")
            self.flow.auditor.record("operation.failed", "operation", oid)
        self._evaluate()

    def _retry(self, name: str) -> None:
        self._launch(name)  # retrying -> scheduled -> running

    def _check_done(self) -> None:
        statuses = [self.status(n) for n in self.ops]
        if all(OperationLifeCycle.is_done(s) for s in statuses):
            rec = self.store.get("pipeline_runs", self.run_id)
            if rec["status"] not in ("finished", "stopped", "skipped"):
                self.store.set_pipeline_run_status(self.run_id, "finished")
                ok = all(s == "succeeded" for s in statuses)
                self.flow.auditor.record("pipeline.succeeded" if ok else "pipeline.failed", "pipeline",
                                         self.pipeline_id, run=self.run_id)
                self.flow.auditor.record("pipeline.done", "pipeline", self.pipeline_id, run=self.run_id)
                self._finish(ok)

    def _finish(self, ok: bool) -> None:
        if self.finished:
            return
        self.finished, self.succeeded = True, ok
        for cb in list(self.on_finished):
            cb(self)

    def stop(self) -> None:
        for name in self.ops:
            st = self.status(name)
            if st == "created":
                self.store.set_operation_run_status(self.op_runs[name], "skipped")
            elif OperationLifeCycle.is_running(st) and name in self.entity:
                kind, eid = self.entity[name]
                if kind == "group":
                    self.flow._stop_group(eid, False, "pipeline stopped")
                else:
                    self.flow._stop("experiment" if kind == "experiment" else "job", eid, "pipeline stopped")
        self.store.set_pipeline_run_status(self.run_id, "stopped")
        self._finish(False)
