"""polyflow: the event-driven node scheduler (replaces the reference's scheduler/ + spawners/ + Celery +
monitors + crons for one 8×MI355X node).

Reference call stacks collapsed here: run one experiment (API → signals → Celery
build/start → spawner → K8s pods → status monitor → events worker → aggregation → stop), groups
(§3.2-3.3, hpsearch tasks), distributed experiments (§3.6, per-framework spawners), generic jobs /
builds / notebooks / tensorboards (scheduler/{job,dockerizer,notebook,tensorboard}_scheduler.py).

Design (MI355X-first, single node):
* one scheduler thread owns all mutable state (allocator, run table, group drivers) — no locks on the
  hot path, no races on device accounting (reference: hpsearch/tasks/base.py:44-47 admits races);
* the thread blocks in the native process monitor (csrc/procmon.cpp: epoll over pidfds + an eventfd),
  so a replica exit, a submitted command and a timer deadline all wake it immediately: the gap between
  a trial ending and the next one being spawned is the cost of one ``posix_spawn``, not a 1–30 s poll;
* replicas are plain processes pinned with ``HIP_VISIBLE_DEVICES`` and the reference env contract
  (polyflow/env.py); gangs (DP=2/4/8) are allocated all-or-nothing by the device allocator;
* every status change goes through the lifecycle FSMs in the store; every lifecycle event goes to the
  auditor (activity log, notifications, webhooks).
"""
from __future__ import annotations

import hashlib
import heapq
import json
import logging
import os
import shlex
import shutil
import signal
import sys
import threading
import time
import traceback
import uuid
from collections import deque
from dataclasses import dataclass, field
from typing import Any, Callable, Deque, Dict, List, Optional, Tuple

from polyaxon_amd.fsm import ExperimentLifeCycle, JobLifeCycle
from polyaxon_amd.obs.events import Auditor
from polyaxon_amd.polyflow import dockerizer
from polyaxon_amd.polyflow.devices import DeviceAllocator, device_cpus
from polyaxon_amd.polyflow.env import cluster_def as make_cluster_def
from polyaxon_amd.polyflow.env import free_port, trial_env
from polyaxon_amd.polyflow.faults import parse_fault
from polyaxon_amd.polyflow.paths import Paths
from polyaxon_amd.polyflow.process import ProcessMonitor
from polyaxon_amd.spec import specification_for
from polyaxon_amd.spec.specification import (BaseSpecification, ExperimentSpecification, GroupSpecification,
                                             Kinds, PolyaxonfileError)
from polyaxon_amd.store import Store

log = logging.getLogger("polyaxon_amd.polyflow")

BUILD_REUSE_S = 6 * 3600  # reference dockerizer_scheduler.py:48-50


@dataclass
class Replica:
    role: str
    index: int
    job_id: int
    gpus: float
    devices: List[int] = field(default_factory=list)
    pid: Optional[int] = None
    exit_code: Optional[int] = None
    done: bool = False


@dataclass
class Run:
    kind: str  # "experiment" | "job"
    id: int
    spec: BaseSpecification
    cwd: str
    replicas: List[Replica] = field(default_factory=list)
    stop_requested: bool = False
    stop_reason: Optional[str] = None
    final_status: Optional[str] = None
    final_message: Optional[str] = None
    created: float = field(default_factory=time.time)
    started: Optional[float] = None
    build_id: Optional[int] = None
    port: Optional[int] = None
    extra_env: Dict[str, str] = field(default_factory=dict)
    on_done: List[Callable[[str], None]] = field(default_factory=list)
    attempt: int = 0  # opt-in retries (environment.max_restarts)
    alloc_owners: List[str] = field(default_factory=list)  # allocator owners of the current placement
    waiting_since: Optional[float] = None  # first time a gang failed to place (gang reservation)

    @property
    def owner(self) -> str:
        return f"{self.kind}:{self.id}"

    @property
    def active(self) -> bool:
        return any(r.pid is not None and not r.done for r in self.replicas)


def _replica_gpus(spec: BaseSpecification, role: str, index: int) -> float:
    if role == "master":
        res = spec.resources
    elif role == "worker":
        res = spec.get_worker_resources(index) or spec.resources
    else:
        res = spec.get_ps_resources(index)
    if res is None or res.gpu is None:
        return 0.0
    return float(res.gpu.value)


_SHELL_OPS = ("&&", "||", ";", "|", ">", "<", "`", "$(", "\n")


def profile_argv(cmd: str, out_dir: str) -> Optional[List[str]]:
    """``rocprofv3 --kernel-trace --stats ... -- <argv>`` for a plain command line, else None.  The profiler must
    start the program itself (its preloaded library initialises the GPU first, so a shell or env wrapper that
    later execs the program is not allowed): commands with shell operators or leading ``VAR=`` assignments are
    run unprofiled."""
    if any(op in cmd for op in _SHELL_OPS):
        return None
    try:
        argv = shlex.split(cmd)
    except ValueError:
        return None
    if not argv or "=" in argv[0]:
        return None
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    return [exe, "--kernel-trace", "--stats", "--output-format", "csv", "-d", out_dir, "-o", "trial", "--", *argv]


def _command(spec: BaseSpecification) -> str:
    if spec.run is None:
        raise PolyaxonfileError("nothing to run: the specification has no `run.cmd`")
    return " && ".join(spec.run.commands)


def device_footprint() -> Dict[str, bool]:
    """Does THIS process hold any GPU state?  The scheduler must not: torch never imported, the HIP runtime not
    mapped, no /dev/kfd descriptor (reported by the bench's control process, checked by
    tests/test_gpu_free_scheduler.py)."""
    import sys

    try:
        maps = open("/proc/self/maps").read()
    except OSError:
        maps = ""
    kfd = False
    try:
        for f in os.listdir("/proc/self/fd"):
            try:
                kfd = kfd or "/dev/kfd" in os.readlink(f"/proc/self/fd/{f}")
            except OSError:
                pass
    except OSError:
        pass
    return {"torch_imported": "torch" in sys.modules, "hip_mapped": "libamdhip64" in maps, "kfd_open": kfd}


class Polyflow:
    """Node scheduler. Public methods are thread-safe (they post commands to the scheduler thread)."""

    def __init__(self, root: str, store: Optional[Store] = None, allocator: Optional[DeviceAllocator] = None,
                 auditor: Optional[Auditor] = None, api_host: Optional[str] = None, stop_grace_s: float = 10.0,
                 python: Optional[str] = None, reconcile_s: float = 5.0,
                 health_check: Optional[Callable[[], List[int]]] = None, clean_on_start: bool = True,
                 settings=None):
        """``settings`` (polyaxon_amd.conf.Settings, e.g. from ``plx server``) supplies the reconcile period,
        stop grace, build reuse window, stats / tracker / notification backends; explicit arguments win."""
        if settings is not None:
            reconcile_s = settings.get("scheduler.reconcile_interval_s") if reconcile_s == 5.0 else reconcile_s
            stop_grace_s = settings.get("scheduler.stop_grace_s") if stop_grace_s == 10.0 else stop_grace_s
        self.settings = settings
        # the scheduler process never initialises HIP: a BO group's GP runs on its resident executors, or on numpy
        from polyaxon_amd.polytune import bo as _bo

        self._device_allowed_before = _bo.device_allowed()
        _bo.set_device_allowed(False)
        self.numa_bind = settings.get("scheduler.numa_bind") if settings is not None else True
        self.build_reuse_s = settings.get("scheduler.build_reuse_s") if settings is not None else BUILD_REUSE_S
        self.build_backend = settings.get("build.backend") if settings is not None else "native"
        self.build_registry = settings.get("build.registry") if settings is not None else dockerizer.DEFAULT_REGISTRY
        self.build_push = settings.get("build.push") if settings is not None else False
        self.paths = Paths(root)
        self.clean_on_start = clean_on_start
        self.store_path = os.path.join(self.paths.root, "polyaxon.sqlite")
        self.store = store or Store(self.store_path)
        if store is not None and store.path != ":memory:":
            self.store_path = store.path
        self.alloc = allocator or DeviceAllocator()
        if auditor is None and settings is not None:
            auditor = Auditor.from_settings(self.store, settings, root=self.paths.root)
        self.auditor = auditor or Auditor(self.store)
        if auditor is None and os.environ.get("PLX_NOTIFICATIONS"):
            from polyaxon_amd.obs.events import load_notification_config

            self.auditor.configure(load_notification_config(os.environ["PLX_NOTIFICATIONS"]))
        self.api_host = api_host
        self.stop_grace_s = stop_grace_s
        self.python = python or sys.executable
        self.pm = ProcessMonitor()
        self.runs: Dict[str, Run] = {}
        self.pending: Deque[str] = deque()
        self.pid_index: Dict[int, Tuple[str, int]] = {}
        self.groups: Dict[int, Any] = {}
        self.pipelines: Dict[int, Any] = {}
        self._cmds: Deque[Tuple[Callable, tuple, Optional["_Result"]]] = deque()
        self._timers: List[Tuple[float, int, Callable]] = []
        self._timer_seq = 0
        self._thread: Optional[threading.Thread] = None
        self._running = False
        self._idle = threading.Event()
        self.stats = {"spawned": 0, "exited": 0, "gaps_ms": [], "retries": 0, "heartbeat_kills": 0,
                      "faults_injected": 0}
        self._last_exit_t: Optional[float] = None
        self.reconcile_s = reconcile_s
        # () -> indices of unhealthy devices.  Default (auto-detected devices only): the RAS/ECC + KFD probe of
        # obs/nodes.py; a test that injects its own allocator keeps the probe off unless it passes one.
        probe_on = settings.get("scheduler.health_probe") if settings is not None else True
        if health_check is None and allocator is None and probe_on:
            from polyaxon_amd.obs.nodes import GpuHealthProbe

            health_check = GpuHealthProbe(events=self.cluster_event, background=True,
                                          interval_s=max(1.0, reconcile_s))
        self.health_check = health_check
        self._unhealthy: set = set()
        self._pool = None  # resident executors (polyflow/pool.py), created on first use

    def resident_pool(self):
        """The pool of warm resident trial executors (scheduler thread only)."""
        if self._pool is None:
            from polyaxon_amd.polyflow.pool import ResidentPool

            idle = self.settings.get("scheduler.resident_idle_s") if self.settings is not None else 300.0
            self._pool = ResidentPool(self, idle_s=float(idle))
        return self._pool

    def attach_resident(self, chan, device: int, program: str, params=None, max_active: int = 8) -> int:
        """Register an already running resident executor that owns ``device`` (bench.py ranks, external
        launchers).  Returns its worker id."""
        return self.call(lambda: self.resident_pool().attach(chan, device, program, params, max_active).wid)

    # ================================================================== lifecycle of the scheduler itself
    def start(self) -> "Polyflow":
        if self._thread is None:
            if self.clean_on_start:  # runs a previous scheduler process left non-terminal
                from polyaxon_amd.polyflow.cleaning import clean_stale

                cleaned = clean_stale(self.store)
                if any(cleaned.values()):
                    log.warning("cleaning hook stopped orphaned runs: %s", cleaned)
            with open(os.path.join(self.paths.root, "scheduler.pid"), "w") as f:
                f.write(str(os.getpid()))
            self._running = True
            self._thread = threading.Thread(target=self._loop, name="polyflow", daemon=True)
            self._thread.start()
            if self.reconcile_s > 0:
                self.after(self.reconcile_s, self._reconcile)
            self.sync_inventory()
        return self

    def sync_inventory(self) -> Dict[str, Any]:
        """Node row + one NodeGPU row per device (KFD topology / amd-smi; reference crons/tasks/nodes.py)."""
        from polyaxon_amd.obs.nodes import sync_node_inventory

        try:
            inv = sync_node_inventory(self.store, self.alloc.n_devices)
        except Exception as e:  # inventory must never keep the scheduler from starting
            log.warning("node inventory failed: %s", e)
            self.store.upsert_node("local", os.uname().nodename, float(os.cpu_count() or 1), 0.0,
                                   self.alloc.n_devices)
            return {}
        by_index = {g["index"]: g for g in inv.get("gpus", [])}
        for d in self.alloc.devices:
            g = by_index.get(d.index)
            if g is not None:
                d.name = g["name"]
                if g["memory_gb"]:
                    d.memory_gb = float(g["memory_gb"])
        return inv

    def cluster_event(self, kind: str, level: str, message: str, data: Optional[Dict[str, Any]] = None) -> None:
        """Persist a node-level event (reference monitor_namespace: k8s warnings -> ClusterEvent rows)."""
        try:
            self.store.add_cluster_event(kind, level, message, data or {})
            self.auditor.record("cluster.event", "cluster", None, kind=kind, level=level, message=message)
        except Exception:
            log.exception("cluster event %s failed", kind)

    def shutdown(self, stop_running: bool = True, timeout: float = 30.0) -> None:
        if self._thread is None:
            return
        if stop_running:
            self.call(self._stop_all)
            end = time.time() + timeout
            while time.time() < end and self.call(lambda: any(r.active for r in self.runs.values())):
                time.sleep(0.05)
        if self._pool is not None:
            self.call(self._pool.close, timeout=timeout + 5)
        self._running = False
        self.pm.wake()
        self._thread.join(timeout=timeout)
        self._thread = None
        from polyaxon_amd.polytune import bo as _bo

        _bo.set_device_allowed(self._device_allowed_before)
        try:
            os.unlink(os.path.join(self.paths.root, "scheduler.pid"))
        except OSError:
            pass

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.shutdown()

    # ================================================================== command plumbing
    def call(self, fn: Callable, *args, timeout: Optional[float] = 60.0):
        """Run ``fn(*args)`` on the scheduler thread and return its result (or raise its exception)."""
        if self._thread is None or threading.current_thread() is self._thread:
            return fn(*args)
        res = _Result()
        self._cmds.append((fn, args, res))
        self.pm.wake()
        return res.get(timeout)

    def post(self, fn: Callable, *args) -> None:
        self._cmds.append((fn, args, None))
        self.pm.wake()

    def after(self, delay_s: float, fn: Callable) -> None:
        """Timer on the scheduler thread."""
        self._timer_seq += 1
        heapq.heappush(self._timers, (time.time() + delay_s, self._timer_seq, fn))
        self.pm.wake()

    def _loop(self) -> None:
        while self._running:
            try:
                self._drain_commands()
                self._fire_timers()
                self._schedule()
                busy = any(r.active for r in self.runs.values()) or bool(self.pending) or bool(self._cmds)
                if not busy:
                    self._idle.set()
                timeout = 1.0
                if self._timers:
                    timeout = max(0.0, min(timeout, self._timers[0][0] - time.time()))
                if self._cmds:
                    timeout = 0.0
                got = self.pm.wait(timeout)
                while got is not None:
                    self._on_exit(*got)
                    got = self.pm.wait(0)
            except Exception:
                log.exception("polyflow loop error")

    def _drain_commands(self) -> None:
        while self._cmds:
            fn, args, res = self._cmds.popleft()
            try:
                out = fn(*args)
                if res is not None:
                    res.set(out)
            except BaseException as e:  # noqa: BLE001 - forwarded to the caller
                if res is not None:
                    res.fail(e)
                else:
                    log.exception("polyflow command failed")

    def _fire_timers(self) -> None:
        now = time.time()
        while self._timers and self._timers[0][0] <= now:
            _, _, fn = heapq.heappop(self._timers)
            try:
                fn()
            except Exception:
                log.exception("polyflow timer failed")

    # ================================================================== submission API
    def submit(self, content, project: str = "default", user: str = "root", cwd: Optional[str] = None,
               name: Optional[str] = None, description: Optional[str] = None) -> Dict[str, Any]:
        """``polyaxon run -f polyaxonfile.yml`` equivalent. Returns {"kind", "id"}."""
        spec = content if isinstance(content, BaseSpecification) else specification_for(content)
        return self.call(self._submit, spec, project, user, cwd or os.getcwd(), name, description)

    def _code_ref(self, cwd: str) -> Optional[int]:
        """One CodeReference per (submission dir, commit); reused by every trial of a group."""
        from polyaxon_amd.polyflow.repos import code_reference

        ref = code_reference(cwd)
        if ref is None:
            return None
        key = f"coderef:{cwd}:{ref['commit']}:{hash(ref['diff'] or '')}"
        cached = self.store.kv_get(key)
        if cached:
            return int(cached)
        rid = self.store.create_code_reference(ref["commit"], ref["branch"], ref["git_url"], ref["is_dirty"],
                                               ref["diff"])
        self.store.kv_set(key, rid)
        return rid

    def _external_checkout(self, spec: BaseSpecification, proj: Dict, user: str) -> Optional[str]:
        """``build.git``: fetch the external repository and check out ``build.ref``; the run executes there."""
        b = spec.build
        if b is None or not b.git:
            return None
        from polyaxon_amd.polyflow.repos import ExternalRepo, GitError

        repo = ExternalRepo(self.paths.repos_root, user, proj["name"], str(b.git))
        try:
            repo.fetch()
            sha = repo.checkout(str(b.ref) if b.ref else None)
        except GitError as e:
            raise PolyaxonfileError(f"external repo {b.git}: {e}") from None
        self.store.upsert_external_repo(proj["id"], str(b.git), repo.path, sha)
        self.auditor.record("repo.new_commit", "repo", proj["id"], git_url=str(b.git), commit=sha)
        return repo.path

    def _submit(self, spec: BaseSpecification, project: str, user: str, cwd: str, name, description):
        proj = self.store.get_or_create_project(spec.project or project, user)
        cwd = self._external_checkout(spec, proj, user) or cwd
        self._current_code_ref = self._code_ref(cwd)
        if spec.kind == Kinds.EXPERIMENT:
            xid = self._create_experiment(spec, proj, user, cwd, name=name, description=description)
            return {"kind": "experiment", "id": xid}
        if spec.kind == Kinds.GROUP:
            from polyaxon_amd.polyflow.groups import make_group_driver

            ex = spec.environment.executor
            if ex is not None and ex.resident:
                if spec.search_algorithm not in ("hyperband", "asha", "bo"):
                    raise PolyaxonfileError(f"resident executors run hyperband, asha and bo groups; "
                                            f"{spec.search_algorithm} groups use executor: process")
                g = spec.resources.gpu.value if (spec.resources is not None and spec.resources.gpu is not None) else 1
                if g > 1 and abs(g - round(g)) > 1e-9:
                    raise PolyaxonfileError("a resident DP gang takes whole devices (resources.gpu <= 1 or an "
                                            "integer)")

            gid = self.store.create_group(proj["id"], spec.raw_data, spec.hptuning.to_dict(), user=user,
                                          name=name or spec.name, description=description, tags=spec.tags,
                                          search_algorithm=spec.search_algorithm, concurrency=spec.concurrency,
                                          code_reference_id=self._current_code_ref)
            self.auditor.record("experiment_group.created", "experiment_group", gid, user)
            driver = make_group_driver(self, gid, spec, proj, user, cwd)
            self.groups[gid] = driver
            driver.start()
            return {"kind": "group", "id": gid}
        if spec.kind in (Kinds.JOB, Kinds.NOTEBOOK, Kinds.TENSORBOARD, Kinds.BUILD):
            jid = self._create_job(spec, proj, user, cwd, name=name, description=description)
            return {"kind": spec.kind, "id": jid}
        if spec.kind == Kinds.PIPELINE:
            from polyaxon_amd.polyflow.pipelines import PipelineRunner

            pid = self.store.create_pipeline(proj["id"], name or spec.name or "pipeline", spec.raw_data, user,
                                             spec.concurrency, spec.schedule)
            from polyaxon_amd.polyflow.schedules import PipelineSchedule, Schedule

            sched = Schedule.from_dict(spec.schedule)
            if sched is not None and (sched.periodic or sched.start_at is not None):
                ps = PipelineSchedule(self, pid, spec, proj, user, cwd, sched)
                self.pipelines[pid] = ps
                rid = ps.start()
                return {"kind": "pipeline", "id": pid, "run_id": rid, "next_at": ps.next_at}
            runner = PipelineRunner(self, pid, spec, proj, user, cwd)
            self.pipelines[pid] = runner
            rid = runner.start()
            return {"kind": "pipeline", "id": pid, "run_id": rid}
        raise PolyaxonfileError(f"cannot run kind {spec.kind}")

    # ------------------------------------------------------------------ experiments
    def _create_experiment(self, spec: ExperimentSpecification, proj: Dict, user: str, cwd: str,
                           group_id: Optional[int] = None, name=None, description=None,
                           original_id: Optional[int] = None, strategy: Optional[str] = None,
                           enqueue: bool = True) -> int:
        xid = self.store.create_experiment(
            proj["id"], spec.raw_data, group_id=group_id, user=user, name=name or spec.name, description=description,
            declarations=spec.declarations, tags=spec.tags, original_experiment_id=original_id,
            cloning_strategy=strategy, framework=spec.framework,
            code_reference_id=self._group_code_ref(group_id),
            resources=spec.total_resources.to_dict() if spec.total_resources else None)
        root = self._clone_root(original_id, strategy)
        outputs = self.paths.experiment_outputs(user, proj["name"], root["id"] if root else xid,
                                                root["group_id"] if root else group_id)
        if strategy == "copy" and original_id:
            orig = self.store.get_experiment(original_id)
            outputs = self.paths.experiment_outputs(user, proj["name"], xid, group_id)
            self.paths.prepare_outputs(outputs, "copy", orig["outputs_path"])
        else:
            self.paths.prepare_outputs(outputs, "resume" if strategy == "resume" else None)
        logs = self.paths.experiment_logs(user, proj["name"], xid, group_id)
        os.makedirs(logs, exist_ok=True)
        self.store.update_experiment(xid, outputs_path=outputs, logs_path=logs)
        self.auditor.record("experiment.created", "experiment", xid, user, group=group_id)
        run = Run("experiment", xid, spec, cwd)
        self.runs[run.owner] = run
        if enqueue:
            self._enqueue(run)
        return xid

    def _group_code_ref(self, group_id: Optional[int]) -> Optional[int]:
        if group_id:
            g = self.store.get_group(group_id)
            if g and g.get("code_reference_id"):
                return g["code_reference_id"]
        return getattr(self, "_current_code_ref", None)

    def _clone_root(self, original_id: Optional[int], strategy: Optional[str]) -> Optional[Dict]:
        """Resuming a resumed experiment resumes the root (reference db/models/experiments.py:261-269)."""
        if not original_id or strategy != "resume":
            return None
        x = self.store.get_experiment(original_id)
        while x and x.get("cloning_strategy") == "resume" and x.get("original_experiment_id"):
            x = self.store.get_experiment(x["original_experiment_id"])
        return x

    def _enqueue(self, run: Run) -> None:
        spec = run.spec
        if spec.build is not None and spec.build.build_steps and run.build_id is None:
            bid = self._ensure_build(spec, run)
            if bid is not None:
                run.build_id = bid
                return  # released by the build's completion callback
        self.pending.append(run.owner)

    # ------------------------------------------------------------------ builds (dockerizer equivalent)
    def _build_hash(self, spec: BaseSpecification, cwd: str) -> str:
        b = spec.build
        h = hashlib.sha256(json.dumps({"image": b.image, "steps": b.build_steps, "env": b.env_vars,
                                       "dockerfile": b.dockerfile, "ref": b.ref, "cwd": cwd},
                                      sort_keys=True).encode())
        return h.hexdigest()[:20]

    def _ensure_build(self, spec: BaseSpecification, dependent: Run) -> Optional[int]:
        """Run ``build.build_steps`` once per (image, steps, env) hash, reusing a success within 6 h.
        Returns the build job id the dependent must wait for, or None if a cached build exists."""
        h = self._build_hash(spec, dependent.cwd)
        cached = self.store.last_build_for_hash(h, self.build_reuse_s)
        if cached and not spec.build.nocache:
            dependent.extra_env.update({"PLX_BUILD_DIR": cached["outputs_path"] or ""})
            if dependent.kind == "experiment":
                self.store.update_experiment(dependent.id, build_job_id=cached["id"])
            return None
        owner = next((o for o, r in self.runs.items() if r.kind == "job" and r.spec.kind == Kinds.BUILD
                      and r.extra_env.get("PLX_BUILD_HASH") == h and r.final_status is None), None)
        if owner is None:
            proj = self.store.get("projects", self._project_id(dependent))
            bspec = specification_for({"version": 1, "kind": "build", "build": spec.build.to_dict()})
            bid = self._create_job(bspec, proj, "root", dependent.cwd, build_hash=h)
            owner = f"job:{bid}"
        brun = self.runs[owner]
        if dependent.kind == "experiment":
            self.store.set_experiment_status(dependent.id, "building")
            self.store.update_experiment(dependent.id, build_job_id=brun.id)

        def release(status: str, dep=dependent, brun=brun):
            if status == "succeeded":
                dep.extra_env["PLX_BUILD_DIR"] = self.store.get_job(brun.id)["outputs_path"] or ""
                self.pending.append(dep.owner)
            else:
                self._finish_unstarted(dep, "failed", f"build {brun.id} {status}")

        brun.on_done.append(release)
        return brun.id

    @staticmethod
    def _bind_cpus(pid: int, devs: List[int]) -> None:
        """Pin a replica to the CPUs local to its GPUs (NUMA-near host threads for the HIP
        runtime, RCCL proxies and data loading).  Set right after spawn; the trial's own children inherit it."""
        cpus = set()
        for d in devs:
            cpus.update(device_cpus(d) or [])
        if not cpus:
            return
        try:
            target = cpus & os.sched_getaffinity(0)
            if target:
                os.sched_setaffinity(pid, target)
        except OSError:
            pass

    def _project_id(self, run: Run) -> int:
        rec = self.store.get_experiment(run.id) if run.kind == "experiment" else self.store.get_job(run.id)
        return rec["project_id"]

    # ------------------------------------------------------------------ generic jobs, notebooks, tensorboards
    def _create_job(self, spec: BaseSpecification, proj: Dict, user: str, cwd: str, name=None, description=None,
                    build_hash: Optional[str] = None) -> int:
        jid = self.store.create_job(spec.kind, proj["id"], spec.raw_data, user=user, name=name or spec.name,
                                    description=description, tags=spec.tags,
                                    image=spec.build.image if spec.build else None, image_hash=build_hash)
        kind_dir = {"job": "jobs", "build": "builds", "notebook": "notebooks", "tensorboard": "tensorboards"}[spec.kind]
        outputs = self.paths.job_outputs(user, proj["name"], jid, kind_dir)
        if spec.kind == Kinds.BUILD and build_hash:
            outputs = os.path.join(self.paths.envs_root, build_hash)
        os.makedirs(outputs, exist_ok=True)
        logs = self.paths.job_logs(user, proj["name"], jid, kind_dir)
        os.makedirs(logs, exist_ok=True)
        self.store.update_job(jid, outputs_path=outputs, logs_path=logs)
        subject = {"job": "job", "build": "build_job", "notebook": "notebook", "tensorboard": "tensorboard"}[spec.kind]
        self.auditor.record(f"{subject}.created" if subject in ("job", "build_job") else f"{subject}.started",
                            spec.kind, jid, user)
        run = Run("job", jid, spec, cwd)
        if build_hash:
            run.extra_env["PLX_BUILD_HASH"] = build_hash
        if spec.kind in (Kinds.NOTEBOOK, Kinds.TENSORBOARD):
            run.port = free_port()
            self.store.update_job(jid, port=run.port)
        self.runs[run.owner] = run
        if spec.kind == Kinds.BUILD:
            self.pending.append(run.owner)
        else:
            self._enqueue(run)
        return jid

    def _build_command(self, run: Run) -> str:
        """Dockerizer equivalent (polyflow/dockerizer.py): the Dockerfile is always rendered into the build's
        environment directory; the command either runs the steps natively or builds the image."""
        b = run.spec.build
        rec = self.store.get_job(run.id)
        env_dir = rec["outputs_path"]
        backend = dockerizer.resolve_backend(self.build_backend)
        dockerfile = os.path.join(run.cwd, b.dockerfile) if b.dockerfile else None
        if b.image:
            written = dockerizer.write_dockerfile(env_dir, b.image, b.build_steps, b.env_vars, run.cwd)
            dockerfile = dockerfile or written
        if backend == "native":
            return dockerizer.native_build_command(b.build_steps)
        proj = self.store.get("projects", rec["project_id"])
        tag = dockerizer.tagged_image(proj["name"], proj["id"], run.extra_env.get("PLX_BUILD_HASH") or str(run.id),
                                      self.build_registry)
        self.store.update_job(run.id, image=tag)
        return dockerizer.container_build_command(dockerfile, run.cwd, tag, nocache=b.nocache, push=self.build_push)

    def _job_command(self, run: Run) -> str:
        spec = run.spec
        if spec.kind == Kinds.BUILD:
            return self._build_command(run)
        if spec.kind == Kinds.NOTEBOOK:
            return (f"{self.python} -m jupyter lab --no-browser --ip=127.0.0.1 --port={run.port} "
                    f"--NotebookApp.token={uuid.uuid4().hex} --notebook-dir={run.cwd}")
        if spec.kind == Kinds.TENSORBOARD:
            return f"{self.python} -m tensorboard.main --logdir={self.paths.outputs_root} --port={run.port} --host=127.0.0.1"
        return _command(spec)

    # ================================================================== placement
    def _requirements(self, run: Run) -> List[Tuple[str, int, float]]:
        spec = run.spec
        if run.kind == "job":
            res = spec.resources
            return [("master", 0, float(res.gpu.value) if res and res.gpu else 0.0)]
        cluster, _ = spec.cluster_def
        reqs = []
        for role in ("master", "worker", "ps"):
            for i in range(cluster.get(role, 0)):
                reqs.append((role, i, _replica_gpus(spec, role, i)))
        return reqs

    def _schedule(self) -> None:
        """Place pending runs in FIFO order.  A run that cannot be placed is kept in order; once the oldest
        waiting gang (a multi-device run) has waited ``scheduler.gang_reserve_s``, smaller runs behind it may only
        use devices the gang cannot need (gang reservation -- a stream of 1-GPU trials cannot starve a DP=8 run)."""
        if not self.pending:
            return
        still: Deque[str] = deque()
        reserve = self._gang_reservation()
        try:
            while self.pending:
                owner = self.pending.popleft()
                run = self.runs.get(owner)
                if run is None or run.final_status is not None or run.stop_requested:
                    continue
                try:
                    placed = self._try_place(run, reserve)
                except Exception as e:  # never lose the run (or the queue behind it) to a placement error
                    log.exception("placement of %s failed", owner)
                    self._release_run(run)
                    self._finish_unstarted(run, "failed", f"placement failed: {e}")
                    placed = True
                if not placed:
                    still.append(owner)
        finally:
            still.extend(self.pending)
            self.pending = still
        if self.pending and self._pool is not None:
            self._pool.yield_to_gangs()

    def waiting_gang(self) -> Optional[Tuple[str, int]]:
        """(owner, whole devices) of the oldest pending multi-device run, however long it has waited: idle resident
        executors are released for it at once (polyflow/pool.py ``yield_to_gangs``)."""
        for owner in self.pending:
            run = self.runs.get(owner)
            if run is None or run.final_status is not None:
                continue
            try:
                whole = sum(int(round(g)) for _, _, g in self._requirements(run) if g >= 1.0 - 1e-9)
            except Exception:
                continue
            if whole > 1:
                return owner, whole
        return None

    def _gang_reservation(self) -> Optional[Tuple[str, int]]:
        """(owner, devices) of the gang that holds a reservation, if one has waited long enough."""
        wait = self.settings.get("scheduler.gang_reserve_s") if self.settings is not None else 30.0
        now = time.time()
        for owner in self.pending:
            run = self.runs.get(owner)
            if run is None or run.final_status is not None:
                continue
            try:
                whole = sum(int(round(g)) for _, _, g in self._requirements(run) if g >= 1.0 - 1e-9)
            except Exception:  # a malformed run is failed by _try_place; it never reserves
                continue
            if whole > 1:
                run.waiting_since = run.waiting_since or now
                if now - run.waiting_since >= wait:
                    return owner, whole
                return None  # only the oldest gang may reserve
        return None

    def _try_place(self, run: Run, reserve: Optional[Tuple[str, int]] = None) -> bool:
        reqs = self._requirements(run)
        need = [g for _, _, g in reqs]
        if any(g > self.alloc.n_devices + 1e-9 for g in need) or sum(g for g in need if g >= 1) > self.alloc.n_devices:
            self.cluster_event("failed_scheduling", "warning",
                               f"{run.owner} requests {need} GPUs but the node has {self.alloc.n_devices}",
                               {"owner": run.owner, "requested": need})
            self._finish_unstarted(run, "failed", f"requests {need} GPUs but the node has {self.alloc.n_devices}")
            return True
        if reserve is not None and reserve[0] != run.owner and any(g > 0 for g in need):
            # keep enough whole devices free for the reserved gang: placing this run must leave them idle
            free_whole = len(self.alloc.free_whole())
            mine = sum(int(round(g)) if g >= 1 else 0 for g in need)
            frac = any(0 < g < 1 for g in need)
            if free_whole - mine - (1 if frac and not self._fraction_fits_shared(need) else 0) < reserve[1]:
                return False
        taken: List[str] = []
        devices: List[List[int]] = []
        hbm = run.spec.resources.hbm_gb if run.spec.resources is not None else 0.0
        try:
            for (role, idx, g) in reqs:
                owner = f"{run.owner}:{role}.{idx}"
                a = self.alloc.allocate(owner, g, hbm) if g > 0 else None
                if g > 0 and a is None:
                    for o in taken:
                        self.alloc.release(o)
                    return False
                if a is not None:
                    taken.append(owner)
                devices.append(a.devices if a else [])
        except Exception:
            for o in taken:
                self.alloc.release(o)
            raise
        run.alloc_owners = list(taken)
        self._spawn(run, reqs, devices)
        return True

    def _fraction_fits_shared(self, need) -> bool:
        """Would the run's fractional replicas fit on devices that already have fractional tenants?"""
        for g in need:
            if 0 < g < 1 and not any(d.healthy and 0 < d.share_used and d.share_free >= g - 1e-9
                                     for d in self.alloc.devices):
                return False
        return True

    def _release_run(self, run: Run) -> None:
        """Release every device allocation the run holds (spawn failures, retries, final states)."""
        for o in getattr(run, "alloc_owners", []) or []:
            self.alloc.release(o)
        run.alloc_owners = []

    def _finish_unstarted(self, run: Run, status: str, message: str) -> None:
        run.final_status = status
        run.final_message = message
        if run.kind == "experiment":
            if status == "stopped":
                self.store.set_experiment_status(run.id, "stopped", message)
            else:
                self.store.set_experiment_status(run.id, status, message)
        else:
            self.store.set_job_status(run.id, status, message)
        self._after_done(run, status)

    # ================================================================== spawning
    def _spawn(self, run: Run, reqs, devices) -> None:
        spec = run.spec
        if run.kind == "experiment":
            rec = self.store.get_experiment(run.id)
            self.store.set_experiment_status(run.id, "scheduled")
        else:
            rec = self.store.get_job(run.id)
            self.store.set_job_status(run.id, "scheduled")
        proj = self.store.get("projects", rec["project_id"])
        group = self.store.get_group(rec["group_id"]) if run.kind == "experiment" and rec.get("group_id") else None
        base_port = free_port()
        cluster, _ = spec.cluster_def if run.kind == "experiment" else ({"master": 1}, False)
        cdef = make_cluster_def(spec.framework, cluster, base_port)
        master_port = base_port
        try:
            cmd = self._job_command(run) if run.kind == "job" else _command(spec)
        except PolyaxonfileError as e:
            for role, idx, _ in reqs:
                self.alloc.release(f"{run.owner}:{role}.{idx}")
            self._finish_unstarted(run, "failed", str(e))
            return
        refs = self._refs_outputs(spec)
        data_paths = {name: os.path.join(self.paths.data_root, name)
                      for name in (spec.environment.persistence.get("data") or [])} if spec.environment else {}
        if run.kind == "experiment":
            self.store.set_experiment_status(run.id, "starting")
        local_rank = 0
        for (role, idx, g), devs in zip(reqs, devices):
            if run.kind == "experiment":
                jid = self.store.create_experiment_job(run.id, role, idx, definition={"cmd": cmd},
                                                       resources={"gpu": g}, devices=devs)
            else:
                jid = run.id
            rep = Replica(role, idx, jid, g, devs)
            run.replicas.append(rep)
            env = trial_env(experiment=rec if run.kind == "experiment" else {"id": rec["id"], "uuid": rec["uuid"]},
                            project=proj["name"], user=rec["user"], group=group, role=role, index=idx,
                            framework=spec.framework if run.kind == "experiment" else None, cluster=cdef,
                            devices=devs, outputs_path=rec["outputs_path"], logs_path=rec["logs_path"],
                            declarations=spec.declarations, data_paths=data_paths, refs_outputs=refs,
                            log_level=(spec.logging or {}).get("level"), store_path=self.store_path,
                            api_host=self.api_host, ephemeral_token=uuid.uuid4().hex, master_port=master_port,
                            local_rank=local_rank,
                            hbm_gb=spec.resources.hbm_gb if spec.resources is not None else 0.0, gpu_share=g)
            env.update(run.extra_env)
            env["POLYAXON_RESTART_COUNT"] = str(run.attempt)
            if spec.kind == Kinds.BUILD:
                env["PLX_BUILD_DIR"] = rec["outputs_path"]
            if env.get("PLX_BUILD_DIR"):  # built environments install into <env>/site (pip --target)
                site = os.path.join(env["PLX_BUILD_DIR"], "site")
                env["PYTHONPATH"] = site + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
            for k, v in (spec.build.env_vars if spec.build else []):
                env[str(k)] = str(v)
            for k, v in spec.environment.env_vars if spec.environment else []:
                env[str(k)] = str(v)
            if run.kind == "job":
                env["POLYAXON_JOB_INFO"] = json.dumps({"job_id": rec["id"], "job_uuid": rec["uuid"],
                                                       "kind": spec.kind, "project_name": proj["name"]})
            log_path = self.paths.replica_log(rec["logs_path"], role, idx)
            argv = ["/bin/bash", "-c", cmd]
            if spec.environment is not None and spec.environment.profile and rec.get("outputs_path"):
                prof = profile_argv(cmd, os.path.join(rec["outputs_path"], "rocprof", f"{role}.{idx}"))
                if prof is not None:
                    argv = prof
                else:
                    with open(log_path, "a") as f:
                        f.write("[polyflow] environment.profile: command uses shell syntax, running unprofiled\n")
            try:
                pid = self.pm.spawn(argv, env, cwd=run.cwd, log_path=log_path)
            except OSError as e:
                rep.done = True
                # replicas after this one were never spawned: release their devices now (they have no pid,
                # so no exit will ever release them)
                for (r2, i2, _g2) in reqs[len(run.replicas):]:
                    self.alloc.release(f"{run.owner}:{r2}.{i2}")
                self.alloc.release(f"{run.owner}:{role}.{idx}")
                self.store.add_cluster_event("spawn_failure", "error", f"{run.owner} {role}.{idx}: {e}",
                                             {"owner": run.owner, "role": role, "index": idx})
                self._replica_status(run, rep, "failed", f"spawn failed: {e}")
                run.final_status = "failed"
                run.final_message = f"{role}.{idx} spawn failed: {e}"
                self._stop_run(run, f"replica {role}.{idx} failed to start")
                self._maybe_finalize(run)
                return
            rep.pid = pid
            if devs and self.numa_bind:
                self._bind_cpus(pid, devs)
            self.pid_index[pid] = (run.owner, len(run.replicas) - 1)
            self.stats["spawned"] += 1
            if self._last_exit_t is not None:
                self.stats["gaps_ms"].append((time.time() - self._last_exit_t) * 1000.0)
                self._last_exit_t = None
            if run.kind == "experiment":
                self.store.update_experiment_job(jid, pid=pid)
                self.store.set_experiment_job_status(jid, "scheduled")
                self.store.set_experiment_job_status(jid, "running")
            else:
                self.store.update_job(jid, pid=pid, devices=devs)
                self.store.set_job_status(jid, "running")
            local_rank += 1 if devs else 0
        run.started = time.time()
        self._arm_fault(run)
        if run.kind == "experiment":
            self.store.set_experiment_status(run.id, "running")
            self.auditor.record("experiment.new_status", "experiment", run.id, status="running")
        else:
            self.auditor.record(f"{self._subject(run)}.new_status", run.spec.kind, run.id, status="running")

    def _subject(self, run: Run) -> str:
        return {"job": "job", "build": "build_job", "notebook": "notebook", "tensorboard": "tensorboard"}.get(
            run.spec.kind, "job")

    def _refs_outputs(self, spec: BaseSpecification) -> Dict[str, List[str]]:
        out: Dict[str, List[str]] = {}
        refs = spec.environment.outputs if spec.environment else {}
        for ref in refs.get("experiments", []) or []:
            x = self._resolve_ref("experiments", ref)
            if x:
                out.setdefault("experiments", []).append(x["outputs_path"])
        for ref in refs.get("jobs", []) or []:
            j = self._resolve_ref("jobs", ref)
            if j:
                out.setdefault("jobs", []).append(j["outputs_path"])
        return out

    def _resolve_ref(self, table: str, ref) -> Optional[Dict]:
        """Outputs references by id, name, project.name or user.project.name (reference signals/outputs.py)."""
        if isinstance(ref, int) or (isinstance(ref, str) and ref.isdigit()):
            return self.store.get(table, int(ref))
        parts = str(ref).split(".")
        name = parts[-1]
        rows = self.store.execute(f"SELECT * FROM {table} WHERE name = ? ORDER BY id DESC", (name,)).fetchall()
        return self.store._row(rows[0]) if rows else None

    # ================================================================== exits and aggregation
    def _replica_status(self, run: Run, rep: Replica, status: str, message: Optional[str] = None) -> None:
        if run.kind == "experiment":
            self.store.set_experiment_job_status(rep.job_id, status, message)
            self.store.update_experiment_job(rep.job_id, exit_code=rep.exit_code)
        else:
            self.store.update_job(rep.job_id, exit_code=rep.exit_code)

    def _on_exit(self, pid: int, status: int) -> None:
        self.stats["exited"] += 1
        self._last_exit_t = time.time()
        key = self.pid_index.pop(pid, None)
        if key is None:
            return
        owner, ri = key
        run = self.runs.get(owner)
        if run is None:
            return
        rep = run.replicas[ri]
        rep.done = True
        rep.exit_code = status
        self.alloc.release(f"{run.owner}:{rep.role}.{rep.index}")
        if run.stop_requested:
            # replicas torn down after the master succeeded count as succeeded ("Master is done.")
            jstatus = "succeeded" if run.final_status == "succeeded" else "stopped"
            self._replica_status(run, rep, jstatus, run.stop_reason)
        elif status == 0:
            self._replica_status(run, rep, "succeeded")
            if rep.role == "master":
                run.final_status = "succeeded"  # master done wins (reference db/models/experiments.py:175-183)
                self._stop_run(run, "Master is done.")
        else:
            msg = f"exit code {status}" if status > 0 else f"killed by signal {-status}"
            self._replica_event(run, rep, status)
            self._replica_status(run, rep, "failed", msg)
            run.final_status = "failed"
            run.final_message = f"{rep.role}.{rep.index} {msg}"
            self._stop_run(run, f"replica {rep.role}.{rep.index} failed")
        self._maybe_finalize(run)

    def _replica_event(self, run: Run, rep: Replica, status: int) -> None:
        """Cluster events for abnormal replica exits (the k8s events the reference's namespace monitor records:
        OOMKilled, Error): an unrequested SIGKILL (the kernel OOM killer's signal), and a GPU fault the HIP runtime
        printed into the replica's log (page fault / illegal address / hang)."""
        from polyaxon_amd.obs.nodes import gpu_fault_in_log

        rec = self.store.get_experiment(run.id) if run.kind == "experiment" else self.store.get_job(run.id)
        logs = rec.get("logs_path") if rec else None
        fault = gpu_fault_in_log(self.paths.replica_log(logs, rep.role, rep.index)) if logs else None
        data = {"owner": run.owner, "replica": f"{rep.role}.{rep.index}", "devices": rep.devices, "status": status}
        if fault:
            self.cluster_event("gpu_fault", "error", f"{run.owner} {rep.role}.{rep.index} on devices "
                                                     f"{rep.devices}: {fault}", data)
        elif status == -signal.SIGKILL:
            self.cluster_event("process_killed", "warning", f"{run.owner} {rep.role}.{rep.index} killed by SIGKILL "
                                                            "(not requested by polyflow; OOM killer?)", data)
        elif status < 0:
            self.cluster_event("process_killed", "warning",
                               f"{run.owner} {rep.role}.{rep.index} killed by signal {-status}", data)

    def _maybe_finalize(self, run: Run) -> None:
        if any(not r.done for r in run.replicas):
            return
        self._release_run(run)
        if run.final_status is None:
            run.final_status = "stopped" if run.stop_requested else "succeeded"
        status = run.final_status
        if status == "failed" and self._maybe_retry(run):
            return
        if run.kind == "experiment":
            # remaining replicas that were stopped because the master finished count as succeeded
            self.store.set_experiment_status(run.id, status, run.final_message)
            self.auditor.record(f"experiment.{'done' if status == 'stopped' else status}", "experiment", run.id,
                                status=status)
        else:
            self.store.set_job_status(run.id, status, run.final_message)
            subj = self._subject(run)
            ev = f"{subj}.{status}" if status in ("succeeded", "failed") else f"{subj}.stopped"
            self.auditor.record(ev, run.spec.kind, run.id, status=status)
        self._after_done(run, status)

    def _after_done(self, run: Run, status: str) -> None:
        for cb in run.on_done:
            try:
                cb(status)
            except Exception:
                log.exception("on_done callback failed")
        if run.kind == "experiment":
            rec = self.store.get_experiment(run.id)
            gid = rec.get("group_id") if rec else None
            if gid in self.groups:
                self.groups[gid].on_experiment_done(run.id, status)

    # ================================================================== failure handling
    def _max_restarts(self, run: Run) -> int:
        env = getattr(run.spec, "environment", None)
        if run.kind != "experiment":
            return 0
        n = int(getattr(env, "max_restarts", 0) or 0)
        return n or (int(self.settings.get("scheduler.max_restarts")) if self.settings is not None else 0)

    def _maybe_retry(self, run: Run) -> bool:
        """Opt-in retry: a failed experiment is re-queued whole (all replicas, fresh rendezvous port) up to
        ``environment.max_restarts`` times; POLYAXON_RESTART_COUNT tells the trial which attempt it is."""
        if run.attempt >= self._max_restarts(run):
            return False
        run.attempt += 1
        self.stats["retries"] += 1
        msg = f"retry {run.attempt}/{self._max_restarts(run)} after: {run.final_message}"
        self.store.set_experiment_status(run.id, "retrying", msg)
        self.auditor.record("experiment.new_status", "experiment", run.id, status="retrying")
        run.replicas = []
        run.stop_requested = False
        run.stop_reason = None
        run.final_status = None
        run.final_message = None
        run.started = None
        self.pending.append(run.owner)
        return True

    def _arm_fault(self, run: Run) -> None:
        """Fault injection for tests: ``POLYFLOW_FAULT=kill_rank:R@t:SECONDS`` SIGKILLs replica R of the
        first attempt that long after spawn (``@step:N`` is handled by the tracking client inside the trial)."""
        fault = run.extra_env.get("POLYFLOW_FAULT") or dict(
            (str(k), str(v)) for k, v in (run.spec.environment.env_vars if run.spec.environment else [])
        ).get("POLYFLOW_FAULT")
        if not fault or run.attempt > 0:
            return
        spec = parse_fault(fault)
        if spec is None or spec["at"] != "t":
            return
        replicas = list(run.replicas)

        def fire():
            if spec["rank"] < len(replicas):
                r = replicas[spec["rank"]]
                if r.pid is not None and not r.done:
                    self.stats["faults_injected"] += 1
                    self.pm.signal(r.pid, signal.SIGKILL, group=True)

        self.after(spec["value"], fire)

    def _reconcile(self) -> None:
        """Periodic health pass (the reference's 30 s cron, crons/tasks/experiments.py:9-17, event-driven
        here except for what cannot raise an event): heartbeat deadlines of hung trials and GPU health."""
        try:
            now = time.time()
            for run in list(self.runs.values()):
                if run.kind != "experiment" or not run.active or run.stop_requested or run.started is None:
                    continue
                env = run.spec.environment
                timeout = getattr(env, "heartbeat_timeout", None) if env else None
                if not timeout and self.settings is not None:
                    timeout = self.settings.get("scheduler.heartbeat_timeout_s") or None
                if not timeout:
                    continue
                last = self.store.kv_get(f"heartbeat:experiment:{run.id}")
                last = max(float(last), run.started) if last else run.started
                if now - last > timeout:
                    self.stats["heartbeat_kills"] += 1
                    run.final_status = "failed"
                    run.final_message = f"no heartbeat for {now - last:.1f}s (timeout {timeout}s)"
                    self._stop_run(run, run.final_message)
            if self.health_check is not None:
                for idx in self.health_check() or []:
                    if idx < self.alloc.n_devices and idx not in self._unhealthy:
                        self._unhealthy.add(idx)
                        self.alloc.mark_unhealthy(idx)
                        self.auditor.record("cluster.node_gpu_unhealthy", "cluster", None, device=idx)
            keep = self.settings.get("scheduler.clean_after_s") if self.settings is not None else 0
            if keep and now - getattr(self, "_last_clean", 0.0) > 600.0:  # outputs retention, at most every 10 min
                from polyaxon_amd.polyflow.cleaning import clean_outputs

                self._last_clean = now
                removed = clean_outputs(self.store, keep)
                if removed:
                    log.info("outputs retention removed %d paths", len(removed))
        except Exception:
            log.exception("reconcile failed")
        finally:
            if self._running and self.reconcile_s > 0:
                self.after(self.reconcile_s, self._reconcile)

    # ================================================================== stopping
    def _stop_run(self, run: Run, reason: str) -> None:
        """SIGTERM every live replica's process group now, SIGKILL whatever is left after the grace period."""
        run.stop_requested = True
        run.stop_reason = reason
        live = [r for r in run.replicas if r.pid is not None and not r.done]
        for r in live:
            self.pm.signal(r.pid, signal.SIGTERM, group=True)
        if live:
            pids = [r.pid for r in live]

            def kill(pids=pids, run=run):
                for r in run.replicas:
                    if r.pid in pids and not r.done:
                        self.pm.signal(r.pid, signal.SIGKILL, group=True)

            self.after(self.stop_grace_s, kill)

    def _stop(self, kind: str, id_: int, message: str = "Stopped by user.") -> bool:
        run = self.runs.get(f"{kind}:{id_}")
        if run is None or run.final_status is not None and not run.active:
            return False
        if not run.replicas:  # never placed
            self._finish_unstarted(run, "stopped", message)
            return True
        if run.final_status is None:
            run.final_status = "stopped"
            run.final_message = message
        self._stop_run(run, message)
        return True

    def stop_experiment(self, xid: int, message: str = "Stopped by user.") -> bool:
        self.auditor.record("experiment.stopped_triggered", "experiment", xid)
        return self.call(self._stop, "experiment", xid, message)

    def stop_job(self, jid: int) -> bool:
        return self.call(self._stop, "job", jid, "Stopped by user.")

    def stop_group(self, gid: int, pending: bool = False, message: str = "Stopped by user.") -> None:
        self.auditor.record("experiment_group.stopped_triggered", "experiment_group", gid)
        self.call(self._stop_group, gid, pending, message)

    def stop_pipeline(self, pid: int) -> bool:
        """Stop a pipeline: its running run(s) and, for a scheduled pipeline, every future firing."""
        def stop():
            p = self.pipelines.get(pid)
            if p is None:
                return False
            p.stop()
            return True

        return self.call(stop)

    def _stop_group(self, gid: int, pending: bool, message: str) -> None:
        driver = self.groups.get(gid)
        if driver is not None:
            driver.stop(pending_only=pending, message=message)

    def _stop_all(self) -> None:
        for run in list(self.runs.values()):
            if run.final_status is None or run.active:
                if run.replicas:
                    if run.final_status is None:
                        run.final_status = "stopped"
                    self._stop_run(run, "Scheduler shutdown.")
                elif run.final_status is None:
                    self._finish_unstarted(run, "stopped", "Scheduler shutdown.")

    # ================================================================== cloning: restart / resume / copy
    def clone_experiment(self, xid: int, strategy: str, declarations: Optional[Dict[str, Any]] = None,
                         content=None) -> int:
        """Reference Experiment.restart/resume/copy (db/models/experiments.py:225-316)."""
        if strategy not in ("restart", "resume", "copy"):
            raise ValueError(f"unknown cloning strategy {strategy}")
        return self.call(self._clone, xid, strategy, declarations, content)

    def _clone(self, xid: int, strategy: str, declarations, content, group_id=None, enqueue: bool = True) -> int:
        """``enqueue=False``: a group driver's promotion -- the driver starts it from its own queue (bounded by the
        group's concurrency); enqueuing it here as well would place the same run twice."""
        orig = self.store.get_experiment(xid)
        if orig is None:
            raise KeyError(f"experiment {xid} not found")
        raw = dict(content) if content is not None else dict(orig["config"])
        if declarations:
            raw["declarations"] = dict(raw.get("declarations") or {}, **declarations)
        spec = ExperimentSpecification(raw)
        proj = self.store.get("projects", orig["project_id"])
        old = self.runs.get(f"experiment:{xid}")
        cwd = old.cwd if old else os.getcwd()
        new = self._create_experiment(spec, proj, orig["user"], cwd,
                                      group_id=orig["group_id"] if group_id is None else group_id,
                                      original_id=xid, strategy=strategy, enqueue=enqueue)
        self.auditor.record(f"experiment.{ {'restart': 'restarted', 'resume': 'resumed', 'copy': 'copied'}[strategy]}",
                            "experiment", new, original=xid)
        return new

    # ================================================================== queries / waiting
    def wait(self, kind: str, id_: int, timeout: Optional[float] = None, poll_s: float = 0.02) -> str:
        end = None if timeout is None else time.time() + timeout
        while True:
            if kind == "experiment":
                rec = self.store.get_experiment(id_)
                st = rec["status"]
                done = ExperimentLifeCycle.is_done(st)
            elif kind == "group":
                rec = self.store.get_group(id_)
                st = rec["status"]
                done = st in ("succeeded", "failed", "stopped")
            elif kind == "pipeline_run":
                rec = self.store.get("pipeline_runs", id_)
                st = rec["status"]
                done = st in ("finished", "stopped", "skipped")
            else:
                rec = self.store.get_job(id_)
                st = rec["status"]
                done = JobLifeCycle.is_done(st)
            if done:
                return st
            if end is not None and time.time() > end:
                raise TimeoutError(f"{kind} {id_} still {st}")
            time.sleep(poll_s)

    def wait_idle(self, timeout: float = 60.0) -> None:
        end = time.time() + timeout
        while time.time() < end:
            busy = self.call(lambda: any(r.active for r in self.runs.values()) or bool(self.pending)
                             or any(not d.done for d in self.groups.values()))
            if not busy:
                return
            time.sleep(0.02)
        raise TimeoutError("scheduler did not become idle")

    def running_experiments(self) -> List[int]:
        return self.call(lambda: [r.id for r in self.runs.values() if r.kind == "experiment" and r.active])

    def logs(self, kind: str, id_: int, tail: Optional[int] = None) -> str:
        """Experiment logs = every replica log prefixed ``role.index -- `` (reference events_handlers/tasks/logs.py)."""
        if kind == "experiment":
            rec = self.store.get_experiment(id_)
            out = []
            for j in self.store.experiment_jobs(id_):
                path = self.paths.replica_log(rec["logs_path"], j["role"], j["idx"])
                for line in Paths.read_log(path).splitlines():
                    out.append(f"{j['role']}.{j['idx']} -- {line}")
            lines = out
        else:
            rec = self.store.get_job(id_)
            lines = Paths.read_log(self.paths.replica_log(rec["logs_path"], "master", 0)).splitlines()
        if tail:
            lines = lines[-tail:]
        return "\n".join(lines)


class _Result:
    def __init__(self):
        self._ev = threading.Event()
        self._val = None
        self._err: Optional[BaseException] = None

    def set(self, v):
        self._val = v
        self._ev.set()

    def fail(self, e: BaseException):
        self._err = e
        self._ev.set()

    def get(self, timeout: Optional[float]):
        if not self._ev.wait(timeout):
            raise TimeoutError("polyflow command timed out")
        if self._err is not None:
            raise self._err
        return self._val
