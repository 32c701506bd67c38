"""In-trial tracking client + helper getters (reference external polyaxon-client/tracking and
polyaxon-helper; contract in docs/templates/polyaxon_tracking/experiments.md and
docs/templates/polyaxon_tracking/polyaxon_helper.md:47-141).

``Experiment()`` inside a polyflow trial picks up its identity from the env contract (polyflow/env.py) and
writes to the node's tracking store directly (``POLYAXON_STORE_PATH``, SQLite/WAL — no HTTP hop, no
20 req/s throttle as in the reference's api/experiments/views.py:389) or, if only
``POLYAXON_API_HTTP_HOST`` is set, through the REST API.  Outside a cluster it can also create a
local experiment in a store of your choice (``Experiment(project=..., store_path=...)``).

Metric values may be Python numbers or (GPU) tensors: tensors are handed to :class:`MetricStream`, which
copies them device→pinned host on a low-priority side stream, records an event, and lets a background
thread write the batch to the store once the event completes — the training stream never synchronises.
"""
from __future__ import annotations

import json
import os
import sys
import signal
import threading
import time
import urllib.request
from typing import Any, Dict, List, Optional


# ------------------------------------------------------------------ helper getters (polyaxon-helper API)
def _env_json(name: str, default=None):
    v = os.environ.get(name)
    if v is None:
        return default
    try:
        return json.loads(v)
    except ValueError:
        return default


def get_cluster_def() -> Optional[Dict[str, List[str]]]:
    return _env_json("POLYAXON_CLUSTER")


def get_declarations() -> Optional[Dict[str, Any]]:
    return _env_json("POLYAXON_DECLARATIONS")


def get_experiment_info() -> Optional[Dict[str, Any]]:
    return _env_json("POLYAXON_EXPERIMENT_INFO")


def get_job_info() -> Optional[Dict[str, Any]]:
    return _env_json("POLYAXON_JOB_INFO")


def get_task_info() -> Optional[Dict[str, Any]]:
    return _env_json("POLYAXON_TASK_INFO")


def get_task_type() -> Optional[str]:
    info = get_task_info()
    return info.get("type") if info else None


def get_task_index() -> Optional[int]:
    info = get_task_info()
    return info.get("index") if info else None


def get_outputs_path() -> Optional[str]:
    return os.environ.get("POLYAXON_RUN_OUTPUTS_PATH")


def get_log_level() -> Optional[str]:
    return os.environ.get("POLYAXON_LOG_LEVEL")


def get_data_paths() -> Optional[Dict[str, str]]:
    return _env_json("POLYAXON_RUN_DATA_PATHS")


def get_outputs_refs_paths() -> Optional[Dict[str, List[str]]]:
    return _env_json("POLYAXON_REFS_OUTPUTS_PATHS")


def get_tf_config(envvar: str = "TF_CONFIG") -> Optional[Dict[str, Any]]:
    return _env_json(envvar)


def is_in_cluster() -> bool:
    return os.environ.get("POLYAXON_IN_CLUSTER", "").lower() in ("1", "true")


# ------------------------------------------------------------------ backends
class _StoreBackend:
    def __init__(self, path: str):
        from polyaxon_amd.store import Store

        self.store = Store(path)

    def log_metrics(self, xid: int, rows):
        self.store.add_metrics_batch([(xid, vals, step, ts) for vals, step, ts in rows])

    def update(self, xid: int, **values):
        rec = self.store.get_experiment(xid)
        if "declarations" in values:
            values["declarations"] = dict(rec["declarations"] or {}, **values["declarations"])
        if "tags" in values:
            values["tags"] = sorted(set(rec["tags"] or []) | set(values["tags"]))
        self.store.update_experiment(xid, **values)

    def status(self, xid: int, status: str, message: Optional[str] = None):
        self.store.set_experiment_status(xid, status, message)

    def heartbeat(self, xid: int):
        self.store.kv_set(f"heartbeat:experiment:{xid}", time.time())


class _HttpBackend:
    def __init__(self, host: str, token: Optional[str], project: str, user: str):
        self.host = host.rstrip("/")
        self.token = token
        self.base = f"{self.host}/api/v1/{user}/{project}"

    def _req(self, method: str, path: str, payload=None):
        data = json.dumps(payload).encode() if payload is not None else None
        req = urllib.request.Request(self.base + path, data=data, method=method,
                                     headers={"Content-Type": "application/json",
                                              **({"Authorization": f"token {self.token}"} if self.token else {})})
        with urllib.request.urlopen(req, timeout=10) as r:
            return json.loads(r.read() or b"null")

    def log_metrics(self, xid: int, rows):
        self._req("POST", f"/experiments/{xid}/metrics",
                  [{"values": vals, "step": step, "created_at": ts} for vals, step, ts in rows])

    def update(self, xid: int, **values):
        self._req("PATCH", f"/experiments/{xid}", values)

    def status(self, xid: int, status: str, message: Optional[str] = None):
        self._req("POST", f"/experiments/{xid}/statuses", {"status": status, "message": message})

    def heartbeat(self, xid: int):
        self._req("POST", f"/experiments/{xid}/heartbeat", {})


class MetricStream:
    """Asynchronous device -> store metric path.

    Device tensors are gathered into one staging vector and copied device->host on a dedicated LOW-priority side
    stream (``Stream.priority_range()[0]``) into a **preallocated pinned ring** (``ring_floats`` fp32 slots,
    allocated once), with one event per ``log_metrics`` call; the training stream never waits.  A flusher thread
    turns rows whose copy event has completed into store writes.  When the ring is full, the oldest pending rows
    are flushed first (their events synchronised), so the ring never grows and nothing is dropped."""

    def __init__(self, sink, xid: int, flush_every_s: float = 0.5, ring_floats: int = 4096):
        self.sink = sink
        self.xid = xid
        self.flush_every_s = flush_every_s
        self.ring_floats = int(ring_floats)
        self._ring = None          # pinned fp32 [ring_floats]
        self._head = 0             # next free slot (monotonic; slot = head % ring_floats)
        self._tail = 0             # oldest slot still referenced by a pending row
        # end of the newest row registered in _pending: slots past it may be reserved by a put() still enqueueing
        # its copy, so an empty queue frees the ring only up to here (not up to _head)
        self._committed = 0
        # (event|None, {name: float | (offset, numel)}, step, ts, end_offset)
        self._pending: List = []
        self._lock = threading.Lock()
        self._flush_lock = threading.Lock()  # taking rows and writing them is one step: the sink sees FIFO order
        self._stop = threading.Event()
        self._side = None
        self._thread = threading.Thread(target=self._run, name="plx-metrics", daemon=True)
        self._thread.start()

    def _stream_for(self, t):
        import torch

        if self._side is None:
            low = torch.cuda.Stream.priority_range()[0]  # least priority: never delays the training kernels
            self._side = torch.cuda.Stream(device=t.device, priority=low)
            self._ring = torch.empty(self.ring_floats, dtype=torch.float32, pin_memory=True)
        return self._side

    def _reserve(self, n: int) -> int:
        """Offset of n contiguous ring slots (wrapping to the start when the tail end is too short)."""
        if n > self.ring_floats:
            raise ValueError(f"metric tensors of {n} elements exceed the {self.ring_floats}-float ring")
        while True:
            with self._lock:
                off = self._head % self.ring_floats
                skip = 0 if off + n <= self.ring_floats else self.ring_floats - off
                if self._head + skip + n - self._tail <= self.ring_floats:
                    self._head += skip
                    start = self._head
                    self._head += n
                    return start
            self.flush(force=True, oldest_only=True)  # ring full: drain the oldest rows first

    def put(self, values: Dict[str, Any], step: Optional[int]) -> None:
        ts = time.time()
        host: Dict[str, Any] = {}
        event = None
        end = None
        tensors = {k: v for k, v in values.items() if hasattr(v, "is_cuda") and v.is_cuda}
        if tensors:
            import torch

            first = next(iter(tensors.values()))
            side = self._stream_for(first)
            sizes = [v.numel() for v in tensors.values()]
            start = self._reserve(sum(sizes))
            off = start % self.ring_floats
            side.wait_stream(torch.cuda.current_stream(first.device))
            with torch.cuda.stream(side):
                flat = torch.cat([v.detach().reshape(-1).float() for v in tensors.values()])  # one gather kernel
                self._ring[off: off + flat.numel()].copy_(flat, non_blocking=True)      # one D2H copy
                for v in tensors.values():
                    v.record_stream(side)
                event = torch.cuda.Event()
                event.record(side)
            o = off
            for (k, _), n in zip(tensors.items(), sizes):
                host[k] = (o, n)
                o += n
            end = start + sum(sizes)
        for k, v in values.items():
            if k not in host:
                host[k] = float(v.item()) if hasattr(v, "item") else float(v)
        with self._lock:
            self._pending.append((event, host, step, ts, end))
            if end is not None:
                self._committed = max(self._committed, end)

    def _ready_rows(self, force: bool, oldest_only: bool = False):
        rows, keep = [], []
        with self._lock:
            for i, (ev, host, step, ts, end) in enumerate(self._pending):
                if keep or (ev is not None and not force and not ev.query()) or (oldest_only and rows):
                    keep.append((ev, host, step, ts, end))  # keep FIFO order: the ring is freed front to back
                    continue
                if ev is not None:
                    ev.synchronize()
                vals = {}
                for k, v in host.items():
                    if isinstance(v, tuple):
                        o, n = v
                        vals[k] = float(self._ring[o])  # metrics are scalars: first element
                    else:
                        vals[k] = v
                rows.append((vals, step, ts))
                if end is not None:
                    self._tail = end
            self._pending = keep
            if not keep:
                self._tail = max(self._tail, self._committed)
        return rows

    def flush(self, force: bool = True, oldest_only: bool = False) -> None:
        with self._flush_lock:
            rows = self._ready_rows(force, oldest_only)
            if rows:
                self.sink.log_metrics(self.xid, rows)

    def _run(self) -> None:
        while not self._stop.wait(self.flush_every_s):
            try:
                self.flush(force=False)
            except Exception:
                pass

    def close(self) -> None:
        self._stop.set()
        self._thread.join(timeout=5)
        self.flush(force=True)


def _step_fault() -> Optional[int]:
    """Step of a ``POLYFLOW_FAULT=kill_rank:R@step:N`` targeting this replica on its first attempt."""
    text = os.environ.get("POLYFLOW_FAULT")
    if not text or os.environ.get("POLYAXON_RESTART_COUNT", "0") != "0":
        return None
    from polyaxon_amd.polyflow.faults import parse_fault

    f = parse_fault(text)
    if f is None or f["at"] != "step" or int(os.environ.get("RANK", "0")) != f["rank"]:
        return None
    return int(f["value"])


class Experiment:
    """Tracking handle (reference ``polyaxon_client.tracking.Experiment``)."""

    def __init__(self, experiment_id: Optional[int] = None, project: Optional[str] = None,
                 store_path: Optional[str] = None, api_host: Optional[str] = None, token: Optional[str] = None,
                 user: str = "root", track: bool = True, async_metrics: bool = True):
        self.experiment_id = experiment_id or (int(os.environ["POLYAXON_EXPERIMENT_ID"])
                                               if os.environ.get("POLYAXON_EXPERIMENT_ID") else None)
        info = get_experiment_info() or {}
        self.project = project or (info.get("project_name", "").split(".")[-1] or None)
        self.user = user
        store_path = store_path or os.environ.get("POLYAXON_STORE_PATH")
        api_host = api_host or os.environ.get("POLYAXON_API_HTTP_HOST")
        self.backend = None
        if track and store_path:
            self.backend = _StoreBackend(store_path)
            if self.experiment_id is None:  # local, outside polyflow
                st = self.backend.store
                proj = st.get_or_create_project(self.project or "default", user)
                self.experiment_id = st.create_experiment(proj["id"], {}, user=user, is_managed=False)
                st.set_experiment_status(self.experiment_id, "scheduled")
                st.set_experiment_status(self.experiment_id, "running")
        elif track and api_host and self.experiment_id is not None:
            self.backend = _HttpBackend(api_host, token or os.environ.get("POLYAXON_SECRET_USER_TOKEN"),
                                        self.project or "default", user)
        self._stream = MetricStream(self.backend, self.experiment_id) if (self.backend and async_metrics) else None
        self._done = False
        self._last_beat = 0.0
        self._fault = _step_fault()
        if "torch" in sys.modules:  # a GPU trial: enforce the replica's HBM reservation (client/budget.py)
            from polyaxon_amd.client.budget import apply_hbm_budget

            try:
                apply_hbm_budget()
            except Exception:  # no device visible / runtime not usable: nothing to cap
                pass

    # ------------------------------------------------------------------ properties
    @property
    def outputs_path(self) -> Optional[str]:
        return get_outputs_path()

    def get_outputs_path(self) -> Optional[str]:
        return self.outputs_path

    def get_cluster_def(self):
        return get_cluster_def()

    def get_declarations(self):
        return get_declarations()

    def get_data_paths(self):
        return get_data_paths()

    def get_outputs_refs_paths(self):
        return get_outputs_refs_paths()

    # ------------------------------------------------------------------ logging
    def heartbeat(self, force: bool = True) -> None:
        """Liveness signal read by the scheduler's ``environment.heartbeat_timeout`` deadline."""
        now = time.time()
        if self.backend is None or (not force and now - self._last_beat < 1.0):
            return
        self._last_beat = now
        try:
            self.backend.heartbeat(self.experiment_id)
        except Exception:  # a missed beat must never kill the trial
            pass

    def log_metrics(self, step: Optional[int] = None, **metrics) -> None:
        if self._fault is not None and step is not None and step >= self._fault:
            os.kill(os.getpid(), signal.SIGKILL)  # POLYFLOW_FAULT=kill_rank:R@step:N (tests only)
        if self.backend is None:
            return
        self.heartbeat(force=False)
        if self._stream is not None:
            self._stream.put(metrics, step)
        else:
            vals = {k: float(v.item()) if hasattr(v, "item") else float(v) for k, v in metrics.items()}
            self.backend.log_metrics(self.experiment_id, [(vals, step, time.time())])

    def log_params(self, **params) -> None:
        if self.backend is not None:
            self.backend.update(self.experiment_id, declarations=params)

    log_declarations = log_params

    def log_tags(self, tags) -> None:
        if self.backend is not None:
            self.backend.update(self.experiment_id, tags=list(tags))

    def set_description(self, description: str) -> None:
        if self.backend is not None:
            self.backend.update(self.experiment_id, description=description)

    def set_name(self, name: str) -> None:
        if self.backend is not None:
            self.backend.update(self.experiment_id, name=name)

    def log_status(self, status: str, message: Optional[str] = None) -> None:
        if self.backend is not None:
            self.backend.status(self.experiment_id, status, message)

    def log_run_env(self, env: Dict[str, Any]) -> None:
        if self.backend is not None:
            self.backend.update(self.experiment_id, run_env=env)

    def flush(self) -> None:
        if self._stream is not None:
            self._stream.flush(force=True)

    def succeeded(self) -> None:
        self._finish("succeeded")

    def failed(self, message: Optional[str] = None) -> None:
        self._finish("failed", message)

    def _finish(self, status: str, message: Optional[str] = None) -> None:
        self.close()
        if self.backend is not None and isinstance(self.backend, _StoreBackend):
            rec = self.backend.store.get_experiment(self.experiment_id)
            if not rec.get("is_managed"):
                self.log_status(status, message)

    def close(self) -> None:
        if self._stream is not None and not self._done:
            self._stream.close()
        self._done = True

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        if exc_type is None:
            self.succeeded()
        else:
            self.failed(str(exc))

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
