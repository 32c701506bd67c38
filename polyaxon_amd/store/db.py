"""Tracking store: one SQLite database (WAL) holding every entity the reference keeps in Postgres + Redis.

Reference: polyaxon/db/models/*.py (Experiment, ExperimentMetric, ExperimentJob, ExperimentGroup,
ExperimentGroupIteration, Job, BuildJob, Notebook/Tensorboard jobs, Pipeline/Operation runs, Project,
ClusterNode/NodeGPU, ActivityLog, Notification, Bookmark, Search, CodeReference, ClusterEvent) and the
ephemeral Redis state (polyaxon/db/redis/*.py).  Status changes go through the lifecycle FSMs
(``can_transition``; reference db/models/abstract_jobs.py:30-47, statuses.py:42-85) and keep the full
history; metrics keep the full history plus the merged ``last_metric`` the HPO code reads
(reference signals/experiments.py:192-208).

Single node, many writers (scheduler loop, API threads, trial processes writing metrics directly): WAL
journal + ``busy_timeout`` give concurrent readers and serialised short writers; every connection is
thread-local.  JSON columns are stored as TEXT and decoded on read.
"""
from __future__ import annotations

import json
import math
import os
import sqlite3
import threading
import time
import uuid as uuidlib
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

from polyaxon_amd.fsm import (ExperimentGroupLifeCycle, ExperimentLifeCycle, JobLifeCycle, OperationLifeCycle,
                              PipelineLifeCycle)

SCHEMA = """
CREATE TABLE IF NOT EXISTS users (id INTEGER PRIMARY KEY, username TEXT UNIQUE, email TEXT, is_superuser INTEGER
    DEFAULT 0, token TEXT UNIQUE, created_at REAL);
CREATE TABLE IF NOT EXISTS projects (id INTEGER PRIMARY KEY, uuid TEXT, user TEXT, name TEXT, description TEXT,
    is_public INTEGER DEFAULT 1, tags TEXT, created_at REAL, updated_at REAL, UNIQUE(user, name));
CREATE TABLE IF NOT EXISTS code_references (id INTEGER PRIMARY KEY, commit_sha TEXT, branch TEXT, git_url TEXT,
    is_dirty INTEGER, diff TEXT, created_at REAL);
CREATE TABLE IF NOT EXISTS experiment_groups (id INTEGER PRIMARY KEY, uuid TEXT, project_id INTEGER, user TEXT,
    name TEXT, description TEXT, content TEXT, hptuning TEXT, tags TEXT, status TEXT, search_algorithm TEXT,
    concurrency INTEGER, code_reference_id INTEGER, created_at REAL, updated_at REAL, started_at REAL,
    finished_at REAL);
CREATE TABLE IF NOT EXISTS experiment_group_statuses (id INTEGER PRIMARY KEY, group_id INTEGER, status TEXT,
    message TEXT, created_at REAL);
CREATE TABLE IF NOT EXISTS experiment_group_iterations (id INTEGER PRIMARY KEY, group_id INTEGER, data TEXT,
    created_at REAL, updated_at REAL);
CREATE TABLE IF NOT EXISTS experiments (id INTEGER PRIMARY KEY, uuid TEXT, project_id INTEGER, group_id INTEGER,
    user TEXT, name TEXT, description TEXT, config TEXT, declarations TEXT, tags TEXT, status TEXT,
    last_metric TEXT, original_experiment_id INTEGER, cloning_strategy TEXT, code_reference_id INTEGER,
    build_job_id INTEGER, framework TEXT, resources TEXT, run_env TEXT, outputs_path TEXT, logs_path TEXT,
    is_managed INTEGER DEFAULT 1, created_at REAL, updated_at REAL, started_at REAL, finished_at REAL);
CREATE INDEX IF NOT EXISTS ix_xp_group ON experiments(group_id);
CREATE INDEX IF NOT EXISTS ix_xp_project ON experiments(project_id);
CREATE TABLE IF NOT EXISTS experiment_statuses (id INTEGER PRIMARY KEY, experiment_id INTEGER, status TEXT,
    message TEXT, traceback TEXT, created_at REAL);
CREATE INDEX IF NOT EXISTS ix_xps_xp ON experiment_statuses(experiment_id);
CREATE TABLE IF NOT EXISTS experiment_metrics (id INTEGER PRIMARY KEY, experiment_id INTEGER, step INTEGER,
    "values" TEXT, created_at REAL);
CREATE INDEX IF NOT EXISTS ix_xpm_xp ON experiment_metrics(experiment_id);
CREATE TABLE IF NOT EXISTS experiment_jobs (id INTEGER PRIMARY KEY, uuid TEXT, experiment_id INTEGER, role TEXT,
    idx INTEGER, status TEXT, definition TEXT, resources TEXT, devices TEXT, pid INTEGER, exit_code INTEGER,
    node TEXT, created_at REAL, updated_at REAL, started_at REAL, finished_at REAL);
CREATE INDEX IF NOT EXISTS ix_xpj_xp ON experiment_jobs(experiment_id);
CREATE TABLE IF NOT EXISTS experiment_job_statuses (id INTEGER PRIMARY KEY, job_id INTEGER, status TEXT,
    message TEXT, details TEXT, created_at REAL);
CREATE TABLE IF NOT EXISTS jobs (id INTEGER PRIMARY KEY, uuid TEXT, kind TEXT, project_id INTEGER, user TEXT,
    name TEXT, description TEXT, config TEXT, tags TEXT, status TEXT, original_job_id INTEGER,
    cloning_strategy TEXT, code_reference_id INTEGER, build_job_id INTEGER, dockerfile TEXT, image TEXT,
    image_hash TEXT, resources TEXT, devices TEXT, pid INTEGER, port INTEGER, exit_code INTEGER,
    outputs_path TEXT, logs_path TEXT, created_at REAL, updated_at REAL, started_at REAL, finished_at REAL);
CREATE TABLE IF NOT EXISTS job_statuses (id INTEGER PRIMARY KEY, job_id INTEGER, status TEXT, message TEXT,
    details TEXT, created_at REAL);
CREATE TABLE IF NOT EXISTS pipelines (id INTEGER PRIMARY KEY, uuid TEXT, project_id INTEGER, user TEXT, name TEXT,
    config TEXT, concurrency INTEGER, schedule TEXT, created_at REAL);
CREATE TABLE IF NOT EXISTS pipeline_runs (id INTEGER PRIMARY KEY, pipeline_id INTEGER, status TEXT,
    created_at REAL, started_at REAL, finished_at REAL);
CREATE TABLE IF NOT EXISTS operation_runs (id INTEGER PRIMARY KEY, pipeline_run_id INTEGER, name TEXT,
    config TEXT, status TEXT, retries INTEGER DEFAULT 0, entity_kind TEXT, entity_id INTEGER, message TEXT,
    created_at REAL, started_at REAL, finished_at REAL);
CREATE TABLE IF NOT EXISTS activity_logs (id INTEGER PRIMARY KEY, event_type TEXT, actor TEXT,
    object_kind TEXT, object_id INTEGER, context TEXT, created_at REAL);
CREATE TABLE IF NOT EXISTS notifications (id INTEGER PRIMARY KEY, event_type TEXT, object_kind TEXT,
    object_id INTEGER, context TEXT, user TEXT, is_read INTEGER DEFAULT 0, created_at REAL);
CREATE TABLE IF NOT EXISTS bookmarks (id INTEGER PRIMARY KEY, user TEXT, object_kind TEXT, object_id INTEGER,
    enabled INTEGER DEFAULT 1, created_at REAL, UNIQUE(user, object_kind, object_id));
CREATE TABLE IF NOT EXISTS searches (id INTEGER PRIMARY KEY, user TEXT, project_id INTEGER, content_kind TEXT,
    name TEXT, query TEXT, created_at REAL);
CREATE TABLE IF NOT EXISTS chart_views (id INTEGER PRIMARY KEY, object_kind TEXT, object_id INTEGER, name TEXT,
    charts TEXT, meta TEXT, created_at REAL);
CREATE TABLE IF NOT EXISTS cluster_nodes (id INTEGER PRIMARY KEY, uuid TEXT, name TEXT UNIQUE, hostname TEXT,
    role TEXT, cpu REAL, memory REAL, n_gpus INTEGER, schedulable INTEGER DEFAULT 1, status TEXT, created_at REAL,
    updated_at REAL);
CREATE TABLE IF NOT EXISTS node_gpus (id INTEGER PRIMARY KEY, node_id INTEGER, idx INTEGER, serial TEXT, name TEXT,
    memory REAL, arch TEXT, created_at REAL, UNIQUE(node_id, idx));
CREATE TABLE IF NOT EXISTS cluster_events (id INTEGER PRIMARY KEY, kind TEXT, level TEXT, message TEXT, data TEXT,
    created_at REAL);
CREATE TABLE IF NOT EXISTS kv (k TEXT PRIMARY KEY, v TEXT, expires_at REAL);
CREATE TABLE IF NOT EXISTS external_repos (id INTEGER PRIMARY KEY, project_id INTEGER, git_url TEXT, path TEXT,
    last_commit TEXT, created_at REAL, updated_at REAL, UNIQUE(project_id, git_url));
"""

JSON_COLS = {"config", "declarations", "tags", "last_metric", "resources", "run_env", "content", "hptuning", "data",
             "definition", "devices", "values", "context", "details", "charts", "meta", "schedule", "query"}


def _now() -> float:
    return time.time()


def _json_safe(v: Any) -> Any:
    """``v`` with every non-finite float replaced by the string "NaN" / "Infinity" / "-Infinity".  json.dumps writes
    bare NaN / Infinity tokens, which are not JSON: SQLite's JSON functions reject the whole document as malformed,
    so one diverged trial's loss made every ``metric.*`` query and sort over its group fail."""
    if isinstance(v, float):
        if math.isfinite(v):
            return v
        return "NaN" if v != v else ("Infinity" if v > 0 else "-Infinity")
    if isinstance(v, dict):
        return {k: _json_safe(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_json_safe(x) for x in v]
    return v


def _enc(v: Any) -> Any:
    return json.dumps(_json_safe(v)) if v is not None else None


class StoreError(RuntimeError):
    pass


class TransitionError(StoreError):
    pass


class Store:
    def __init__(self, path: str = ":memory:"):
        self.path = path
        self._local = threading.local()
        self._lock = threading.RLock()
        if path == ":memory:":
            # one shared connection (memory DBs are per-connection)
            self._shared = sqlite3.connect(":memory:", check_same_thread=False, isolation_level=None)
            self._shared.row_factory = sqlite3.Row
            self._shared.executescript(SCHEMA)
        else:
            self._shared = None
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.conn().executescript(SCHEMA)

    # ------------------------------------------------------------------ connections
    def conn(self) -> sqlite3.Connection:
        if self._shared is not None:
            return self._shared
        c = getattr(self._local, "conn", None)
        if c is None:
            c = sqlite3.connect(self.path, timeout=30.0, isolation_level=None, check_same_thread=False)
            c.row_factory = sqlite3.Row
            c.execute("PRAGMA journal_mode=WAL")
            c.execute("PRAGMA synchronous=NORMAL")
            c.execute("PRAGMA busy_timeout=30000")
            self._local.conn = c
        return c

    def execute(self, sql: str, params: Sequence[Any] = ()) -> sqlite3.Cursor:
        with self._lock:
            return self.conn().execute(sql, params)

    def executemany(self, sql: str, rows: Iterable[Sequence[Any]]) -> None:
        with self._lock:
            c = self.conn()
            c.execute("BEGIN IMMEDIATE")
            try:
                c.executemany(sql, rows)
                c.execute("COMMIT")
            except Exception:
                c.execute("ROLLBACK")
                raise

    def _row(self, r: Optional[sqlite3.Row]) -> Optional[Dict[str, Any]]:
        if r is None:
            return None
        d = dict(r)
        for k, v in d.items():
            if k in JSON_COLS and isinstance(v, str):
                try:
                    d[k] = json.loads(v)
                except ValueError:
                    pass
        return d

    def _rows(self, rs) -> List[Dict[str, Any]]:
        return [self._row(r) for r in rs]

    def _insert(self, table: str, values: Dict[str, Any]) -> int:
        cols = list(values)
        vals = [_enc(v) if k in JSON_COLS else v for k, v in values.items()]
        sql = f"INSERT INTO {table} ({', '.join(_q(c) for c in cols)}) VALUES ({', '.join('?' * len(cols))})"
        return int(self.execute(sql, vals).lastrowid)

    def _update(self, table: str, id_: int, values: Dict[str, Any]) -> None:
        if not values:
            return
        sets = ", ".join(f"{_q(k)} = ?" for k in values)
        vals = [_enc(v) if k in JSON_COLS else v for k, v in values.items()]
        self.execute(f"UPDATE {table} SET {sets} WHERE id = ?", vals + [id_])

    def get(self, table: str, id_: int) -> Optional[Dict[str, Any]]:
        return self._row(self.execute(f"SELECT * FROM {table} WHERE id = ?", (id_,)).fetchone())

    # ------------------------------------------------------------------ users / projects
    def create_user(self, username: str, email: str = "", is_superuser: bool = False,
                    token: Optional[str] = None) -> Dict[str, Any]:
        token = token or uuidlib.uuid4().hex
        uid = self._insert("users", dict(username=username, email=email, is_superuser=int(is_superuser), token=token,
                                         created_at=_now()))
        return self.get("users", uid)

    def user_for_token(self, token: str) -> Optional[Dict[str, Any]]:
        return self._row(self.execute("SELECT * FROM users WHERE token = ?", (token,)).fetchone())

    def get_user(self, username: str):
        return self._row(self.execute("SELECT * FROM users WHERE username = ?", (username,)).fetchone())

    def create_project(self, name: str, user: str = "root", description: str = "", is_public: bool = True,
                       tags=None) -> Dict[str, Any]:
        existing = self.get_project(name, user)
        if existing:
            raise StoreError(f"project {user}/{name} already exists")
        pid = self._insert("projects", dict(uuid=uuidlib.uuid4().hex, user=user, name=name, description=description,
                                            is_public=int(is_public), tags=list(tags or []), created_at=_now(),
                                            updated_at=_now()))
        return self.get("projects", pid)

    def get_project(self, name: str, user: str = "root") -> Optional[Dict[str, Any]]:
        return self._row(self.execute("SELECT * FROM projects WHERE name = ? AND user = ?", (name, user)).fetchone())

    def get_or_create_project(self, name: str, user: str = "root") -> Dict[str, Any]:
        return self.get_project(name, user) or self.create_project(name, user)

    def list_projects(self, user: Optional[str] = None) -> List[Dict[str, Any]]:
        if user:
            return self._rows(self.execute("SELECT * FROM projects WHERE user = ? ORDER BY id", (user,)))
        return self._rows(self.execute("SELECT * FROM projects ORDER BY id"))

    def update_project(self, pid: int, **values) -> None:
        values["updated_at"] = _now()
        self._update("projects", pid, values)

    def delete_project(self, pid: int) -> None:
        for t, col in (("experiments", "project_id"), ("experiment_groups", "project_id"), ("jobs", "project_id")):
            self.execute(f"DELETE FROM {t} WHERE {col} = ?", (pid,))
        self.execute("DELETE FROM projects WHERE id = ?", (pid,))

    # ------------------------------------------------------------------ code references
    def create_code_reference(self, commit: Optional[str], branch: Optional[str] = None, git_url: Optional[str] = None,
                              is_dirty: bool = False, diff: Optional[str] = None) -> int:
        return self._insert("code_references", dict(commit_sha=commit, branch=branch, git_url=git_url,
                                                    is_dirty=int(is_dirty), diff=diff, created_at=_now()))

    # ------------------------------------------------------------------ experiments
    def create_experiment(self, project_id: int, config: Optional[Dict[str, Any]] = None, group_id: Optional[int] = None,
                          user: str = "root", name: Optional[str] = None, description: Optional[str] = None,
                          declarations: Optional[Dict[str, Any]] = None, tags=None,
                          original_experiment_id: Optional[int] = None, cloning_strategy: Optional[str] = None,
                          code_reference_id: Optional[int] = None, framework: Optional[str] = None,
                          resources: Optional[Dict[str, Any]] = None, is_managed: bool = True,
                          status: Optional[str] = "created") -> int:
        now = _now()
        xid = self._insert("experiments", dict(
            uuid=uuidlib.uuid4().hex, project_id=project_id, group_id=group_id, user=user, name=name,
            description=description, config=config, declarations=declarations or {}, tags=list(tags or []),
            status=None, last_metric={}, original_experiment_id=original_experiment_id,
            cloning_strategy=cloning_strategy, code_reference_id=code_reference_id, framework=framework,
            resources=resources, is_managed=int(is_managed), created_at=now, updated_at=now))
        if status:
            self.set_experiment_status(xid, status)
        return xid

    def get_experiment(self, xid: int) -> Optional[Dict[str, Any]]:
        return self.get("experiments", xid)

    def update_experiment(self, xid: int, **values) -> None:
        values["updated_at"] = _now()
        self._update("experiments", xid, values)

    def delete_experiment(self, xid: int) -> None:
        for t, c in (("experiment_metrics", "experiment_id"), ("experiment_statuses", "experiment_id"),
                     ("experiment_jobs", "experiment_id")):
            self.execute(f"DELETE FROM {t} WHERE {c} = ?", (xid,))
        self.execute("DELETE FROM experiments WHERE id = ?", (xid,))

    def set_experiment_status(self, xid: int, status: str, message: Optional[str] = None,
                              traceback: Optional[str] = None, force: bool = False) -> bool:
        """FSM-checked status change; returns False (and records nothing) for an illegal transition."""
        with self._lock:
            cur = self.execute("SELECT status, started_at FROM experiments WHERE id = ?", (xid,)).fetchone()
            if cur is None:
                raise StoreError(f"experiment {xid} does not exist")
            if not force and not ExperimentLifeCycle.can_transition(cur["status"], status):
                return False
            now = _now()
            self._insert("experiment_statuses", dict(experiment_id=xid, status=status, message=message,
                                                     traceback=traceback, created_at=now))
            vals: Dict[str, Any] = {"status": status, "updated_at": now}
            if status in ("starting", "running") and cur["started_at"] is None:
                vals["started_at"] = now
            if ExperimentLifeCycle.is_done(status):
                vals["finished_at"] = now
                if cur["started_at"] is None:
                    vals["started_at"] = now
            if status in ("resuming", "created"):
                vals["finished_at"] = None
            self._update("experiments", xid, vals)
            return True

    def experiment_statuses(self, xid: int) -> List[Dict[str, Any]]:
        return self._rows(self.execute("SELECT * FROM experiment_statuses WHERE experiment_id = ? ORDER BY id", (xid,)))

    def add_metrics(self, xid: int, values: Dict[str, float], step: Optional[int] = None,
                    created_at: Optional[float] = None) -> None:
        self.add_metrics_batch([(xid, values, step, created_at)])

    def add_metrics_batch(self, rows: Sequence[Tuple[int, Dict[str, float], Optional[int], Optional[float]]]) -> None:
        """Insert metric rows and merge each experiment's ``last_metric`` (one write transaction)."""
        if not rows:
            return
        now = _now()
        merged: Dict[int, Dict[str, float]] = {}
        for xid, vals, _, _ in rows:
            merged.setdefault(xid, {}).update({k: float(v) for k, v in vals.items()})
        with self._lock:
            c = self.conn()
            c.execute("BEGIN IMMEDIATE")
            try:
                c.executemany('INSERT INTO experiment_metrics (experiment_id, step, "values", created_at) '
                              "VALUES (?, ?, ?, ?)",
                              [(x, s, json.dumps(_json_safe({k: float(v) for k, v in vals.items()})), ts or now)
                               for x, vals, s, ts in rows])
                for xid, vals in merged.items():
                    r = c.execute("SELECT last_metric FROM experiments WHERE id = ?", (xid,)).fetchone()
                    if r is None:
                        raise StoreError(f"experiment {xid} does not exist")
                    last = json.loads(r["last_metric"] or "{}")
                    last.update(vals)
                    c.execute("UPDATE experiments SET last_metric = ?, updated_at = ? WHERE id = ?",
                              (json.dumps(_json_safe(last)), now, xid))
                c.execute("COMMIT")
            except Exception:
                c.execute("ROLLBACK")
                raise

    def get_metrics(self, xid: int) -> List[Dict[str, Any]]:
        return self._rows(self.execute('SELECT * FROM experiment_metrics WHERE experiment_id = ? ORDER BY id', (xid,)))

    def list_experiments(self, project_id: Optional[int] = None, group_id: Optional[int] = None,
                         independent: Optional[bool] = None, ids: Optional[Sequence[int]] = None,
                         query: Optional[str] = None, sort: Optional[str] = None, limit: Optional[int] = None,
                         offset: int = 0) -> List[Dict[str, Any]]:
        from polyaxon_amd.store.query import ExperimentQuery

        where, params = [], []
        if project_id is not None:
            where.append("e.project_id = ?")
            params.append(project_id)
        if group_id is not None:
            where.append("e.group_id = ?")
            params.append(group_id)
        if independent:
            where.append("e.group_id IS NULL")
        if ids is not None:
            ids = list(ids)
            if not ids:
                return []
            where.append(f"e.id IN ({', '.join('?' * len(ids))})")
            params.extend(ids)
        q = ExperimentQuery()
        if query:
            w, p = q.where(query)
            where.extend(w)
            params.extend(p)
        order = q.order_by(sort) if sort else "e.id ASC"
        sql = "SELECT e.* FROM experiments e"
        if where:
            sql += " WHERE " + " AND ".join(where)
        sql += f" ORDER BY {order}"
        if limit is not None:
            sql += f" LIMIT {int(limit)} OFFSET {int(offset)}"
        return self._rows(self.execute(sql, params))

    def experiments_metrics(self, ids: Sequence[int], metric: str) -> List[Tuple[int, Optional[float]]]:
        """(id, last_metric[metric]) pairs — reference ExperimentGroup.get_experiments_metrics."""
        ids = list(ids)
        if not ids:
            return []
        rows = self.execute(f"SELECT id, json_extract(last_metric, ?) AS m FROM experiments WHERE id IN "
                            f"({', '.join('?' * len(ids))}) ORDER BY id", [f'$."{metric}"'] + ids).fetchall()
        # a non-finite value (stored as a string, _json_safe) ranks nothing: reported as missing
        return [(r["id"], r["m"] if isinstance(r["m"], (int, float)) else None) for r in rows]

    # ------------------------------------------------------------------ experiment jobs (replicas)
    def create_experiment_job(self, xid: int, role: str, index: int, definition: Optional[Dict[str, Any]] = None,
                              resources: Optional[Dict[str, Any]] = None, devices: Optional[List[int]] = None) -> int:
        now = _now()
        jid = self._insert("experiment_jobs", dict(uuid=uuidlib.uuid4().hex, experiment_id=xid, role=role, idx=index,
                                                   status=None, definition=definition or {}, resources=resources,
                                                   devices=devices, created_at=now, updated_at=now))
        self.set_experiment_job_status(jid, "created")
        return jid

    def experiment_jobs(self, xid: int) -> List[Dict[str, Any]]:
        return self._rows(self.execute("SELECT * FROM experiment_jobs WHERE experiment_id = ? ORDER BY id", (xid,)))

    def update_experiment_job(self, jid: int, **values) -> None:
        values["updated_at"] = _now()
        self._update("experiment_jobs", jid, values)

    def set_experiment_job_status(self, jid: int, status: str, message: Optional[str] = None,
                                  details: Optional[Dict[str, Any]] = None) -> bool:
        with self._lock:
            cur = self.execute("SELECT status, started_at FROM experiment_jobs WHERE id = ?", (jid,)).fetchone()
            if cur is None:
                raise StoreError(f"experiment job {jid} does not exist")
            if not JobLifeCycle.can_transition(cur["status"], status):
                return False
            now = _now()
            self._insert("experiment_job_statuses", dict(job_id=jid, status=status, message=message, details=details,
                                                         created_at=now))
            vals: Dict[str, Any] = {"status": status, "updated_at": now}
            if status == "running" and cur["started_at"] is None:
                vals["started_at"] = now
            if JobLifeCycle.is_done(status):
                vals["finished_at"] = now
            self._update("experiment_jobs", jid, vals)
            return True

    def experiment_job_statuses(self, jid: int) -> List[Dict[str, Any]]:
        return self._rows(self.execute("SELECT * FROM experiment_job_statuses WHERE job_id = ? ORDER BY id", (jid,)))

    # ------------------------------------------------------------------ groups
    def create_group(self, project_id: int, content: Dict[str, Any], hptuning: Dict[str, Any], user: str = "root",
                     name: Optional[str] = None, description: Optional[str] = None, tags=None,
                     search_algorithm: Optional[str] = None, concurrency: int = 1,
                     code_reference_id: Optional[int] = None) -> int:
        now = _now()
        gid = self._insert("experiment_groups", dict(
            uuid=uuidlib.uuid4().hex, project_id=project_id, user=user, name=name, description=description,
            content=content, hptuning=hptuning, tags=list(tags or []), status=None, search_algorithm=search_algorithm,
            concurrency=concurrency, code_reference_id=code_reference_id, created_at=now, updated_at=now))
        self.set_group_status(gid, "created")
        return gid

    def get_group(self, gid: int) -> Optional[Dict[str, Any]]:
        return self.get("experiment_groups", gid)

    def list_groups(self, project_id: Optional[int] = None) -> List[Dict[str, Any]]:
        if project_id is None:
            return self._rows(self.execute("SELECT * FROM experiment_groups ORDER BY id"))
        return self._rows(self.execute("SELECT * FROM experiment_groups WHERE project_id = ? ORDER BY id",
                                       (project_id,)))

    def set_group_status(self, gid: int, status: str, message: Optional[str] = None) -> bool:
        with self._lock:
            cur = self.execute("SELECT status, started_at FROM experiment_groups WHERE id = ?", (gid,)).fetchone()
            if cur is None:
                raise StoreError(f"group {gid} does not exist")
            if not ExperimentGroupLifeCycle.can_transition(cur["status"], status):
                return False
            now = _now()
            self._insert("experiment_group_statuses", dict(group_id=gid, status=status, message=message,
                                                           created_at=now))
            vals: Dict[str, Any] = {"status": status, "updated_at": now}
            if status == "running" and cur["started_at"] is None:
                vals["started_at"] = now
            if ExperimentGroupLifeCycle.is_done(status):
                vals["finished_at"] = now
            self._update("experiment_groups", gid, vals)
            return True

    def group_statuses(self, gid: int) -> List[Dict[str, Any]]:
        return self._rows(self.execute("SELECT * FROM experiment_group_statuses WHERE group_id = ? ORDER BY id",
                                       (gid,)))

    def group_status_counts(self, gid: int) -> Dict[str, int]:
        rows = self.execute("SELECT status, COUNT(*) AS n FROM experiments WHERE group_id = ? GROUP BY status", (gid,))
        return {r["status"]: r["n"] for r in rows}

    def create_iteration(self, gid: int, data: Dict[str, Any]) -> int:
        return self._insert("experiment_group_iterations", dict(group_id=gid, data=data, created_at=_now(),
                                                                updated_at=_now()))

    def update_iteration(self, iid: int, data: Dict[str, Any]) -> None:
        self._update("experiment_group_iterations", iid, dict(data=data, updated_at=_now()))

    def last_iteration(self, gid: int) -> Optional[Dict[str, Any]]:
        return self._row(self.execute("SELECT * FROM experiment_group_iterations WHERE group_id = ? ORDER BY id DESC "
                                      "LIMIT 1", (gid,)).fetchone())

    def iterations(self, gid: int) -> List[Dict[str, Any]]:
        return self._rows(self.execute("SELECT * FROM experiment_group_iterations WHERE group_id = ? ORDER BY id",
                                       (gid,)))

    # ------------------------------------------------------------------ generic jobs (job/build/notebook/tensorboard)
    def create_job(self, kind: str, project_id: int, config: Optional[Dict[str, Any]] = None, user: str = "root",
                   name: Optional[str] = None, description: Optional[str] = None, tags=None, **extra) -> int:
        now = _now()
        jid = self._insert("jobs", dict(uuid=uuidlib.uuid4().hex, kind=kind, project_id=project_id, user=user,
                                        name=name, description=description, config=config, tags=list(tags or []),
                                        status=None, created_at=now, updated_at=now, **extra))
        self.set_job_status(jid, "created")
        return jid

    def get_job(self, jid: int) -> Optional[Dict[str, Any]]:
        return self.get("jobs", jid)

    def update_job(self, jid: int, **values) -> None:
        values["updated_at"] = _now()
        self._update("jobs", jid, values)

    def list_jobs(self, kind: Optional[str] = None, project_id: Optional[int] = None,
                  status: Optional[str] = None) -> List[Dict[str, Any]]:
        where, params = [], []
        for col, v in (("kind", kind), ("project_id", project_id), ("status", status)):
            if v is not None:
                where.append(f"{col} = ?")
                params.append(v)
        sql = "SELECT * FROM jobs" + (" WHERE " + " AND ".join(where) if where else "") + " ORDER BY id"
        return self._rows(self.execute(sql, params))

    def set_job_status(self, jid: int, status: str, message: Optional[str] = None,
                       details: Optional[Dict[str, Any]] = None) -> bool:
        with self._lock:
            cur = self.execute("SELECT status, started_at FROM jobs WHERE id = ?", (jid,)).fetchone()
            if cur is None:
                raise StoreError(f"job {jid} does not exist")
            if not JobLifeCycle.can_transition(cur["status"], status):
                return False
            now = _now()
            self._insert("job_statuses", dict(job_id=jid, status=status, message=message, details=details,
                                              created_at=now))
            vals: Dict[str, Any] = {"status": status, "updated_at": now}
            if status == "running" and cur["started_at"] is None:
                vals["started_at"] = now
            if JobLifeCycle.is_done(status):
                vals["finished_at"] = now
            self._update("jobs", jid, vals)
            return True

    def job_statuses(self, jid: int) -> List[Dict[str, Any]]:
        return self._rows(self.execute("SELECT * FROM job_statuses WHERE job_id = ? ORDER BY id", (jid,)))

    def last_build_for_hash(self, image_hash: str, max_age_s: float) -> Optional[Dict[str, Any]]:
        """Reuse window for built environments (reference dockerizer_scheduler.py:48-50, 6 h)."""
        r = self.execute("SELECT * FROM jobs WHERE kind = 'build' AND image_hash = ? AND status = 'succeeded' "
                         "AND finished_at >= ? ORDER BY id DESC LIMIT 1", (image_hash, _now() - max_age_s)).fetchone()
        return self._row(r)

    # ------------------------------------------------------------------ pipelines
    def create_pipeline(self, project_id: int, name: str, config: Dict[str, Any], user: str = "root",
                        concurrency: Optional[int] = None, schedule=None) -> int:
        return self._insert("pipelines", dict(uuid=uuidlib.uuid4().hex, project_id=project_id, user=user, name=name,
                                              config=config, concurrency=concurrency, schedule=schedule,
                                              created_at=_now()))

    def create_pipeline_run(self, pipeline_id: int) -> int:
        rid = self._insert("pipeline_runs", dict(pipeline_id=pipeline_id, status="created", created_at=_now()))
        return rid

    def set_pipeline_run_status(self, rid: int, status: str) -> bool:
        cur = self.get("pipeline_runs", rid)
        if not PipelineLifeCycle.can_transition(cur["status"], status) and cur["status"] != status:
            return False
        vals: Dict[str, Any] = {"status": status}
        if status == "running":
            vals["started_at"] = _now()
        if PipelineLifeCycle.is_done(status):
            vals["finished_at"] = _now()
        self._update("pipeline_runs", rid, vals)
        return True

    def create_operation_run(self, pipeline_run_id: int, name: str, config: Dict[str, Any]) -> int:
        return self._insert("operation_runs", dict(pipeline_run_id=pipeline_run_id, name=name, config=config,
                                                   status="created", created_at=_now()))

    def set_operation_run_status(self, oid: int, status: str, message: Optional[str] = None) -> bool:
        cur = self.get("operation_runs", oid)
        if not OperationLifeCycle.can_transition(cur["status"], status):
            return False
        vals: Dict[str, Any] = {"status": status, "message": message}
        if status == "running":
            vals["started_at"] = _now()
        if OperationLifeCycle.is_done(status):
            vals["finished_at"] = _now()
        self._update("operation_runs", oid, vals)
        return True

    def operation_runs(self, pipeline_run_id: int) -> List[Dict[str, Any]]:
        return self._rows(self.execute("SELECT * FROM operation_runs WHERE pipeline_run_id = ? ORDER BY id",
                                       (pipeline_run_id,)))

    def update_operation_run(self, oid: int, **values) -> None:
        self._update("operation_runs", oid, values)

    # ------------------------------------------------------------------ activity / notifications / bookmarks / searches
    def add_activity(self, event_type: str, actor: Optional[str], object_kind: Optional[str],
                     object_id: Optional[int], context: Optional[Dict[str, Any]] = None) -> int:
        return self._insert("activity_logs", dict(event_type=event_type, actor=actor, object_kind=object_kind,
                                                  object_id=object_id, context=context or {}, created_at=_now()))

    def activities(self, object_kind: Optional[str] = None, object_id: Optional[int] = None, limit: int = 100):
        if object_kind is None:
            return self._rows(self.execute("SELECT * FROM activity_logs ORDER BY id DESC LIMIT ?", (limit,)))
        return self._rows(self.execute("SELECT * FROM activity_logs WHERE object_kind = ? AND object_id = ? "
                                       "ORDER BY id DESC LIMIT ?", (object_kind, object_id, limit)))

    def add_notification(self, event_type: str, object_kind: Optional[str], object_id: Optional[int],
                         context: Optional[Dict[str, Any]] = None, user: Optional[str] = None) -> int:
        return self._insert("notifications", dict(event_type=event_type, object_kind=object_kind, object_id=object_id,
                                                  context=context or {}, user=user, created_at=_now()))

    def notifications(self, user: Optional[str] = None, unread_only: bool = False):
        sql, params = "SELECT * FROM notifications", []
        cond = []
        if user is not None:
            cond.append("user = ?")
            params.append(user)
        if unread_only:
            cond.append("is_read = 0")
        if cond:
            sql += " WHERE " + " AND ".join(cond)
        return self._rows(self.execute(sql + " ORDER BY id DESC", params))

    def set_bookmark(self, user: str, object_kind: str, object_id: int, enabled: bool = True) -> None:
        self.execute("INSERT INTO bookmarks (user, object_kind, object_id, enabled, created_at) VALUES (?, ?, ?, ?, ?) "
                     "ON CONFLICT(user, object_kind, object_id) DO UPDATE SET enabled = excluded.enabled",
                     (user, object_kind, object_id, int(enabled), _now()))

    def bookmarks(self, user: str, object_kind: Optional[str] = None):
        if object_kind:
            return self._rows(self.execute("SELECT * FROM bookmarks WHERE user = ? AND object_kind = ? AND enabled = 1",
                                           (user, object_kind)))
        return self._rows(self.execute("SELECT * FROM bookmarks WHERE user = ? AND enabled = 1", (user,)))

    def create_search(self, user: str, project_id: int, content_kind: str, name: str, query: Dict[str, Any]) -> int:
        return self._insert("searches", dict(user=user, project_id=project_id, content_kind=content_kind, name=name,
                                             query=query, created_at=_now()))

    def searches(self, project_id: int, content_kind: Optional[str] = None):
        if content_kind:
            return self._rows(self.execute("SELECT * FROM searches WHERE project_id = ? AND content_kind = ?",
                                           (project_id, content_kind)))
        return self._rows(self.execute("SELECT * FROM searches WHERE project_id = ?", (project_id,)))

    def create_chart_view(self, object_kind: str, object_id: int, name: str, charts, meta=None) -> int:
        return self._insert("chart_views", dict(object_kind=object_kind, object_id=object_id, name=name,
                                                charts=charts, meta=meta or {}, created_at=_now()))

    def chart_views(self, object_kind: str, object_id: int):
        return self._rows(self.execute("SELECT * FROM chart_views WHERE object_kind = ? AND object_id = ?",
                                       (object_kind, object_id)))

    # ------------------------------------------------------------------ cluster inventory / events
    def upsert_node(self, name: str, hostname: str, cpu: float, memory: float, n_gpus: int, role: str = "master",
                    status: str = "ready") -> int:
        r = self.execute("SELECT id FROM cluster_nodes WHERE name = ?", (name,)).fetchone()
        now = _now()
        if r:
            self._update("cluster_nodes", r["id"], dict(hostname=hostname, cpu=cpu, memory=memory, n_gpus=n_gpus,
                                                        role=role, status=status, updated_at=now))
            return int(r["id"])
        return self._insert("cluster_nodes", dict(uuid=uuidlib.uuid4().hex, name=name, hostname=hostname, role=role,
                                                  cpu=cpu, memory=memory, n_gpus=n_gpus, status=status,
                                                  created_at=now, updated_at=now))

    def upsert_node_gpu(self, node_id: int, index: int, name: str, memory: float, serial: str = "",
                        arch: str = "gfx950") -> None:
        self.execute("INSERT INTO node_gpus (node_id, idx, serial, name, memory, arch, created_at) VALUES "
                     "(?, ?, ?, ?, ?, ?, ?) ON CONFLICT(node_id, idx) DO UPDATE SET name = excluded.name, "
                     "memory = excluded.memory, serial = excluded.serial, arch = excluded.arch",
                     (node_id, index, serial, name, memory, arch, _now()))

    def nodes(self):
        return self._rows(self.execute("SELECT * FROM cluster_nodes ORDER BY id"))

    def node_gpus(self, node_id: int):
        return self._rows(self.execute("SELECT * FROM node_gpus WHERE node_id = ? ORDER BY idx", (node_id,)))

    def add_cluster_event(self, kind: str, level: str, message: str, data=None) -> int:
        return self._insert("cluster_events", dict(kind=kind, level=level, message=message, data=data or {},
                                                   created_at=_now()))

    def cluster_events(self, limit: int = 100):
        return self._rows(self.execute("SELECT * FROM cluster_events ORDER BY id DESC LIMIT ?", (limit,)))

    # ------------------------------------------------------------------ ephemeral key/value (Redis replacement)
    def upsert_external_repo(self, project_id: int, git_url: str, path: str, last_commit: Optional[str]) -> int:
        """Reference ExternalRepo (db/models/repos.py): one row per (project, git url)."""
        row = self.execute("SELECT id FROM external_repos WHERE project_id = ? AND git_url = ?",
                           (project_id, git_url)).fetchone()
        if row:
            self._update("external_repos", row["id"], {"path": path, "last_commit": last_commit,
                                                        "updated_at": _now()})
            return int(row["id"])
        return self._insert("external_repos", dict(project_id=project_id, git_url=git_url, path=path,
                                                   last_commit=last_commit, created_at=_now(), updated_at=_now()))

    def external_repos(self, project_id: Optional[int] = None) -> List[Dict[str, Any]]:
        if project_id is None:
            return self._rows(self.execute("SELECT * FROM external_repos ORDER BY id"))
        return self._rows(self.execute("SELECT * FROM external_repos WHERE project_id = ? ORDER BY id", (project_id,)))

    def kv_set(self, key: str, value: Any, ttl: Optional[float] = None) -> None:
        exp = _now() + ttl if ttl else None
        self.execute("INSERT INTO kv (k, v, expires_at) VALUES (?, ?, ?) ON CONFLICT(k) DO UPDATE SET "
                     "v = excluded.v, expires_at = excluded.expires_at", (key, json.dumps(value), exp))

    def kv_get(self, key: str, default: Any = None) -> Any:
        r = self.execute("SELECT v, expires_at FROM kv WHERE k = ?", (key,)).fetchone()
        if r is None:
            return default
        if r["expires_at"] is not None and r["expires_at"] < _now():
            self.execute("DELETE FROM kv WHERE k = ?", (key,))
            return default
        return json.loads(r["v"])

    def kv_delete(self, key: str) -> None:
        self.execute("DELETE FROM kv WHERE k = ?", (key,))


def _q(col: str) -> str:
    return f'"{col}"'
