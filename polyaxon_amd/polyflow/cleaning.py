"""Cleaning hooks: reconcile runs orphaned by a previous scheduler process, and expire old outputs.

Reference: commands/management/commands/clean_{experiments,experiment_groups,jobs,project_jobs,notebooks,
tensorboards}.py (stop everything the DB still calls running, message "Stop triggered by the cleaning hook.")
and crons/tasks/cleaning.py (periodic outputs/logs cleanup).  The reference runs these from a management
command at platform (re)start; here :meth:`Polyflow.start` runs :func:`clean_stale` before it schedules
anything, and ``plx admin clean`` runs any of them by hand.

An orphan's processes are only signalled when ``/proc/<pid>/environ`` still carries that run's
``POLYAXON_RUN_OUTPUTS_PATH`` — a recycled PID that belongs to someone else is never touched.
"""
from __future__ import annotations

import os
import shutil
import signal
import time
from typing import Dict, Iterable, List, Optional, Set, Tuple

from polyaxon_amd.fsm import ExperimentGroupLifeCycle, ExperimentLifeCycle, JobLifeCycle

MESSAGE = "Stop triggered by the cleaning hook."

JOB_KINDS = ("job", "build", "notebook", "tensorboard")


def _owned_pid(pid: Optional[int], outputs_path: Optional[str]) -> bool:
    if not pid or not outputs_path:
        return False
    try:
        with open(f"/proc/{pid}/environ", "rb") as f:
            env = f.read().split(b"\0")
    except OSError:
        return False
    return f"POLYAXON_RUN_OUTPUTS_PATH={outputs_path}".encode() in env


def _kill(pid: int) -> bool:
    try:
        if os.getpgid(pid) == pid and pid != os.getpgid(0):  # trial spawned as its own group leader: take
            os.killpg(pid, signal.SIGKILL)                     # its whole process tree
        else:
            os.kill(pid, signal.SIGKILL)
        return True
    except (ProcessLookupError, PermissionError):
        return False


def scheduler_alive(root: str) -> bool:
    try:
        with open(os.path.join(root, "scheduler.pid")) as f:
            pid = int(f.read().strip())
        os.kill(pid, 0)
        return True
    except (OSError, ValueError):
        return False


def clean_stale(store, live: Iterable[Tuple[str, int]] = (), kinds: Iterable[str] = ("experiments", "groups",
                                                                                            "jobs"),
                kill: bool = True) -> Dict[str, List[int]]:
    """Mark every non-terminal run that this scheduler does not own as stopped (killing its leftover
    processes).  ``live`` = ``(kind, id)`` pairs of runs the running scheduler does own."""
    live_set: Set[Tuple[str, int]] = set(live)
    out: Dict[str, List[int]] = {"experiments": [], "groups": [], "jobs": [], "killed": []}
    kinds = set(kinds)
    if "experiments" in kinds:
        xdone = tuple(ExperimentLifeCycle.DONE_STATUS)
        # unmanaged experiments are tracked by an external process through the client: not ours to stop
        rows = store.execute(f"SELECT id, outputs_path FROM experiments WHERE status IS NOT NULL AND is_managed = 1 "
                             f"AND status NOT IN ({','.join('?' * len(xdone))})", xdone).fetchall()
        for xid, outputs in rows:
            if ("experiment", xid) in live_set:
                continue
            if kill:
                for (pid,) in store.execute("SELECT pid FROM experiment_jobs WHERE experiment_id = ?",
                                            (xid,)).fetchall():
                    if _owned_pid(pid, outputs) and _kill(pid):
                        out["killed"].append(pid)
            for j in store.experiment_jobs(xid):
                if j.get("status") not in JobLifeCycle.DONE_STATUS:
                    store.set_experiment_job_status(j["id"], "stopped", MESSAGE)
            store.set_experiment_status(xid, "stopped", MESSAGE)
            out["experiments"].append(xid)
    if "jobs" in kinds:
        jdone = tuple(JobLifeCycle.DONE_STATUS)
        rows = store.execute(f"SELECT id, kind, pid, outputs_path FROM jobs WHERE status IS NOT NULL AND status NOT IN "
                             f"({','.join('?' * len(jdone))})", jdone).fetchall()
        for jid, kind, pid, outputs in rows:
            if (kind, jid) in live_set or ("job", jid) in live_set:
                continue
            if kill and _owned_pid(pid, outputs) and _kill(pid):
                out["killed"].append(pid)
            store.set_job_status(jid, "stopped", MESSAGE)
            out["jobs"].append(jid)
    if "groups" in kinds:
        gdone = tuple(ExperimentGroupLifeCycle.DONE_STATUS)
        rows = store.execute(f"SELECT id FROM experiment_groups WHERE status IS NOT NULL AND status NOT IN "
                             f"({','.join('?' * len(gdone))})", gdone).fetchall()
        for (gid,) in rows:
            if ("group", gid) in live_set:
                continue
            store.set_group_status(gid, "stopped", MESSAGE)
            out["groups"].append(gid)
    return out


def clean_outputs(store, older_than_s: float, now: Optional[float] = None, dry_run: bool = False) -> List[str]:
    """Delete outputs and logs of finished experiments/jobs whose ``finished_at`` is older than the cutoff
    (reference crons/tasks/cleaning.py).  Returns the deleted paths.

    RESUME clones share their root's outputs directory (reference libs/paths/experiments.py:17-18), so an outputs
    path is only removed once EVERY row that points at it is finished and past the retention window: a Hyperband
    root that finished long ago keeps its checkpoints while a resumed promotion still uses (or just used) them."""
    cutoff = (now if now is not None else time.time()) - older_than_s
    deleted: List[str] = []
    for table in ("experiments", "jobs"):
        rows = store.execute(f"SELECT id, outputs_path, logs_path FROM {table} WHERE finished_at IS NOT NULL "
                             f"AND finished_at < ?", (cutoff,)).fetchall()
        for rid, outputs, logs in rows:
            if outputs and store.execute(
                    f"SELECT 1 FROM {table} WHERE outputs_path = ? AND id != ? AND "
                    f"(finished_at IS NULL OR finished_at >= ?) LIMIT 1", (outputs, rid, cutoff)).fetchone():
                outputs = None  # still shared with a live or recent run
            for p in (outputs, logs):
                if p and os.path.isdir(p):
                    if not dry_run:
                        shutil.rmtree(p, ignore_errors=True)
                    deleted.append(p)
            if not dry_run and outputs:
                store.execute(f"UPDATE {table} SET outputs_path = NULL WHERE outputs_path = ? AND finished_at IS NOT "
                              f"NULL AND finished_at < ?", (outputs, cutoff))
    return deleted
