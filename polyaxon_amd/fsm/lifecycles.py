"""Lifecycle state machines for experiments, jobs, groups, pipelines and operations.

Semantics are the reference's (polyaxon/constants/{statuses,experiments,jobs,experiment_groups,
pipelines}.py): a transition ``from → to`` is legal iff ``from`` is in ``allowed[to]``; ``None`` is the
"no status yet" state; ``jobs_status`` aggregates replica statuses with the reference precedence
(unknown > stopped > all-succeeded > failed > starting > running, constants/experiments.py:97-120).

Here each lifecycle is one immutable :class:`Lifecycle` object built from a compact table instead of a
class hierarchy, and the status groups (pending / running / done / failed) are plain frozensets.
"""
from __future__ import annotations

from typing import Dict, FrozenSet, Iterable, Optional


class S:
    CREATED = "created"
    SCHEDULED = "scheduled"
    BUILDING = "building"
    RESUMING = "resuming"
    STARTING = "starting"
    RUNNING = "running"
    SUCCEEDED = "succeeded"
    FAILED = "failed"
    UPSTREAM_FAILED = "upstream_failed"
    STOPPED = "stopped"
    FINISHED = "finished"
    SKIPPED = "skipped"
    RETRYING = "retrying"
    UNKNOWN = "unknown"


class Lifecycle:
    def __init__(self, name: str, values: Iterable[str], allowed: Dict[str, Iterable[Optional[str]]],
                 pending=(), starting=(), running=(), done=(), failed=()):
        self.name = name
        self.VALUES: FrozenSet[str] = frozenset(values)
        self.TRANSITION_MATRIX: Dict[str, FrozenSet[Optional[str]]] = {k: frozenset(v) for k, v in allowed.items()}
        self.PENDING_STATUS = frozenset(pending)
        self.STARTING_STATUS = frozenset(starting)
        self.RUNNING_STATUS = frozenset(running)
        self.DONE_STATUS = frozenset(done)
        self.FAILED_STATUS = frozenset(failed)
        for v in self.VALUES:
            setattr(self, v.upper(), v)

    def can_transition(self, status_from: Optional[str], status_to: str) -> bool:
        allowed = self.TRANSITION_MATRIX.get(status_to)
        return allowed is not None and status_from in allowed

    def is_pending(self, s) -> bool:
        return s in self.PENDING_STATUS

    def is_starting(self, s) -> bool:
        return s in self.STARTING_STATUS

    def is_running(self, s) -> bool:
        return s in self.RUNNING_STATUS

    def is_done(self, s) -> bool:
        return s in self.DONE_STATUS

    def failed(self, s) -> bool:
        return s in self.FAILED_STATUS

    def succeeded(self, s) -> bool:
        return s == S.SUCCEEDED

    def stopped(self, s) -> bool:
        return s == S.STOPPED

    def skipped(self, s) -> bool:
        return s == S.SKIPPED

    def __repr__(self) -> str:
        return f"Lifecycle({self.name})"


def _all_but(values, *excluded):
    return set(values) - set(excluded)


_JOB_VALUES = (S.CREATED, S.BUILDING, S.SCHEDULED, S.RUNNING, S.SUCCEEDED, S.FAILED, S.STOPPED, S.UNKNOWN)
JobLifeCycle = Lifecycle(
    "job", _JOB_VALUES,
    {
        S.CREATED: [None],
        S.BUILDING: [None, S.CREATED, S.SCHEDULED],  # image build, then placement "build" phase
        S.SCHEDULED: [S.CREATED, S.BUILDING],
        S.RUNNING: [S.CREATED, S.SCHEDULED, S.BUILDING, S.UNKNOWN],
        S.SUCCEEDED: [S.CREATED, S.BUILDING, S.SCHEDULED, S.RUNNING, S.UNKNOWN],
        S.FAILED: [S.CREATED, S.BUILDING, S.SCHEDULED, S.RUNNING, S.UNKNOWN],
        S.STOPPED: _all_but(_JOB_VALUES, S.STOPPED),
        S.UNKNOWN: set(_JOB_VALUES),
    },
    starting=(S.CREATED, S.BUILDING), running=(S.BUILDING, S.SCHEDULED, S.RUNNING),
    done=(S.FAILED, S.STOPPED, S.SUCCEEDED), failed=(S.FAILED,))

_XP_VALUES = (S.CREATED, S.RESUMING, S.BUILDING, S.SCHEDULED, S.STARTING, S.RUNNING, S.SUCCEEDED, S.FAILED,
              S.STOPPED, S.UNKNOWN, S.RETRYING)


class _ExperimentLifecycle(Lifecycle):
    def jobs_status(self, job_statuses) -> Optional[str]:
        """Aggregate replica (job) statuses into the experiment status."""
        js = list(job_statuses)
        if not js:
            return None
        if any(s == S.UNKNOWN for s in js):
            return S.UNKNOWN
        if any(s == S.STOPPED for s in js):
            return S.STOPPED
        if all(s == S.SUCCEEDED for s in js):
            return S.SUCCEEDED
        if any(s == S.FAILED for s in js):
            return S.FAILED
        if any(JobLifeCycle.is_starting(s) for s in js):
            return S.STARTING
        if any(JobLifeCycle.is_running(s) for s in js):
            return S.RUNNING
        return S.UNKNOWN


ExperimentLifeCycle = _ExperimentLifecycle(
    "experiment", _XP_VALUES,
    {
        S.CREATED: [None],
        S.RESUMING: [S.SUCCEEDED, S.STOPPED],
        S.BUILDING: [S.CREATED, S.RESUMING],
        S.SCHEDULED: [S.CREATED, S.RESUMING, S.BUILDING, S.RETRYING],
        S.STARTING: [S.SCHEDULED],
        # opt-in retry (environment.max_restarts, an MI355X extension; the reference never retries)
        S.RETRYING: [S.SCHEDULED, S.STARTING, S.RUNNING],
        S.RUNNING: [S.SCHEDULED, S.STARTING, S.UNKNOWN],
        S.SUCCEEDED: [S.SCHEDULED, S.STARTING, S.RUNNING, S.UNKNOWN],
        S.FAILED: [S.CREATED, S.RESUMING, S.BUILDING, S.SCHEDULED, S.STARTING, S.RUNNING, S.UNKNOWN, S.RETRYING],
        S.STOPPED: _all_but(_XP_VALUES, S.STOPPED),
        S.UNKNOWN: set(_XP_VALUES),
    },
    pending=(S.CREATED, S.RESUMING), running=(S.SCHEDULED, S.BUILDING, S.STARTING, S.RUNNING, S.RETRYING),
    done=(S.FAILED, S.STOPPED, S.SUCCEEDED), failed=(S.FAILED,))

_GROUP_VALUES = (S.CREATED, S.RUNNING, S.SUCCEEDED, S.FAILED, S.STOPPED)
ExperimentGroupLifeCycle = Lifecycle(
    "experiment_group", _GROUP_VALUES,
    {
        S.CREATED: [None],
        S.RUNNING: [S.CREATED, S.STOPPED],
        S.SUCCEEDED: [S.RUNNING],
        S.FAILED: [S.CREATED, S.RUNNING],
        S.STOPPED: _all_but(_GROUP_VALUES, S.STOPPED),
    },
    pending=(S.CREATED,), running=(S.RUNNING,), done=(S.FAILED, S.STOPPED, S.SUCCEEDED), failed=(S.FAILED,))

_PIPE_VALUES = (S.CREATED, S.SCHEDULED, S.RUNNING, S.FINISHED, S.STOPPED, S.SKIPPED)
PipelineLifeCycle = Lifecycle(
    "pipeline", _PIPE_VALUES,
    {
        S.CREATED: [None],
        S.SCHEDULED: [S.CREATED],
        S.RUNNING: [S.SCHEDULED],
        S.FINISHED: [S.CREATED, S.SCHEDULED, S.RUNNING],
        S.STOPPED: [S.CREATED, S.SCHEDULED, S.RUNNING],
        S.SKIPPED: [S.CREATED, S.SCHEDULED, S.STOPPED],
    },
    running=(S.SCHEDULED, S.RUNNING), done=(S.FINISHED, S.STOPPED, S.SKIPPED))

_OP_VALUES = (S.CREATED, S.SCHEDULED, S.RUNNING, S.SUCCEEDED, S.FAILED, S.UPSTREAM_FAILED, S.STOPPED, S.SKIPPED,
              S.RETRYING)
OperationLifeCycle = Lifecycle(
    "operation", _OP_VALUES,
    {
        S.CREATED: [None],
        S.SCHEDULED: [S.CREATED, S.RETRYING],
        S.RUNNING: [S.SCHEDULED],
        S.SUCCEEDED: [S.RUNNING],
        S.FAILED: [S.SCHEDULED, S.RUNNING],
        S.UPSTREAM_FAILED: _all_but(_OP_VALUES, S.UPSTREAM_FAILED),
        S.STOPPED: [S.CREATED, S.SCHEDULED, S.RUNNING],
        S.SKIPPED: [S.CREATED, S.SCHEDULED, S.STOPPED],
        S.RETRYING: [S.SCHEDULED, S.RUNNING, S.FAILED, S.STOPPED, S.SKIPPED, S.RETRYING],
    },
    running=(S.SCHEDULED, S.RUNNING), done=(S.SUCCEEDED, S.FAILED, S.UPSTREAM_FAILED, S.STOPPED, S.SKIPPED),
    failed=(S.FAILED, S.UPSTREAM_FAILED))


class TriggerPolicy:
    ALL_SUCCEEDED = "all_succeeded"
    ALL_FAILED = "all_failed"
    ALL_DONE = "all_done"
    ONE_SUCCEEDED = "one_succeeded"
    ONE_FAILED = "one_failed"
    ONE_DONE = "one_done"
    VALUES = frozenset({ALL_SUCCEEDED, ALL_FAILED, ALL_DONE, ONE_SUCCEEDED, ONE_FAILED, ONE_DONE})


# jobs / builds / notebooks / tensorboards share the job lifecycle (reference constants/jobs.py)
BuildJobLifeCycle = JobLifeCycle
PluginLifeCycle = JobLifeCycle
