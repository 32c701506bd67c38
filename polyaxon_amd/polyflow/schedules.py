"""Pipeline schedules: periodic pipeline runs (frequency or cron), bounded by start_at / end_at, optionally
depending on the previous run's success.

Reference: the ``Schedule`` model (polyaxon/db/models/pipelines.py:23-47: ``frequency`` "gets added to your latest
operation instance's execution_date to figure out the next schedule", ``start_at`` default now, ``end_at`` default
open-ended, ``depends_on_past`` "instances will run sequentially while relying on the previous instances' schedule
to succeed") and ``ExecutableModel.execute_at`` (:52-74).  The reference leaves firing to Celery beat; here a
``PipelineSchedule`` owns a polyflow timer: each firing creates a new pipeline run (a fresh ``PipelineRunner``),
and the next fire time is computed from the *scheduled* time (not the completion time), so runs do not drift.

Spec (Polyaxonfile ``kind: pipeline``)::

    schedule:
      frequency: 3600 | "1h30m" | "45s"      # or
      cron: "*/15 9-17 * * 1-5"               # minute hour day-of-month month day-of-week (0 = Sunday)
      start_at: 1790000000 | "2026-10-16T12:00:00"   # default: now
      end_at: ...                                     # default: open-ended
      depends_on_past: false
      max_runs: 10                                    # MI355X extension: stop after this many runs
"""
from __future__ import annotations

import calendar
import logging
import re
import time
from dataclasses import dataclass
from datetime import datetime, timezone
from typing import Any, Dict, List, Optional, Set

log = logging.getLogger("polyaxon_amd.polyflow.schedules")

_UNITS = {"w": 604800, "d": 86400, "h": 3600, "m": 60, "s": 1}


class ScheduleError(ValueError):
    pass


def parse_frequency(v) -> float:
    """Seconds from a number, a numeric string or a duration like ``1h30m`` / ``45s`` / ``2d``."""
    if isinstance(v, (int, float)):
        out = float(v)
    else:
        s = str(v).strip().lower()
        if re.fullmatch(r"\d+(\.\d+)?", s):
            out = float(s)
        else:
            parts = re.findall(r"(\d+(?:\.\d+)?)([wdhms])", s)
            if not parts or "".join(a + b for a, b in parts) != s.replace(" ", ""):
                raise ScheduleError(f"cannot parse frequency {v!r} (use seconds or e.g. 1h30m)")
            out = sum(float(a) * _UNITS[b] for a, b in parts)
    if out <= 0:
        raise ScheduleError("schedule frequency must be positive")
    return out


def parse_time(v) -> Optional[float]:
    if v is None:
        return None
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip()
    if re.fullmatch(r"\d+(\.\d+)?", s):
        return float(s)
    try:
        dt = datetime.fromisoformat(s.replace("Z", "+00:00"))
    except ValueError:
        raise ScheduleError(f"cannot parse time {v!r} (epoch seconds or ISO 8601)") from None
    if dt.tzinfo is None:
        dt = dt.replace(tzinfo=timezone.utc)
    return dt.timestamp()


class Cron:
    """5-field cron (minute hour day-of-month month day-of-week) with ``*``, ``*/n``, ``a-b``, ``a-b/n`` and lists;
    evaluated in UTC.  When both day fields are restricted, a day matches either (Vixie cron)."""

    RANGES = ((0, 59), (0, 23), (1, 31), (1, 12), (0, 6))

    def __init__(self, expr: str):
        fields = expr.split()
        if len(fields) != 5:
            raise ScheduleError(f"cron needs 5 fields, got {expr!r}")
        self.expr = expr
        self.sets: List[Set[int]] = []
        self.restricted = []
        for f, (lo, hi) in zip(fields, self.RANGES):
            self.sets.append(self._field(f, lo, hi))
            self.restricted.append(f != "*")
        self.sets[4] = {d % 7 for d in self.sets[4]}  # 7 = Sunday too

    @staticmethod
    def _field(f: str, lo: int, hi: int) -> Set[int]:
        out: Set[int] = set()
        for part in f.split(","):
            step = 1
            if "/" in part:
                part, st = part.split("/", 1)
                step = int(st)
                if step <= 0:
                    raise ScheduleError("cron step must be positive")
            if part in ("*", ""):
                a, b = lo, hi
            elif "-" in part:
                a, b = (int(x) for x in part.split("-", 1))
            else:
                a = b = int(part)
                if step > 1:
                    b = hi
            if a < lo or b > (7 if hi == 6 else hi) or a > b:
                raise ScheduleError(f"cron value {part} outside [{lo}, {hi}]")
            out.update(range(a, b + 1, step))
        return out

    def matches(self, t: float) -> bool:
        tm = time.gmtime(t)
        mi, hr, dom, mon, dow = tm.tm_min, tm.tm_hour, tm.tm_mday, tm.tm_mon, (tm.tm_wday + 1) % 7
        if mi not in self.sets[0] or hr not in self.sets[1] or mon not in self.sets[3]:
            return False
        dom_ok, dow_ok = dom in self.sets[2], dow in self.sets[4]
        if self.restricted[2] and self.restricted[4]:
            return dom_ok or dow_ok
        return dom_ok and dow_ok

    def next_after(self, t: float) -> float:
        """First matching minute strictly after ``t``."""
        m = (int(t) // 60 + 1) * 60
        end = m + 4 * 366 * 86400
        while m < end:
            tm = time.gmtime(m)
            if tm.tm_mon not in self.sets[3]:  # skip to the first minute of the next month
                y, mo = tm.tm_year + (tm.tm_mon == 12), tm.tm_mon % 12 + 1
                m = calendar.timegm((y, mo, 1, 0, 0, 0))
                continue
            if not self._day_ok(tm):
                m = calendar.timegm((tm.tm_year, tm.tm_mon, tm.tm_mday, 0, 0, 0)) + 86400
                continue
            if tm.tm_hour not in self.sets[1]:
                m = calendar.timegm((tm.tm_year, tm.tm_mon, tm.tm_mday, tm.tm_hour, 0, 0)) + 3600
                continue
            if tm.tm_min in self.sets[0]:
                return float(m)
            m += 60
        raise ScheduleError(f"cron {self.expr!r} never fires")

    def _day_ok(self, tm) -> bool:
        dom_ok = tm.tm_mday in self.sets[2]
        dow_ok = (tm.tm_wday + 1) % 7 in self.sets[4]
        if self.restricted[2] and self.restricted[4]:
            return dom_ok or dow_ok
        return dom_ok and dow_ok


@dataclass
class Schedule:
    frequency: Optional[float] = None
    cron: Optional[Cron] = None
    start_at: Optional[float] = None
    end_at: Optional[float] = None
    depends_on_past: bool = False
    max_runs: Optional[int] = None

    @classmethod
    def from_dict(cls, d: Optional[Dict[str, Any]]) -> Optional["Schedule"]:
        if not d:
            return None
        if not isinstance(d, dict):
            raise ScheduleError("schedule must be a mapping")
        unknown = set(d) - {"frequency", "cron", "start_at", "end_at", "depends_on_past", "max_runs", "execute_at"}
        if unknown:
            raise ScheduleError(f"unknown schedule keys {sorted(unknown)}")
        if d.get("frequency") is not None and d.get("cron"):
            raise ScheduleError("a schedule has either `frequency` or `cron`, not both")
        s = cls(frequency=parse_frequency(d["frequency"]) if d.get("frequency") is not None else None,
                cron=Cron(str(d["cron"])) if d.get("cron") else None,
                start_at=parse_time(d.get("start_at", d.get("execute_at"))), end_at=parse_time(d.get("end_at")),
                depends_on_past=bool(d.get("depends_on_past", False)),
                max_runs=int(d["max_runs"]) if d.get("max_runs") is not None else None)
        if s.start_at is not None and s.end_at is not None and s.end_at < s.start_at:
            raise ScheduleError("schedule end_at is before start_at")
        if s.max_runs is not None and s.max_runs < 1:
            raise ScheduleError("schedule max_runs must be >= 1")
        return s

    @property
    def periodic(self) -> bool:
        return self.frequency is not None or self.cron is not None

    def first(self, now: float) -> float:
        t = self.start_at if self.start_at is not None else now
        if self.cron is not None and not self.cron.matches(t):
            t = self.cron.next_after(t)
        return t

    def next(self, prev_scheduled: float) -> Optional[float]:
        if self.frequency is not None:
            t = prev_scheduled + self.frequency
        elif self.cron is not None:
            t = self.cron.next_after(prev_scheduled)
        else:
            return None
        if self.end_at is not None and t > self.end_at:
            return None
        return t


class PipelineSchedule:
    """Fires pipeline runs on the scheduler thread.  ``runners`` keeps every run's PipelineRunner."""

    def __init__(self, flow, pipeline_id: int, spec, project: Dict, user: str, cwd: str, schedule: Schedule):
        self.flow = flow
        self.pipeline_id = pipeline_id
        self.spec, self.project, self.user, self.cwd = spec, project, user, cwd
        self.schedule = schedule
        self.runners: List[Any] = []
        self.fired = 0
        self.stopped = False
        self.next_at: Optional[float] = None
        self._waiting: Optional[float] = None  # depends_on_past: scheduled time held until the previous run ends

    def start(self) -> Optional[int]:
        """Arm the first run (or start it now).  Returns the run id when one started immediately."""
        t = self.schedule.first(time.time())
        if self.schedule.end_at is not None and t > self.schedule.end_at:
            self.stopped = True
            return None
        return self._arm(t)

    def _arm(self, t: float) -> Optional[int]:
        self.next_at = t
        self.flow.store.kv_set(f"pipeline_schedule:{self.pipeline_id}", {"next_at": t, "fired": self.fired})
        delay = t - time.time()
        if delay <= 0:
            return self._fire(t)
        self.flow.after(delay, lambda t=t: self._fire(t))
        return None

    def _fire(self, scheduled: float) -> Optional[int]:
        if self.stopped or scheduled != self.next_at:
            return None
        prev = self.runners[-1] if self.runners else None
        rid = None
        if self.schedule.depends_on_past and prev is not None and not prev.finished:
            self._waiting = scheduled  # run when the previous one finishes
            return None
        if self.schedule.depends_on_past and prev is not None and not prev.succeeded:
            rid = self._skip()
        else:
            rid = self._launch()
        self.fired += 1
        self._arm_next(scheduled)
        return rid

    def _arm_next(self, scheduled: float) -> None:
        if self.schedule.max_runs is not None and self.fired >= self.schedule.max_runs:
            self.stopped = True
            self.next_at = None
            return
        nxt = self.schedule.next(scheduled)
        if nxt is None:
            self.stopped = True
            self.next_at = None
            return
        self._arm(nxt)

    def _launch(self) -> int:
        from polyaxon_amd.polyflow.pipelines import PipelineRunner

        r = PipelineRunner(self.flow, self.pipeline_id, self.spec, self.project, self.user, self.cwd)
        r.on_finished.append(self._on_run_finished)
        self.runners.append(r)
        return r.start()

    def _skip(self) -> int:
        """depends_on_past and the previous run did not succeed: record the run as skipped."""
        rid = self.flow.store.create_pipeline_run(self.pipeline_id)
        self.flow.store.set_pipeline_run_status(rid, "skipped")
        self.flow.auditor.record("pipeline.stopped", "pipeline", self.pipeline_id, run=rid,
                                 reason="depends_on_past: previous run did not succeed")
        return rid

    def _on_run_finished(self, runner) -> None:
        if self._waiting is None or runner is not self.runners[-1]:
            return
        t, self._waiting = self._waiting, None
        if self.stopped:
            return
        if runner.succeeded:
            self._launch()
        else:
            self._skip()
        self.fired += 1
        self._arm_next(t)

    def stop(self) -> None:
        self.stopped = True
        self.next_at = None
        for r in self.runners:
            if not r.finished:
                r.stop()

    @property
    def run_id(self) -> Optional[int]:
        return self.runners[-1].run_id if self.runners else None
