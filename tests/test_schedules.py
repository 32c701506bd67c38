"""Pipeline schedules (reference Schedule model, polyaxon/db/models/pipelines.py:23-47): frequency / cron parsing,
start_at / end_at windows, max_runs, depends_on_past, stop."""
import calendar
import sys
import time

import pytest

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow
from polyaxon_amd.polyflow.schedules import Cron, Schedule, ScheduleError, parse_frequency, parse_time
from polyaxon_amd.spec import specification_for
from polyaxon_amd.spec.specification import PolyaxonfileError

PY = sys.executable


def test_frequency_and_time_parsing():
    assert parse_frequency(30) == 30 and parse_frequency("45") == 45
    assert parse_frequency("1h30m") == 5400 and parse_frequency("2d") == 172800 and parse_frequency("1w") == 604800
    for bad in ("soon", "-3", "1x", 0):
        with pytest.raises(ScheduleError):
            parse_frequency(bad)
    assert parse_time("2026-01-01T00:00:00") == calendar.timegm((2026, 1, 1, 0, 0, 0))
    assert parse_time("2026-01-01T01:00:00+01:00") == calendar.timegm((2026, 1, 1, 0, 0, 0))
    assert parse_time(123.5) == 123.5 and parse_time(None) is None


def test_cron_next_after():
    t0 = calendar.timegm((2026, 10, 16, 12, 7, 30))  # a Friday
    c = Cron("*/15 * * * *")
    assert c.next_after(t0) == calendar.timegm((2026, 10, 16, 12, 15, 0))
    c = Cron("0 9-17 * * 1-5")  # top of the hour, business hours, weekdays
    assert c.next_after(t0) == calendar.timegm((2026, 10, 16, 13, 0, 0))
    late = calendar.timegm((2026, 10, 16, 17, 30, 0))
    assert c.next_after(late) == calendar.timegm((2026, 10, 19, 9, 0, 0))  # Monday
    c = Cron("30 2 1 * *")
    assert c.next_after(t0) == calendar.timegm((2026, 11, 1, 2, 30, 0))
    c = Cron("0 0 29 2 *")  # leap day
    assert c.next_after(t0) == calendar.timegm((2028, 2, 29, 0, 0, 0))
    c = Cron("0 12 13 * 5")  # the 13th OR a Friday (both day fields restricted)
    assert c.next_after(calendar.timegm((2026, 10, 16, 12, 0, 0))) == calendar.timegm((2026, 10, 23, 12, 0, 0))
    for bad in ("* * * *", "61 * * * *", "*/0 * * * *", "5-2 * * * *"):
        with pytest.raises(ScheduleError):
            Cron(bad)


def test_schedule_windows():
    s = Schedule.from_dict({"frequency": "10s", "start_at": 1000, "end_at": 1025})
    assert s.first(500) == 1000 and s.next(1000) == 1010 and s.next(1010) == 1020 and s.next(1020) is None
    with pytest.raises(ScheduleError):
        Schedule.from_dict({"frequency": 10, "cron": "* * * * *"})
    with pytest.raises(ScheduleError):
        Schedule.from_dict({"frequency": 10, "start_at": 10, "end_at": 5})
    c = Schedule.from_dict({"cron": "*/5 * * * *"})
    t = c.first(calendar.timegm((2026, 1, 1, 0, 1, 0)))
    assert t == calendar.timegm((2026, 1, 1, 0, 5, 0))


def _pipeline(cmd, schedule, ops=None):
    return {"version": 1, "kind": "pipeline", "schedule": schedule,
            "ops": ops or [{"name": "a", "template": {"version": 1, "kind": "job", "run": {"cmd": cmd}}}]}


def test_spec_rejects_bad_schedule():
    with pytest.raises(PolyaxonfileError):
        specification_for(_pipeline("true", {"frequency": "often"}))
    with pytest.raises(PolyaxonfileError):
        specification_for(_pipeline("true", {"cron": "* *"}))
    assert specification_for(_pipeline("true", {"frequency": 1, "max_runs": 2})).schedule["max_runs"] == 2


def _flow(tmp_path):
    return Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0)]), reconcile_s=0).start()


def _runs(flow, pid):
    return flow.store._rows(flow.store.execute("SELECT * FROM pipeline_runs WHERE pipeline_id = ? ORDER BY id", (pid,)))


def _wait_runs(flow, pid, n, timeout=30):
    end = time.time() + timeout
    while time.time() < end:
        rs = _runs(flow, pid)
        if len(rs) >= n and all(r["status"] in ("finished", "stopped", "skipped") for r in rs[:n]):
            return rs
        time.sleep(0.05)
    raise TimeoutError(f"pipeline {pid}: {[r['status'] for r in _runs(flow, pid)]}")


def test_periodic_runs_with_max_runs(tmp_path):
    flow = _flow(tmp_path)
    try:
        r = flow.submit(_pipeline("true", {"frequency": 0.4, "max_runs": 3}))
        assert r["run_id"] is not None  # start_at defaults to now: the first run starts at once
        rs = _wait_runs(flow, r["id"], 3)
        time.sleep(0.8)
        rs = _runs(flow, r["id"])
        assert len(rs) == 3 and all(x["status"] == "finished" for x in rs)
        starts = [x["started_at"] for x in rs]
        assert all(0.3 < b - a < 1.5 for a, b in zip(starts, starts[1:]))  # ~frequency apart, no drift pile-up
        # every run executed its op
        assert all(len(flow.store.operation_runs(x["id"])) == 1 for x in rs)
    finally:
        flow.shutdown()


def test_start_at_in_future_and_end_at(tmp_path):
    flow = _flow(tmp_path)
    try:
        now = time.time()
        r = flow.submit(_pipeline("true", {"frequency": 0.3, "start_at": now + 0.5, "end_at": now + 1.25}))
        assert r["run_id"] is None and r["next_at"] == pytest.approx(now + 0.5)
        time.sleep(0.2)
        assert _runs(flow, r["id"]) == []
        rs = _wait_runs(flow, r["id"], 3, timeout=10)
        time.sleep(0.6)
        assert len(_runs(flow, r["id"])) == 3  # 0.5, 0.8, 1.1 -- 1.4 is past end_at
    finally:
        flow.shutdown()


def test_depends_on_past_waits_and_skips_after_failure(tmp_path, monkeypatch):
    flow = _flow(tmp_path)
    marker = tmp_path / "fail_now"
    try:
        # run k takes 0.6 s > frequency: with depends_on_past the next run waits for it instead of overlapping
        cmd = f"sleep 0.6; test ! -e {marker}"
        r = flow.submit(_pipeline(cmd, {"frequency": 0.2, "depends_on_past": True, "max_runs": 4}))
        rs = _wait_runs(flow, r["id"], 2, timeout=20)
        assert rs[1]["started_at"] >= rs[0]["finished_at"] - 0.05  # sequential, never overlapping
        marker.write_text("x")  # the next run fails ...
        rs = _wait_runs(flow, r["id"], 4, timeout=20)
        st = [x["status"] for x in rs]
        ops = [flow.store.operation_runs(x["id"]) for x in rs]
        failed = [i for i, o in enumerate(ops) if o and o[0]["status"] == "failed"]
        assert failed, st
        k = failed[0]
        assert all(s == "skipped" for s in st[k + 1:])  # ... so the ones after it are skipped
    finally:
        flow.shutdown()


def test_stop_scheduled_pipeline(tmp_path):
    flow = _flow(tmp_path)
    try:
        r = flow.submit(_pipeline("true", {"frequency": 0.2}))
        _wait_runs(flow, r["id"], 2)
        assert flow.stop_pipeline(r["id"])
        n = len(_runs(flow, r["id"]))
        time.sleep(0.6)
        assert len(_runs(flow, r["id"])) <= n + 1
        m = len(_runs(flow, r["id"]))
        time.sleep(0.5)
        assert len(_runs(flow, r["id"])) == m
    finally:
        flow.shutdown()
