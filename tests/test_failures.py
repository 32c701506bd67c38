"""Failure detection / opt-in retry / fault injection / heartbeats and the async
checkpoint + tracing helpers (§5.4, §5.1). CPU only: trials are real subprocesses."""
import sys
import time

import pytest
import torch

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.faults import parse_fault
from polyaxon_amd.polyflow.scheduler import Polyflow

PY = sys.executable


def _flow(tmp_path, **kw):
    alloc = DeviceAllocator([Device(i) for i in range(2)])
    return Polyflow(str(tmp_path / "plx"), allocator=alloc, stop_grace_s=1.0, **kw).start()


def _xp(cmd, **env):
    return {"version": 1, "kind": "experiment", "run": {"cmd": cmd}, "environment": env}


def _last_message(flow, xid):
    return flow.store.experiment_statuses(xid)[-1]["message"] or ""


def test_parse_fault():
    assert parse_fault("kill_rank:1@step:100") == {"rank": 1, "at": "step", "value": 100}
    assert parse_fault("kill_rank:0@t:2.5") == {"rank": 0, "at": "t", "value": 2.5}
    assert parse_fault("explode") is None and parse_fault("kill_rank:x@t:1") is None


def test_time_fault_fails_without_retry(tmp_path):
    flow = _flow(tmp_path)
    try:
        r = flow.submit(_xp("sleep 20", env_vars=[["POLYFLOW_FAULT", "kill_rank:0@t:0.3"]]))
        t0 = time.time()
        assert flow.wait("experiment", r["id"], timeout=30) == "failed"
        assert time.time() - t0 < 10
        assert "signal 9" in _last_message(flow, r["id"])
        assert flow.stats["faults_injected"] == 1
    finally:
        flow.shutdown()


def test_opt_in_retry_recovers(tmp_path):
    flow = _flow(tmp_path)
    try:
        cmd = 'if [ "$POLYAXON_RESTART_COUNT" = 0 ]; then sleep 20; fi; echo attempt=$POLYAXON_RESTART_COUNT'
        r = flow.submit(_xp(cmd, max_restarts=2, env_vars=[["POLYFLOW_FAULT", "kill_rank:0@t:0.3"]]))
        assert flow.wait("experiment", r["id"], timeout=30) == "succeeded"
        statuses = [s["status"] for s in flow.store.experiment_statuses(r["id"])]
        assert "retrying" in statuses and statuses[-1] == "succeeded"
        assert flow.stats["retries"] == 1
        assert "attempt=1" in flow.logs("experiment", r["id"])
        assert len(flow.store.experiment_jobs(r["id"])) == 2  # one job row per attempt
    finally:
        flow.shutdown()


def test_retry_budget_exhausted(tmp_path):
    flow = _flow(tmp_path)
    try:
        r = flow.submit(_xp("exit 3", max_restarts=2))
        assert flow.wait("experiment", r["id"], timeout=30) == "failed"
        assert flow.stats["retries"] == 2
        assert len(flow.store.experiment_jobs(r["id"])) == 3
    finally:
        flow.shutdown()


def test_step_fault_from_tracking_client(tmp_path):
    flow = _flow(tmp_path)
    try:
        script = ("from polyaxon_amd.client.tracking import Experiment; x = Experiment(async_metrics=False); "
                  "[x.log_metrics(step=i, loss=1.0 / (i + 1)) for i in range(6)]; print('done')")
        r = flow.submit(_xp(f"{PY} -c \"{script}\"", max_restarts=1,
                            env_vars=[["POLYFLOW_FAULT", "kill_rank:0@step:3"]]))
        assert flow.wait("experiment", r["id"], timeout=60) == "succeeded"
        assert flow.stats["retries"] == 1
        steps = [m["step"] for m in flow.store.get_metrics(r["id"])]
        assert steps == [0, 1, 2, 0, 1, 2, 3, 4, 5]  # first attempt died at step 3, second ran through
    finally:
        flow.shutdown()


def test_distributed_fault_tears_down_surviving_ranks(tmp_path):
    flow = _flow(tmp_path)
    try:
        r = flow.submit(_xp("sleep 30", pytorch={"n_workers": 1},
                            env_vars=[["POLYFLOW_FAULT", "kill_rank:1@t:0.3"]]))
        t0 = time.time()
        assert flow.wait("experiment", r["id"], timeout=30) == "failed"
        assert time.time() - t0 < 10
        jobs = {j["role"]: j["status"] for j in flow.store.experiment_jobs(r["id"])}
        assert jobs == {"master": "stopped", "worker": "failed"}
    finally:
        flow.shutdown()


def test_heartbeat_timeout_kills_hung_trial(tmp_path):
    flow = _flow(tmp_path, reconcile_s=0.2)
    try:
        r = flow.submit(_xp("sleep 30", heartbeat_timeout=0.8))
        t0 = time.time()
        assert flow.wait("experiment", r["id"], timeout=30) == "failed"
        assert time.time() - t0 < 10
        assert "no heartbeat" in _last_message(flow, r["id"])
        # a trial that beats stays alive past the deadline
        script = ("import time; from polyaxon_amd.client.tracking import Experiment; x = Experiment(); "
                  "[(x.heartbeat(), time.sleep(0.2)) for _ in range(10)]")
        r2 = flow.submit(_xp(f"{PY} -c \"{script}\"", heartbeat_timeout=1.5))
        assert flow.wait("experiment", r2["id"], timeout=60) == "succeeded"
    finally:
        flow.shutdown()


def test_health_check_cordons_devices(tmp_path):
    flow = _flow(tmp_path, reconcile_s=0.1, health_check=lambda: [1])
    try:
        time.sleep(0.5)
        assert [d["healthy"] for d in flow.alloc.snapshot()] == [True, False]
    finally:
        flow.shutdown()


def test_async_checkpointer_roundtrip(tmp_path):
    from polyaxon_amd.client.checkpoint import AsyncCheckpointer

    ck = AsyncCheckpointer(str(tmp_path))
    w = torch.randn(64, 32)
    ref = w.clone()
    ck.save({"w": w, "step": torch.tensor([7])}, meta={"step": 7})
    w.add_(1.0)  # mutation after save() must not leak into the checkpoint
    ck.wait()
    got = ck.load()
    assert torch.equal(got["w"], ref) and int(got["step"]) == 7
    assert ck.meta()["step"] == "7"
    assert ck.load("missing") is None


def test_trace_range_records(monkeypatch):
    from polyaxon_amd.obs import tracing

    monkeypatch.setattr(tracing, "_RECORD", True)
    tracing.SPANS.clear()
    with tracing.trace_range("outer"):
        with tracing.trace_range("inner"):
            pass
    assert [s["name"] for s in tracing.SPANS] == ["inner", "outer"]
