"""Distributed runner end to end on CPU (the PyTorchJob equivalent): polyflow launches a DP=2
``pytorch`` experiment whose ranks are the real LM trainer; they rendezvous from the env contract (MASTER_ADDR /
MASTER_PORT / WORLD_SIZE / RANK), train through FlatDDP over gloo, rank 0's metrics land in the store; a killed
worker fails the experiment and the surviving rank is torn down (reference constants/experiments.py:97-120)."""
import os
import sys

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow

PY = sys.executable
CMD = f"{PY} -m polyaxon_amd.trainers lm --model tiny --cpu --bs 2 --seq 16 --log_every 2"


def _flow(tmp_path):
    return Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0), Device(1)]), reconcile_s=0,
                    stop_grace_s=2.0).start()


def _spec(steps, **env):
    e = {"pytorch": {"n_workers": 1}, "env_vars": [["OMP_NUM_THREADS", "2"]]}
    e.update(env)
    return {"version": 1, "kind": "experiment", "run": {"cmd": f"{CMD} --steps {steps}"}, "environment": e}


def test_dp2_lm_trainer_through_polyflow(tmp_path):
    flow = _flow(tmp_path)
    try:
        r = flow.submit(_spec(6), project="dist")
        assert flow.wait("experiment", r["id"], timeout=240) == "succeeded", flow.logs("experiment", r["id"])[-3000:]
        jobs = flow.store.experiment_jobs(r["id"])
        assert sorted((j["role"], j["status"]) for j in jobs) == [("master", "succeeded"), ("worker", "succeeded")]
        last = flow.store.get_experiment(r["id"])["last_metric"]
        assert "loss" in last and "tokens_per_s" in last
        logs = flow.logs("experiment", r["id"])
        assert '"world": 2' in logs  # rank 0 reports the DP world it trained in
        # gradient buckets planned for 2 ranks from all-reduces timed on the trial's communicator at start-up
        # (parallel/comm_plan.py calibrate; the trainer's --bucket_mb auto), or the xGMI link model when the timings
        # of a loaded CPU host do not fit a line
        assert '"bucket_plan": {"bucket_bytes"' in logs
        assert '"world": 2, "source": "measured"' in logs or '"world": 2, "source": "link-model"' in logs
        steps = [m["step"] for m in flow.store.get_metrics(r["id"])]
        assert 6 in steps
    finally:
        flow.shutdown()


def test_killed_worker_fails_the_dp_experiment(tmp_path):
    flow = _flow(tmp_path)
    try:
        spec = _spec(100000)
        spec["environment"]["env_vars"].append(["POLYFLOW_FAULT", "kill_rank:1@t:3"])
        spec["environment"]["env_vars"].append(["PLX_COLLECTIVE_TIMEOUT_S", "20"])
        r = flow.submit(spec, project="dist")
        assert flow.wait("experiment", r["id"], timeout=120) == "failed"
        jobs = {j["role"]: j for j in flow.store.experiment_jobs(r["id"])}
        assert jobs["worker"]["status"] == "failed"
        assert jobs["master"]["status"] in ("stopped", "failed")
        assert flow.stats["faults_injected"] == 1
        assert flow.call(lambda: dict(flow.alloc.allocations)) == {}
    finally:
        flow.shutdown()


def test_dp2_lm_trainer_zero1_through_polyflow(tmp_path):
    """The same DP=2 job with ``--zero1`` (reduce-scatter, AdamW on each rank's half, all-gather): it succeeds and
    lands the same final loss as the all-reduce run (ZeRO-1 is bitwise the unsharded trajectory)."""
    flow = _flow(tmp_path)
    try:
        losses = {}
        for zero in (False, True):
            spec = _spec(6)
            if zero:
                spec["run"]["cmd"] += " --zero1"
            r = flow.submit(spec, project="dist")
            assert flow.wait("experiment", r["id"], timeout=240) == "succeeded", flow.logs("experiment", r["id"])[-3000:]
            losses[zero] = flow.store.get_experiment(r["id"])["last_metric"]["loss"]
        assert losses[True] == losses[False]
    finally:
        flow.shutdown()
