"""Experiment-group lifecycle on the CPU scheduler: user stop (pending only vs all), Hyperband RESTART
promotions, BO iteration rows and maximise-direction early stopping.

Reference behaviour pinned here:
* ``stop pending`` finishes only the not-yet-started experiments; running ones complete
  (polyaxon/scheduler/tasks/experiment_groups.py:50-73, tests/test_experiment_groups/test_models.py:535-622);
* ``stop all`` also stops running experiments and the group ends STOPPED;
* Hyperband ``resume: false`` promotes with RESTART clones, which get their own outputs path
  (iteration_managers/hyperband.py:79-113, libs/paths/experiments.py:11-23);
* BO iterations persist ``experiment_ids`` and the combined ``experiments_metrics`` of all earlier
  iterations (iteration_managers/bayesian_optimization.py:9-37);
* early stopping with ``optimization: maximize`` triggers on ``last_metric >= value``
  (db/models/experiment_groups.py:211-221).
"""
import os
import sys
import time

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow

PY = sys.executable
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TRIAL = ("from polyaxon_amd.client import Experiment, get_declarations; import time; d = get_declarations(); "
         "e = Experiment(); time.sleep(float(d.get('sleep', 0.05))); "
         "e.log_metrics(step=1, loss=(d['lr'] - 0.3) ** 2 + 1.0 / float(d.get('steps', 1)), acc=d['lr']); e.close()")


def _flow(tmp_path, n_gpus=1):
    alloc = DeviceAllocator([Device(i) for i in range(n_gpus)])
    return Polyflow(str(tmp_path / "plx"), allocator=alloc, stop_grace_s=1.0).start()


def _group(algo_block, matrix, concurrency):
    return {"version": 1, "kind": "group",
            "hptuning": {"concurrency": concurrency, "matrix": matrix, **algo_block},
            "run": {"cmd": f"PYTHONPATH={ROOT} {PY} -c \"{TRIAL}\""}}


def _wait_running(flow, gid, n, timeout=30):
    deadline = time.time() + timeout
    while time.time() < deadline:
        xps = flow.store.list_experiments(group_id=gid)
        if sum(x["status"] == "running" for x in xps) >= n:
            return xps
        time.sleep(0.02)
    raise AssertionError("group experiments never reached running")


def test_stop_pending_lets_running_experiments_finish(tmp_path):
    flow = _flow(tmp_path)
    try:
        g = flow.submit(_group({}, {"lr": {"values": [0.1, 0.2, 0.3, 0.4, 0.5]}, "sleep": {"values": [1.5]}}, 2))
        _wait_running(flow, g["id"], 2)
        flow.stop_group(g["id"], pending=True)
        # the group is STOPPED at once (reference view sets it); the running trials still run to completion
        assert flow.wait("group", g["id"], timeout=60) == "stopped"
        for x in flow.store.list_experiments(group_id=g["id"]):
            flow.wait("experiment", x["id"], timeout=30)
        st = sorted(x["status"] for x in flow.store.list_experiments(group_id=g["id"]))
        assert st == ["stopped", "stopped", "stopped", "succeeded", "succeeded"]
    finally:
        flow.shutdown()


def test_stop_all_stops_running_experiments(tmp_path):
    flow = _flow(tmp_path)
    try:
        g = flow.submit(_group({}, {"lr": {"values": [0.1, 0.2, 0.3, 0.4]}, "sleep": {"values": [30.0]}}, 2))
        _wait_running(flow, g["id"], 2)
        t0 = time.time()
        flow.stop_group(g["id"], pending=False)
        assert flow.wait("group", g["id"], timeout=30) == "stopped"
        for x in flow.store.list_experiments(group_id=g["id"]):
            flow.wait("experiment", x["id"], timeout=15)
        assert time.time() - t0 < 15  # running trials were signalled, not waited out
        xps = flow.store.list_experiments(group_id=g["id"])
        assert sorted(x["status"] for x in xps) == ["stopped"] * 4
        assert [s["status"] for s in flow.store.group_statuses(g["id"])][-1] == "stopped"
    finally:
        flow.shutdown()


def test_hyperband_restart_promotions_get_fresh_outputs(tmp_path):
    flow = _flow(tmp_path)
    try:
        hb = {"hyperband": {"max_iter": 3, "eta": 3, "resource": {"name": "steps", "type": "int"},
                            "metric": {"name": "loss", "optimization": "minimize"}, "resume": False}, "seed": 5}
        g = flow.submit(_group(hb, {"lr": {"values": [0.1, 0.2, 0.3, 0.4, 0.5]}}, 3))
        assert flow.wait("group", g["id"], timeout=120) == "succeeded"
        xps = flow.store.list_experiments(group_id=g["id"])
        promoted = [x for x in xps if x["original_experiment_id"] is not None]
        assert promoted and all(x["cloning_strategy"] == "restart" for x in promoted)
        for x in promoted:
            orig = flow.store.get_experiment(x["original_experiment_id"])
            assert x["outputs_path"] != orig["outputs_path"]
            assert x["declarations"]["steps"] == 3 and orig["declarations"]["steps"] == 1
            assert x["declarations"]["lr"] == orig["declarations"]["lr"]
        # every rung is recorded with the metrics it was reduced from
        for it in flow.store.iterations(g["id"]):
            d = it["data"]
            assert {x for x, _ in d["experiments_metrics"]} == set(d["experiment_ids"])
    finally:
        flow.shutdown()


def test_bo_iterations_persist_combined_metrics(tmp_path):
    flow = _flow(tmp_path)
    try:
        bo = {"bo": {"n_iterations": 2, "n_initial_trials": 2, "metric": {"name": "loss", "optimization": "minimize"},
                     "utility_function": {"acquisition_function": "ei", "eps": 0.0,
                                          "gaussian_process": {"kernel": "rbf", "length_scale": 1.0}}}, "seed": 7}
        g = flow.submit(_group(bo, {"lr": {"uniform": [0.0, 1.0]}}, 2))
        assert flow.wait("group", g["id"], timeout=120) == "succeeded"
        its = [i["data"] for i in flow.store.iterations(g["id"])]
        assert [d["iteration"] for d in its] == [0, 1, 2]
        assert [len(d["experiment_ids"]) for d in its] == [2, 1, 1]
        # metrics accumulate across iterations (combined observations feed the GP)
        assert [len(d["experiments_metrics"]) for d in its] == [2, 3, 4]
        xps = flow.store.list_experiments(group_id=g["id"])
        assert len(xps) == 4 and all(0.0 <= x["declarations"]["lr"] <= 1.0 for x in xps)
    finally:
        flow.shutdown()


def test_early_stopping_maximize(tmp_path):
    flow = _flow(tmp_path)
    try:
        spec = _group({"early_stopping": [{"metric": "acc", "value": 0.25, "optimization": "maximize"}]},
                      {"lr": {"values": [0.1, 0.3, 0.05, 0.02]}}, 1)
        g = flow.submit(spec)
        assert flow.wait("group", g["id"], timeout=60) == "stopped"
        xps = sorted(flow.store.list_experiments(group_id=g["id"]), key=lambda x: x["id"])
        # trial 1 (acc 0.1) does not trigger; trial 2 (acc 0.3 >= 0.25) does; the rest never start
        assert [x["status"] for x in xps] == ["succeeded", "succeeded", "stopped", "stopped"]
    finally:
        flow.shutdown()
