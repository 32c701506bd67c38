"""The polyflow scheduler process stays free of device work: a BO group's GP fit + acquisition search runs on the
group's resident executor (``bo_suggest``), never in the scheduler.  The scheduler runs in a
fresh subprocess, so nothing else in the test session can have touched the GPU or imported torch there."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCHEDULER = r"""
import json, os, sys
from polyaxon_amd.polyflow.scheduler import Polyflow

hp = {"seed": 3, "concurrency": 1,
      "bo": {"n_initial_trials": 2, "n_iterations": 1, "metric": {"name": "loss", "optimization": "minimize"},
             "utility_function": {"acquisition_function": "ucb", "kappa": 1.5,
                                  "gaussian_process": {"kernel": "matern", "length_scale": 1.0, "nu": 1.5},
                                  "n_warmup": 1000, "n_iter": 3}},
      "matrix": {"lr": {"loguniform": [-9, -3]}, "weight_decay": {"uniform": [0.0, 0.2]}}}
spec = {"version": 1, "kind": "group", "project": "gpufree", "hptuning": hp,
        "environment": {"resources": {"gpu": 1},
                        "executor": {"kind": "resident", "program": "gpt2_tiny",
                                     "params": {"batch": 2, "seq": 32, "unit_steps": 2, "trial_units": 2}}}}
with Polyflow(sys.argv[1], reconcile_s=0) as flow:
    r = flow.submit(spec)
    status = flow.wait("group", r["id"], timeout=240)
    its = sorted(flow.store.iterations(r["id"]), key=lambda i: i["data"]["iteration"])
    n = len(flow.store.list_experiments(group_id=r["id"]))
maps = open("/proc/self/maps").read()
fds = []
for f in os.listdir("/proc/self/fd"):
    try:
        fds.append(os.readlink("/proc/self/fd/" + f))
    except OSError:
        pass
print(json.dumps({"status": status, "experiments": n, "suggest": [i["data"].get("suggest") for i in its],
                  "hip_mapped": "libamdhip64" in maps, "kfd_open": any("/dev/kfd" in x for x in fds),
                  "torch_imported": "torch" in sys.modules}))
"""


def _run_scheduler(tmp_path, env_extra):
    env = dict(os.environ, PYTHONPATH=REPO, **env_extra)
    out = subprocess.run([sys.executable, "-c", SCHEDULER, str(tmp_path)], capture_output=True, text=True,
                         timeout=290, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_scheduler_process_never_imports_torch_for_bo(tmp_path):
    """CPU executors: the BO iteration's suggestions come from the executor (numpy there) and the scheduler process
    never imports torch."""
    r = _run_scheduler(tmp_path, {"PLX_CPU_ONLY": "1", "PLX_NUM_GPUS": "1", "OMP_NUM_THREADS": "2"})
    assert r["status"] == "succeeded" and r["experiments"] == 3, r
    assert r["suggest"][1]["where"].startswith("executor"), r
    assert not r["torch_imported"] and not r["hip_mapped"] and not r["kfd_open"], r


@pytest.mark.gpu
def test_bo_group_gp_runs_on_the_executor_and_the_scheduler_stays_gpu_free(tmp_path):
    """A BO group through polyflow on one MI355X: the GP of the BO iteration runs with the HIP kernels on the
    resident executor's device; the scheduler process has no /dev/kfd descriptor, no libamdhip64 mapping and never
    imported torch."""
    r = _run_scheduler(tmp_path, {})
    assert r["status"] == "succeeded" and r["experiments"] == 3, r
    s = r["suggest"][1]
    assert s["where"].startswith("executor") and s["backend"] == "hip", r
    assert not r["kfd_open"] and not r["hip_mapped"] and not r["torch_imported"], r


@pytest.mark.gpu
def test_device_detection_without_hip_matches_the_runtime():
    """The scheduler counts devices from the KFD topology and the render nodes it can see (no HIP runtime); the
    count equals what the HIP runtime enumerates."""
    code = ("import json, torch; from polyaxon_amd.polyflow.devices import detect_devices; "
            "print(json.dumps([len(detect_devices()), torch.cuda.device_count()]))")
    env = {k: v for k, v in os.environ.items() if k != "PLX_NUM_GPUS"}
    env["PYTHONPATH"] = REPO
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    mine, hip = json.loads(out.stdout.strip().splitlines()[-1])
    assert mine == hip >= 1


STATUS_API = r"""
import json, os, sys
from fastapi.testclient import TestClient
from polyaxon_amd.api.server import create_app
from polyaxon_amd.polyflow.scheduler import Polyflow
from polyaxon_amd.polyflow.devices import Device, DeviceAllocator

flow = Polyflow(sys.argv[1], allocator=DeviceAllocator([Device(0)]), reconcile_s=0).start()
client = TestClient(create_app(flow, admin_token="t"))
first = client.get("/_status").json()
second = client.get("/_status").json()
flow.shutdown()
maps = open("/proc/self/maps").read()
print(json.dumps({"first": first, "second": second["checks"]["rccl"], "hip_mapped": "libamdhip64" in maps,
                  "torch_imported": "torch" in sys.modules}))
"""


def _status_api(tmp_path, env_extra):
    env = dict(os.environ, PYTHONPATH=REPO, **env_extra)
    out = subprocess.run([sys.executable, "-c", STATUS_API, str(tmp_path)], capture_output=True, text=True,
                         timeout=240, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_status_endpoint_keeps_the_api_process_gpu_free(tmp_path):
    """``/_status``'s RCCL check runs in a child process (obs/rccl_probe.py): the API process never imports torch
    nor maps the HIP runtime, and a second poll is served from the check's cache.  On this CPU box the probe
    reports "skipped" (no device), which counts as healthy."""
    r = _status_api(tmp_path, {"OMP_NUM_THREADS": "2"})
    rccl = r["first"]["checks"]["rccl"]
    assert rccl["status"] == "ok" and rccl["cached"] is False, r
    assert r["second"]["cached"] is True, r
    assert not r["torch_imported"] and not r["hip_mapped"], r


@pytest.mark.gpu
def test_status_endpoint_runs_a_real_rccl_round_trip(tmp_path):
    """On the GPU box the check is a real RCCL all-reduce on the framework communicator, in a child process: status
    ok with a measured latency, and still no HIP runtime in the API process (reference
    /root/reference/polyaxon/checks/worker.py:16-45)."""
    r = _status_api(tmp_path, {})
    rccl = r["first"]["checks"]["rccl"]
    assert rccl["status"] == "ok" and not rccl.get("skipped") and rccl["all_reduce_us"] > 0, r
    assert not r["torch_imported"] and not r["hip_mapped"], r
