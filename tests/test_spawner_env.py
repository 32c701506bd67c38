"""Per-framework topology and the in-trial environment contract, as pure functions.

Covers what the reference checks in tests/test_spawner/test_env_vars.py and the framework spawners
(pytorch_spawner.py:12-25,94-121; tensorflow_spawner.py:14-24,117-123; mxnet_spawner.py:13-29,122-128;
horovod_spawner.py; templates/experiment_jobs/pods.py:151-159,243-249), with the MI355X device wiring
(HIP_VISIBLE_DEVICES, LOCAL_RANK, 127.0.0.1 rendezvous) instead of NVIDIA/k8s DNS."""
import json

import pytest

from polyaxon_amd.polyflow.env import cluster_def, framework_env, trial_env

XP = {"id": 12, "uuid": "abc123"}


def _env(**kw):
    args = dict(base_env={"PATH": "/usr/bin", "POLYAXON_STALE": "x", "RANK": "9", "DMLC_ROLE": "old",
                          "ROCR_VISIBLE_DEVICES": "3", "TF_CONFIG": "{}"},
                experiment=XP, project="mnist", user="root", group=None, role="master", index=0,
                framework=None, cluster={"master": ["127.0.0.1:4000"]}, devices=[0], outputs_path="/o",
                logs_path="/l", declarations={"lr": 0.1}, data_paths={"data": "/d"}, refs_outputs={},
                log_level=None, store_path=None, api_host=None, ephemeral_token=None, master_port=4000,
                local_rank=0)
    args.update(kw)
    return trial_env(**args)


def test_cluster_def_ports_and_roles():
    c = cluster_def("tensorflow", {"master": 1, "worker": 2, "ps": 1}, 5000)
    assert c == {"master": ["127.0.0.1:5000"], "worker": ["127.0.0.1:5001", "127.0.0.1:5002"],
                 "ps": ["127.0.0.1:5003"]}
    assert cluster_def(None, {"master": 1}, 7) == {"master": ["127.0.0.1:7"]}
    assert cluster_def("pytorch", {"master": 1, "worker": 0}, 10) == {"master": ["127.0.0.1:10"]}


@pytest.mark.parametrize("role,index,rank", [("master", 0, 0), ("worker", 0, 1), ("worker", 2, 3)])
def test_pytorch_rendezvous(role, index, rank):
    c = cluster_def("pytorch", {"master": 1, "worker": 3}, 6000)
    e = framework_env("pytorch", role, index, c, "/o", 6000)
    assert e == {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "6000", "WORLD_SIZE": "4", "RANK": str(rank)}


def test_horovod_gets_rank_and_size():
    c = cluster_def("horovod", {"master": 1, "worker": 1}, 6000)
    e = framework_env("horovod", "worker", 0, c, "/o", 6000)
    assert e["HOROVOD_RANK"] == "1" and e["HOROVOD_SIZE"] == "2" and e["RANK"] == "1"


@pytest.mark.parametrize("role,index", [("master", 0), ("worker", 1), ("ps", 0)])
def test_tensorflow_tf_config(role, index):
    c = cluster_def("tensorflow", {"master": 1, "worker": 2, "ps": 1}, 7000)
    tf = json.loads(framework_env("tensorflow", role, index, c, "/outputs/x", 7000)["TF_CONFIG"])
    assert tf["cluster"] == c
    assert tf["task"] == {"type": role, "index": index}
    assert tf["model_dir"] == "/outputs/x" and tf["environment"] == "cloud"


def test_tensorflow_without_ps_or_workers():
    c = cluster_def("tensorflow", {"master": 1}, 7000)
    tf = json.loads(framework_env("tensorflow", "master", 0, c, "/o", 7000)["TF_CONFIG"])
    assert tf["cluster"] == {"master": ["127.0.0.1:7000"]}


@pytest.mark.parametrize("role,index,dmlc_role,extra", [
    ("master", 0, "scheduler", {}),
    ("worker", 1, "worker", {"DMLC_WORKER_ID": "1"}),
    ("ps", 0, "server", {"DMLC_SERVER_ID": "0"}),
])
def test_mxnet_dmlc(role, index, dmlc_role, extra):
    c = cluster_def("mxnet", {"master": 1, "worker": 2, "ps": 1}, 8000)
    e = framework_env("mxnet", role, index, c, "/o", 8000)
    assert e["DMLC_ROLE"] == dmlc_role
    assert e["DMLC_NUM_WORKER"] == "2" and e["DMLC_NUM_SERVER"] == "1"
    assert e["DMLC_PS_ROOT_URI"] == "127.0.0.1" and e["DMLC_PS_ROOT_PORT"] == "8000"
    for k, v in extra.items():
        assert e[k] == v
    assert ("DMLC_WORKER_ID" in e) == (role == "worker") and ("DMLC_SERVER_ID" in e) == (role == "ps")


def test_unknown_framework_injects_nothing():
    assert framework_env(None, "master", 0, {"master": ["127.0.0.1:1"]}, "/o", 1) == {}


def test_trial_env_contract():
    e = _env()
    # stale platform / rendezvous variables from the parent never leak into a trial
    assert "POLYAXON_STALE" not in e and "DMLC_ROLE" not in e and "TF_CONFIG" not in e and "RANK" not in e
    assert "ROCR_VISIBLE_DEVICES" not in e and e["PATH"] == "/usr/bin"
    assert json.loads(e["POLYAXON_CLUSTER"]) == {"master": ["127.0.0.1:4000"]}
    assert json.loads(e["POLYAXON_TASK_INFO"]) == {"type": "master", "index": 0}
    assert json.loads(e["POLYAXON_DECLARATIONS"]) == {"lr": 0.1}
    info = json.loads(e["POLYAXON_EXPERIMENT_INFO"])
    assert info["experiment_name"] == "root.mnist.12" and info["project_name"] == "root.mnist"
    assert info["experiment_uuid"] == "abc123" and info["group_name"] is None
    assert e["POLYAXON_RUN_OUTPUTS_PATH"] == "/o" and e["POLYAXON_LOGS_PATH"] == "/l"
    assert json.loads(e["POLYAXON_RUN_DATA_PATHS"]) == {"data": "/d"}
    assert e["POLYAXON_LOG_LEVEL"] == "INFO" and e["POLYAXON_IN_CLUSTER"] == "true"
    assert e["POLYAXON_API_VERSION"] == "v1" and e["POLYAXON_EXPERIMENT_ID"] == "12"
    assert e["HIP_VISIBLE_DEVICES"] == "0" and e["LOCAL_RANK"] == "0"
    assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert "TORCH_NCCL_ASYNC_ERROR_HANDLING" not in e and "PLX_CPU_ONLY" not in e
    assert "POLYAXON_API_HTTP_HOST" not in e and "POLYAXON_SECRET_EPHEMERAL_TOKEN" not in e


def test_trial_env_group_api_token_and_cpu_only():
    e = _env(group={"id": 3, "uuid": "g"}, api_host="http://127.0.0.1:8000", ephemeral_token="tok",
             devices=[], log_level="DEBUG", store_path="/s.sqlite")
    info = json.loads(e["POLYAXON_EXPERIMENT_INFO"])
    assert info["group_name"] == "root.mnist.3" and info["group_uuid"] == "g"
    assert e["POLYAXON_API_HTTP_HOST"] == "http://127.0.0.1:8000"
    assert e["POLYAXON_API_WS_HOST"] == "ws://127.0.0.1:8000"
    assert e["POLYAXON_SECRET_EPHEMERAL_TOKEN"] == "tok" and e["POLYAXON_STORE_PATH"] == "/s.sqlite"
    assert e["HIP_VISIBLE_DEVICES"] == "" and e["PLX_CPU_ONLY"] == "1"
    assert e["POLYAXON_LOG_LEVEL"] == "DEBUG"


def test_multi_rank_trials_get_the_rccl_watchdog():
    c = cluster_def("pytorch", {"master": 1, "worker": 1}, 6000)
    e = _env(framework="pytorch", cluster=c, role="worker", index=0, devices=[5], local_rank=0)
    assert e["RANK"] == "1" and e["WORLD_SIZE"] == "2" and e["HIP_VISIBLE_DEVICES"] == "5"
    assert e["TORCH_NCCL_ASYNC_ERROR_HANDLING"] == "1" and e["PLX_COLLECTIVE_TIMEOUT_S"] == "600"
    e = _env(framework="pytorch", cluster=c, base_env={"PLX_COLLECTIVE_TIMEOUT_S": "30"})
    assert e["PLX_COLLECTIVE_TIMEOUT_S"] == "30"  # operator override wins


def test_rccl_channel_count_is_opt_in_and_multi_rank_only(monkeypatch):
    """PLX_RCCL_MIN_CHANNELS (operator side) becomes NCCL_MIN_NCHANNELS for multi-rank trials only; a value the
    trial's own env already carries is kept."""
    c = cluster_def("pytorch", {"master": 1, "worker": 1}, 6000)
    assert "NCCL_MIN_NCHANNELS" not in _env(framework="pytorch", cluster=c)
    monkeypatch.setenv("PLX_RCCL_MIN_CHANNELS", "32")
    assert _env(framework="pytorch", cluster=c)["NCCL_MIN_NCHANNELS"] == "32"
    assert "NCCL_MIN_NCHANNELS" not in _env()  # single rank: no collectives
    e = _env(framework="pytorch", cluster=c, base_env={"NCCL_MIN_NCHANNELS": "8"})
    assert e["NCCL_MIN_NCHANNELS"] == "8"
    monkeypatch.setenv("PLX_RCCL_MIN_CHANNELS", "lots")
    assert "NCCL_MIN_NCHANNELS" not in _env(framework="pytorch", cluster=c)


def test_trial_env_carries_the_hbm_budget():
    """resources.hbm (GB) and fractional gpu shares reach the trial as PLX_HBM_GB / PLX_HBM_FRACTION, which
    client/budget.py turns into a caching-allocator cap (set_per_process_memory_fraction)."""
    from polyaxon_amd.client.budget import budget_fraction

    e = _env(hbm_gb=72.0, gpu_share=0.25, base_env={"PLX_HBM_FRACTION": "0.9"})
    assert e["PLX_HBM_GB"] == "72" and "PLX_HBM_FRACTION" not in e
    e = _env(gpu_share=0.25)
    assert e["PLX_HBM_FRACTION"] == "0.25" and "PLX_HBM_GB" not in e
    e = _env()
    assert "PLX_HBM_GB" not in e and "PLX_HBM_FRACTION" not in e
    e = _env(devices=[], hbm_gb=10.0)  # CPU replica: nothing to cap
    assert "PLX_HBM_GB" not in e
    total = 288 * 2 ** 30
    assert budget_fraction(total, {"PLX_HBM_GB": "72"}) == pytest.approx(0.25)
    assert budget_fraction(total, {"PLX_HBM_FRACTION": "0.5"}) == 0.5
    assert budget_fraction(total, {"PLX_HBM_GB": "1000"}) == 1.0
    assert budget_fraction(total, {}) is None


def test_scheduler_exports_the_budget_to_packed_trials(tmp_path):
    """Two gpu: 0.5 trials with hbm: 100 share one device; each sees its own budget in its environment."""
    from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
    from polyaxon_amd.polyflow.scheduler import Polyflow

    with Polyflow(str(tmp_path), allocator=DeviceAllocator([Device(0)]), reconcile_s=0) as flow:
        ids = [flow.submit({"version": 1, "kind": "experiment",
                            "run": {"cmd": "echo BUDGET=$PLX_HBM_GB/$PLX_HBM_FRACTION/$HIP_VISIBLE_DEVICES"},
                            "environment": {"resources": {"gpu": 0.5, "hbm": 100}}})["id"] for _ in range(2)]
        for i in ids:
            assert flow.wait("experiment", i, timeout=30) == "succeeded"
        for i in ids:
            x = flow.store.get_experiment(i)
            logs = open(flow.paths.replica_log(x["logs_path"], "master", 0)).read()
            assert "BUDGET=100//0" in logs
