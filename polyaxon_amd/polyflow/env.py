"""In-trial environment contract.

Reproduces what the reference injects into every pod (scheduler/spawners/templates/constants.py:6-24,
env_vars.py:97-179, experiment_jobs/pods.py:151-159,243-249, and the framework spawners) so user code
written against ``polyaxon-helper`` / the tracking client keeps working — with the MI355X-native device
wiring instead of NVIDIA's: ``HIP_VISIBLE_DEVICES`` holds the allocated
devices (empty for CPU-only replicas instead of ``NVIDIA_VISIBLE_DEVICES=none``), PyTorch rendezvous is
``MASTER_ADDR=127.0.0.1`` on a free local port, and ``LOCAL_RANK`` is set for one-process-per-GPU RCCL.
"""
from __future__ import annotations

import json
import os
import socket
from typing import Any, Dict, List, Optional

API_VERSION = "v1"


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def hw_queue_env(env: Dict[str, str]) -> Dict[str, str]:
    """PLX_HW_QUEUES=n (opt-in): raise GPU_MAX_HW_QUEUES to n (at most 32) in the environment of a process polyflow
    launches; never lowered, and nothing changes without it (the framework's streams fit the box's default 4 queues:
    profiles/r5_hw_queues.md).  Returns ``env``."""
    try:
        want = int(env.get("PLX_HW_QUEUES", "0") or 0)
        have = int(env.get("GPU_MAX_HW_QUEUES", "0") or 0)
    except ValueError:
        return env
    if want > have:
        env["GPU_MAX_HW_QUEUES"] = str(min(want, 32))
    return env


def cluster_def(framework: Optional[str], cluster: Dict[str, int], base_port: int) -> Dict[str, List[str]]:
    """POLYAXON_CLUSTER: {role: [host:port, ...]} for every replica (all on 127.0.0.1, distinct ports)."""
    out: Dict[str, List[str]] = {}
    port = base_port
    for role in ("master", "worker", "ps"):
        n = cluster.get(role, 0)
        if n:
            out[role] = []
            for _ in range(n):
                out[role].append(f"127.0.0.1:{port}")
                port += 1
    return out


def framework_env(framework: Optional[str], role: str, index: int, cluster: Dict[str, List[str]],
                  outputs_path: str, master_port: int) -> Dict[str, str]:
    n_workers = len(cluster.get("worker", []))
    n_ps = len(cluster.get("ps", []))
    if framework == "pytorch":
        rank = 0 if role == "master" else index + 1
        return {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(master_port), "WORLD_SIZE": str(n_workers + 1),
                "RANK": str(rank)}
    if framework == "horovod":  # reference injects nothing; give MPI-free launchers the same rendezvous
        rank = 0 if role == "master" else index + 1
        return {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(master_port), "WORLD_SIZE": str(n_workers + 1),
                "RANK": str(rank), "HOROVOD_RANK": str(rank), "HOROVOD_SIZE": str(n_workers + 1)}
    if framework == "tensorflow":
        tf_cluster = {"master": cluster.get("master", [])}
        if n_workers:
            tf_cluster["worker"] = cluster["worker"]
        if n_ps:
            tf_cluster["ps"] = cluster["ps"]
        return {"TF_CONFIG": json.dumps({"cluster": tf_cluster, "task": {"type": role, "index": index},
                                         "model_dir": outputs_path, "environment": "cloud"})}
    if framework == "mxnet":
        dmlc_role = {"master": "scheduler", "worker": "worker", "ps": "server"}[role]
        env = {"DMLC_NUM_WORKER": str(n_workers), "DMLC_NUM_SERVER": str(n_ps),
               "DMLC_PS_ROOT_URI": "127.0.0.1", "DMLC_PS_ROOT_PORT": str(master_port), "DMLC_ROLE": dmlc_role}
        if role == "worker":
            env["DMLC_WORKER_ID"] = str(index)
        if role == "ps":
            env["DMLC_SERVER_ID"] = str(index)
        return env
    return {}


def trial_env(*, base_env: Optional[Dict[str, str]] = None, experiment: Dict[str, Any], project: str, user: str,
              group: Optional[Dict[str, Any]], role: str, index: int, framework: Optional[str],
              cluster: Dict[str, List[str]], devices: List[int], outputs_path: str, logs_path: str,
              declarations: Dict[str, Any], data_paths: Dict[str, str], refs_outputs: Dict[str, List[str]],
              log_level: Optional[str], store_path: Optional[str], api_host: Optional[str],
              ephemeral_token: Optional[str], master_port: int, local_rank: int, hbm_gb: float = 0.0,
              gpu_share: float = 1.0) -> Dict[str, str]:
    env = dict(base_env if base_env is not None else os.environ)
    for k in list(env):
        if k.startswith("POLYAXON_") or k in ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK",
                                              "TF_CONFIG") or k.startswith("DMLC_"):
            env.pop(k)
    info = {"project_name": f"{user}.{project}", "experiment_name": f"{user}.{project}.{experiment['id']}",
            "experiment_uuid": experiment["uuid"], "experiment_id": experiment["id"],
            "group_name": f"{user}.{project}.{group['id']}" if group else None,
            "group_uuid": group["uuid"] if group else None}
    env.update({
        "POLYAXON_CLUSTER": json.dumps(cluster),
        "POLYAXON_TASK_INFO": json.dumps({"type": role, "index": index}),
        "POLYAXON_DECLARATIONS": json.dumps(declarations),
        "POLYAXON_EXPERIMENT_INFO": json.dumps(info),
        "POLYAXON_LOG_LEVEL": log_level or "INFO",
        "POLYAXON_RUN_OUTPUTS_PATH": outputs_path,
        "POLYAXON_LOGS_PATH": logs_path,
        "POLYAXON_RUN_DATA_PATHS": json.dumps(data_paths),
        "POLYAXON_REFS_OUTPUTS_PATHS": json.dumps(refs_outputs),
        "POLYAXON_IN_CLUSTER": "true",
        "POLYAXON_API_VERSION": API_VERSION,
        "POLYAXON_EXPERIMENT_ID": str(experiment["id"]),
        "POLYAXON_INTERNAL_HEADER": "X-POLYAXON-INTERNAL",
        "POLYAXON_INTERNAL_HEADER_SERVICE": "experiments",
    })
    if store_path:
        env["POLYAXON_STORE_PATH"] = store_path
    if api_host:
        env["POLYAXON_API_HTTP_HOST"] = api_host
        env["POLYAXON_API_WS_HOST"] = api_host.replace("http", "ws", 1)
    if ephemeral_token:
        env["POLYAXON_SECRET_EPHEMERAL_TOKEN"] = ephemeral_token
    env.update(framework_env(framework, role, index, cluster, outputs_path, master_port))
    # HIP_VISIBLE_DEVICES only: ROCR_VISIBLE_DEVICES would renumber first and the two would compose
    env.pop("ROCR_VISIBLE_DEVICES", None)
    env["HIP_VISIBLE_DEVICES"] = ",".join(str(d) for d in devices)
    env["LOCAL_RANK"] = str(local_rank)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    hw_queue_env(env)
    n_ranks = sum(len(v) for v in cluster.values()) if cluster else 1
    if n_ranks > 1:
        # Collective deadlines, one variable for both planes:
        # * the framework RCCL communicator's watchdog (csrc/rccl_comm.cpp) aborts it when a peer does not join within
        #   PLX_COLLECTIVE_TIMEOUT_S or a collective stays incomplete that long: the rank raises RcclError and exits;
        # * the gloo rendezvous group carries the same timeout (parallel/ddp.init_from_env);
        # * a user program's own ProcessGroupNCCL gets torch's async error handling.
        # The scheduler sees the failed rank and tears down the surviving ones.
        env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        env.setdefault("PLX_COLLECTIVE_TIMEOUT_S", "600")
        # RCCL channel count of the DP ranks' communicators (several channels spread a ring
        # collective over the node's 7 xGMI links per GPU).  PLX_RCCL_MIN_CHANNELS=n on the scheduler sets
        # NCCL_MIN_NCHANNELS=n for every multi-rank trial unless its own environment already does; unset: RCCL's
        # topology-based choice.  The bucket planner times the result at start-up (parallel/comm_plan.py calibrate).
        ch = os.environ.get("PLX_RCCL_MIN_CHANNELS", "")
        if ch.isdigit() and int(ch) > 0:
            env.setdefault("NCCL_MIN_NCHANNELS", ch)
    if not devices:
        env["PLX_CPU_ONLY"] = "1"
    # HBM budget of the replica (client/budget.py enforces it in the trial process): the reserved GB, else the
    # device share of a fractional request, so packed trials cannot exhaust each other's memory
    env.pop("PLX_HBM_GB", None)
    env.pop("PLX_HBM_FRACTION", None)
    if devices and hbm_gb > 0:
        env["PLX_HBM_GB"] = f"{hbm_gb:g}"
    elif devices and 0 < gpu_share < 1:
        env["PLX_HBM_FRACTION"] = f"{gpu_share:g}"
    return env
