"""Outputs / logs / data path layout (reference polyaxon/libs/paths/*.py).

Layout (identical to the reference so user code that reads POLYAXON_RUN_OUTPUTS_PATH keeps working):
    <outputs_root>/<user>/<project>/experiments/<id>               independent experiment
    <outputs_root>/<user>/<project>/groups/<group_id>/<id>         experiment of a group
    <outputs_root>/<user>/<project>/jobs/<id>                      generic job
    <logs_root>/<user>/<project>/experiments/<id>[/<role>.<index>.log]
RESUME reuses the ORIGINAL experiment's outputs path (libs/paths/experiments.py:11-23); COPY copies the
original's outputs into the new path; RESTART starts with a clean directory.
"""
from __future__ import annotations

import os
import shutil
from typing import Optional


class Paths:
    def __init__(self, root: str):
        self.root = os.path.abspath(root)
        self.outputs_root = os.path.join(self.root, "outputs")
        self.logs_root = os.path.join(self.root, "logs")
        self.data_root = os.path.join(self.root, "data")
        self.repos_root = os.path.join(self.root, "repos")
        self.envs_root = os.path.join(self.root, "envs")
        for p in (self.outputs_root, self.logs_root, self.data_root, self.repos_root, self.envs_root):
            os.makedirs(p, exist_ok=True)

    def experiment_outputs(self, user: str, project: str, xid: int, group_id: Optional[int] = None) -> str:
        if group_id:
            return os.path.join(self.outputs_root, user, project, "groups", str(group_id), str(xid))
        return os.path.join(self.outputs_root, user, project, "experiments", str(xid))

    def experiment_logs(self, user: str, project: str, xid: int, group_id: Optional[int] = None) -> str:
        if group_id:
            return os.path.join(self.logs_root, user, project, "groups", str(group_id), str(xid))
        return os.path.join(self.logs_root, user, project, "experiments", str(xid))

    def replica_log(self, logs_dir: str, role: str, index: int) -> str:
        return os.path.join(logs_dir, f"{role}.{index}.log")

    def job_outputs(self, user: str, project: str, jid: int, kind: str = "jobs") -> str:
        return os.path.join(self.outputs_root, user, project, kind, str(jid))

    def job_logs(self, user: str, project: str, jid: int, kind: str = "jobs") -> str:
        return os.path.join(self.logs_root, user, project, kind, str(jid))

    def group_outputs(self, user: str, project: str, gid: int) -> str:
        return os.path.join(self.outputs_root, user, project, "groups", str(gid))

    @staticmethod
    def prepare_outputs(path: str, strategy: Optional[str] = None, original: Optional[str] = None) -> None:
        """Init-container equivalent (reference templates/init_containers.py:19-33)."""
        if strategy == "copy" and original and os.path.isdir(original):
            if os.path.exists(path):
                shutil.rmtree(path)
            shutil.copytree(original, path)
            return
        if strategy in (None, "restart") and os.path.isdir(path) and strategy == "restart":
            shutil.rmtree(path)
        os.makedirs(path, exist_ok=True)

    @staticmethod
    def read_log(path: str, tail: Optional[int] = None) -> str:
        if not os.path.exists(path):
            return ""
        with open(path, "r", errors="replace") as f:
            data = f.read()
        if tail:
            return "\n".join(data.splitlines()[-tail:])
        return data
