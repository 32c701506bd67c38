"""Code references and project repos (reference polyaxon/libs/repos/git.py:18-132,
libs/repos/utils.py:22-27, api/repos/tasks.py:20-73, libs/archive.py:10-58).

* ``code_reference(path)`` captures the commit SHA, branch, remote URL and whether the tree is dirty
  (with the diff, truncated) of the directory a run is submitted from — stored as a CodeReference row and
  linked to every experiment of the submission (the reference's ``assign_code_reference``);
* ``ProjectRepo`` is the ``polyaxon upload`` equivalent: a tarball of the user's code is extracted into
  ``<root>/repos/<user>/<project>`` and committed into a local git repository so each upload gets a SHA;
  runs submitted with ``cwd=repo.path`` execute that snapshot.
"""
from __future__ import annotations

import io
import os
import subprocess
import tarfile
from typing import Dict, Optional

MAX_DIFF = 256 * 1024


def _git(args, cwd: str, timeout: float = 10.0) -> Optional[str]:
    try:
        out = subprocess.run(["git", *args], cwd=cwd, capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.SubprocessError):
        return None
    return out.stdout.strip() if out.returncode == 0 else None


def code_reference(path: str) -> Optional[Dict[str, object]]:
    if not path or not os.path.isdir(path):
        return None
    sha = _git(["rev-parse", "HEAD"], path)
    if not sha:
        return None
    status = _git(["status", "--porcelain", "--untracked-files=no"], path) or ""
    diff = _git(["diff", "HEAD"], path) if status else None
    return {"commit": sha, "branch": _git(["rev-parse", "--abbrev-ref", "HEAD"], path),
            "git_url": _git(["config", "--get", "remote.origin.url"], path), "is_dirty": bool(status),
            "diff": diff[:MAX_DIFF] if diff else None}


class ProjectRepo:
    def __init__(self, repos_root: str, user: str, project: str):
        self.path = os.path.join(repos_root, user, project)

    def upload_tarball(self, data: bytes, message: str = "upload") -> str:
        """Replace the repo's working tree with the tarball's content and commit it; returns the SHA."""
        os.makedirs(self.path, exist_ok=True)
        if not os.path.isdir(os.path.join(self.path, ".git")):
            _git(["init", "-q"], self.path)
            _git(["config", "user.email", "plx@localhost"], self.path)
            _git(["config", "user.name", "plx"], self.path)
        for name in os.listdir(self.path):
            if name == ".git":
                continue
            full = os.path.join(self.path, name)
            if os.path.isdir(full) and not os.path.islink(full):
                import shutil

                shutil.rmtree(full)
            else:
                os.remove(full)
        with tarfile.open(fileobj=io.BytesIO(data), mode="r:*") as tar:
            safe = []
            for m in tar.getmembers():
                target = os.path.realpath(os.path.join(self.path, m.name))
                if not target.startswith(os.path.realpath(self.path) + os.sep) or m.issym() or m.islnk() or m.isdev():
                    continue  # path traversal / links / devices are dropped
                safe.append(m)
            tar.extractall(self.path, members=safe)
        _git(["add", "-A"], self.path)
        _git(["commit", "-q", "--allow-empty", "-m", message], self.path)
        return _git(["rev-parse", "HEAD"], self.path) or ""

    def archive(self) -> bytes:
        """Tarball of the current tree (reference repo download)."""
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w:gz") as tar:
            for name in sorted(os.listdir(self.path)):
                if name != ".git":
                    tar.add(os.path.join(self.path, name), arcname=name)
        return buf.getvalue()

    @property
    def last_commit(self) -> Optional[str]:
        return _git(["rev-parse", "HEAD"], self.path) if os.path.isdir(self.path) else None
