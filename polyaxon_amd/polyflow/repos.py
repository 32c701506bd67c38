"""Code references and project repos (reference polyaxon/libs/repos/git.py:18-132,
libs/repos/utils.py:22-27, api/repos/tasks.py:20-73, libs/archive.py:10-58).

* ``code_reference(path)`` captures the commit SHA, branch, remote URL and whether the tree is dirty
  (with the diff, truncated) of the directory a run is submitted from — stored as a CodeReference row and
  linked to every experiment of the submission (the reference's ``assign_code_reference``);
* ``ProjectRepo`` is the ``polyaxon upload`` equivalent: a tarball of the user's code is extracted into
  ``<root>/repos/<user>/<project>`` and committed into a local git repository so each upload gets a SHA;
  runs submitted with ``cwd=repo.path`` execute that snapshot;
* ``ExternalRepo`` is the reference's external git repository (``build: {git: <url>, ref: <commit|branch|tag>}``;
  ExternalRepo model db/models/repos.py, libs/repos/git.py:54-115 ``clone_git_repo`` / ``fetch`` /
  ``checkout_commit``): cloned once under ``<root>/repos/<user>/<project>/external/<name>``, fetched and hard-reset
  on later submissions, checked out at ``ref`` -- the run executes in that checkout and its code reference is the
  checked-out commit.
"""
from __future__ import annotations

import io
import os
import re
import shutil
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


class GitError(RuntimeError):
    pass


def _git_checked(args, cwd: str, timeout: float = 300.0) -> str:
    try:
        out = subprocess.run(["git", *args], cwd=cwd, capture_output=True, text=True, timeout=timeout,
                             env=dict(os.environ, GIT_TERMINAL_PROMPT="0"))
    except (OSError, subprocess.SubprocessError) as e:
        raise GitError(f"git {' '.join(args)}: {e}") from None
    if out.returncode != 0:
        raise GitError(f"git {' '.join(args)} failed: {out.stderr.strip()[-2000:]}")
    return out.stdout.strip()


def repo_name(git_url: str) -> str:
    name = re.sub(r"\.git$", "", git_url.rstrip("/").rsplit("/", 1)[-1].rsplit(":", 1)[-1]) or "repo"
    return re.sub(r"[^A-Za-z0-9_.-]", "_", name)


class ExternalRepo:
    def __init__(self, repos_root: str, user: str, project: str, git_url: str):
        self.git_url = git_url
        self.name = repo_name(git_url)
        self.path = os.path.join(repos_root, user, project, "external", self.name)

    @property
    def cloned(self) -> bool:
        return os.path.isdir(os.path.join(self.path, ".git"))

    def fetch(self, overwrite: bool = False) -> str:
        """Clone on first use; afterwards fetch every branch and tag and clean the tree (reference ``fetch``).
        Returns the HEAD commit."""
        if self.cloned and overwrite:
            shutil.rmtree(self.path)
        if not self.cloned:
            os.makedirs(os.path.dirname(self.path), exist_ok=True)
            if os.path.exists(self.path):
                shutil.rmtree(self.path)
            _git_checked(["clone", "-q", self.git_url, self.path], cwd=os.path.dirname(self.path))
        else:
            if _git_checked(["config", "--get", "remote.origin.url"], self.path) != self.git_url:
                _git_checked(["remote", "set-url", "origin", self.git_url], self.path)
            _git_checked(["fetch", "-q", "--tags", "--prune", "origin", "+refs/heads/*:refs/remotes/origin/*"],
                         self.path)
            _git_checked(["reset", "-q", "--hard"], self.path)
            _git_checked(["clean", "-q", "-fdx"], self.path)
        return self.head()

    def checkout(self, ref: Optional[str] = None) -> str:
        """Check out ``ref`` (commit SHA, tag, or branch -- a branch resolves to the freshly fetched remote branch);
        None = the remote's default branch.  Returns the checked-out commit."""
        if ref is None:
            target = _git_checked(["rev-parse", "--abbrev-ref", "origin/HEAD"], self.path) if \
                _git(["rev-parse", "--verify", "-q", "origin/HEAD"], self.path) else "HEAD"
        elif _git(["rev-parse", "--verify", "-q", f"origin/{ref}"], self.path):
            target = f"origin/{ref}"
        else:
            target = ref
        _git_checked(["checkout", "-q", "--detach", target], self.path)
        return self.head()

    def head(self) -> str:
        return _git_checked(["rev-parse", "HEAD"], self.path)
