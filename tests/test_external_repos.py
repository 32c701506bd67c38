"""External git repositories (reference ExternalRepo, libs/repos/git.py:54-115): ``build: {git, ref}`` clones the
repository once, fetches it on later submissions, checks out the ref, runs there and records the commit."""
import os
import subprocess

import pytest

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.repos import ExternalRepo, GitError, repo_name
from polyaxon_amd.polyflow.scheduler import Polyflow
from polyaxon_amd.spec.specification import PolyaxonfileError


def _git(cwd, *args):
    return subprocess.run(["git", *args], cwd=cwd, check=True, capture_output=True, text=True).stdout.strip()


@pytest.fixture
def remote(tmp_path):
    src = tmp_path / "upstream"
    src.mkdir()
    _git(src, "init", "-q", "-b", "main")
    _git(src, "config", "user.email", "t@t")
    _git(src, "config", "user.name", "t")
    (src / "train.txt").write_text("v1\n")
    _git(src, "add", "-A")
    _git(src, "commit", "-q", "-m", "one")
    c1 = _git(src, "rev-parse", "HEAD")
    _git(src, "tag", "release-1")
    (src / "train.txt").write_text("v2\n")
    _git(src, "commit", "-q", "-am", "two")
    c2 = _git(src, "rev-parse", "HEAD")
    return src, c1, c2


def test_repo_name():
    assert repo_name("https://github.com/org/model-zoo.git") == "model-zoo"
    assert repo_name("git@github.com:org/zoo") == "zoo"
    assert repo_name("/srv/git/x.git/") == "x"


def test_external_repo_clone_fetch_checkout(tmp_path, remote):
    src, c1, c2 = remote
    r = ExternalRepo(str(tmp_path / "repos"), "u", "p", str(src))
    assert r.fetch() == c2 and r.cloned
    assert r.checkout(c1) == c1 and (r.path and open(os.path.join(r.path, "train.txt")).read() == "v1\n")
    assert r.checkout("release-1") == c1
    assert r.checkout("main") == c2
    # a new upstream commit arrives; fetch + checkout the branch picks it up (no re-clone)
    (src / "train.txt").write_text("v3\n")
    _git(src, "commit", "-q", "-am", "three")
    c3 = _git(src, "rev-parse", "HEAD")
    r.fetch()
    assert r.checkout("main") == c3
    with pytest.raises(GitError):
        r.checkout("no-such-ref")
    with pytest.raises(GitError):
        ExternalRepo(str(tmp_path / "repos"), "u", "p", str(tmp_path / "missing")).fetch()


def test_experiment_runs_in_external_checkout(tmp_path, remote):
    src, c1, c2 = remote
    flow = Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0)]), reconcile_s=0).start()
    try:
        spec = {"version": 1, "kind": "experiment", "build": {"git": str(src), "ref": c1},
                "run": {"cmd": "cat train.txt"}}
        r = flow.submit(spec, project="zoo")
        assert flow.wait("experiment", r["id"], timeout=30) == "succeeded"
        assert "v1" in flow.logs("experiment", r["id"])
        x = flow.store.get_experiment(r["id"])
        ref = flow.store.get("code_references", x["code_reference_id"])
        assert ref["commit_sha"] == c1
        spec["build"]["ref"] = "main"
        r2 = flow.submit(spec, project="zoo")
        assert flow.wait("experiment", r2["id"], timeout=30) == "succeeded"
        assert "v2" in flow.logs("experiment", r2["id"])
        repos = flow.store.external_repos()
        assert len(repos) == 1 and repos[0]["last_commit"] == c2 and repos[0]["git_url"] == str(src)
        bad = dict(spec, build={"git": str(tmp_path / "nowhere")})
        with pytest.raises(PolyaxonfileError):
            flow.submit(bad, project="zoo")
    finally:
        flow.shutdown()
