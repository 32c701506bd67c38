"""Cleaning hooks: orphaned runs are stopped at scheduler start (their processes killed only when they
are provably theirs), unmanaged runs are left alone, old outputs expire."""
import os
import subprocess
import sys
import time

from polyaxon_amd.polyflow.cleaning import MESSAGE, clean_outputs, clean_stale, scheduler_alive
from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow
from polyaxon_amd.store import Store


def _sleeper(env_extra):
    env = dict(os.environ, **env_extra)
    return subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"], env=env,
                            start_new_session=True)


def test_orphans_stopped_on_start(tmp_path):
    root = tmp_path / "plx"
    root.mkdir()
    store = Store(str(root / "polyaxon.sqlite"))
    pid = store.create_project("p")["id"]
    outs = str(tmp_path / "outs" / "1")
    os.makedirs(outs)
    x = store.create_experiment(pid, {"run": {"cmd": "x"}})
    xid = x["id"] if isinstance(x, dict) else x
    store.update_experiment(xid, outputs_path=outs)
    for s in ("scheduled", "starting", "running"):
        store.set_experiment_status(xid, s)
    mine = _sleeper({"POLYAXON_RUN_OUTPUTS_PATH": outs})
    decoy = _sleeper({"POLYAXON_RUN_OUTPUTS_PATH": outs + "-other"})
    jid = store.create_experiment_job(xid, "master", 0)
    jid = jid["id"] if isinstance(jid, dict) else jid
    store.update_experiment_job(jid, pid=mine.pid)
    # an experiment tracked from outside the scheduler (client-created) is not the scheduler's to stop
    u = store.create_experiment(pid, {})
    uid = u["id"] if isinstance(u, dict) else u
    store.update_experiment(uid, is_managed=0)
    store.set_experiment_status(uid, "running", force=True)
    try:
        flow = Polyflow(str(root), store=store, allocator=DeviceAllocator([Device(0)])).start()
        try:
            assert scheduler_alive(str(root))
            assert store.get_experiment(xid)["status"] == "stopped"
            assert store.experiment_statuses(xid)[-1]["message"] == MESSAGE
            assert mine.wait(timeout=10) != 0
            assert decoy.poll() is None
            assert store.get_experiment(uid)["status"] == "running"
        finally:
            flow.shutdown()
        assert not scheduler_alive(str(root))
    finally:
        for p in (mine, decoy):
            if p.poll() is None:
                p.kill()
                p.wait()


def test_clean_stale_respects_live_and_kinds(tmp_path):
    store = Store(str(tmp_path / "s.sqlite"))
    pid = store.create_project("p")["id"]
    g = store.create_group(pid, {}, {})
    gid = g["id"] if isinstance(g, dict) else g
    store.set_group_status(gid, "running")
    j = store.create_job("job", pid, {})
    jid = j["id"] if isinstance(j, dict) else j
    store.set_job_status(jid, "scheduled")
    out = clean_stale(store, live=[("group", gid)], kinds=("groups", "jobs"))
    assert out["groups"] == [] and out["jobs"] == [jid]
    assert store.get_group(gid)["status"] == "running"
    assert store.get_job(jid)["status"] == "stopped"


def test_clean_outputs(tmp_path):
    store = Store(str(tmp_path / "s.sqlite"))
    pid = store.create_project("p")["id"]
    old_dir, new_dir = tmp_path / "old", tmp_path / "new"
    old_dir.mkdir()
    new_dir.mkdir()
    ids = []
    for d in (old_dir, new_dir):
        x = store.create_experiment(pid, {})
        xid = x["id"] if isinstance(x, dict) else x
        store.update_experiment(xid, outputs_path=str(d))
        store.set_experiment_status(xid, "failed", force=True)
        ids.append(xid)
    store.update_experiment(ids[0], finished_at=time.time() - 3 * 86400)
    assert clean_outputs(store, 86400, dry_run=True) == [str(old_dir)] and old_dir.exists()
    assert clean_outputs(store, 86400) == [str(old_dir)]
    assert not old_dir.exists() and new_dir.exists()
    assert store.get_experiment(ids[0])["outputs_path"] is None


def test_clean_outputs_keeps_paths_shared_with_live_resume_clones(tmp_path):
    """A Hyperband root finished long ago shares its outputs with a RESUME clone that is still running (or
    finished recently): the checkpoints must survive until every row using them is past the window."""
    store = Store(str(tmp_path / "s.sqlite"))
    pid = store.create_project("p")["id"]
    shared = tmp_path / "root_outputs"
    shared.mkdir()
    (shared / "model.pt").write_text("ckpt")
    root = store.create_experiment(pid, {})
    store.update_experiment(root, outputs_path=str(shared), logs_path=str(tmp_path / "logs_root"))
    store.set_experiment_status(root, "succeeded", force=True)
    store.update_experiment(root, finished_at=time.time() - 3 * 86400)
    clone = store.create_experiment(pid, {}, original_experiment_id=root, cloning_strategy="resume")
    store.update_experiment(clone, outputs_path=str(shared))
    store.set_experiment_status(clone, "running", force=True)  # still training from the root's checkpoint
    assert clean_outputs(store, 86400) == []
    assert (shared / "model.pt").exists() and store.get_experiment(root)["outputs_path"] == str(shared)
    store.set_experiment_status(clone, "succeeded")  # finished just now: still inside the window
    assert clean_outputs(store, 86400) == [] and shared.exists()
    store.update_experiment(clone, finished_at=time.time() - 2 * 86400)  # both past the window: now it goes
    assert clean_outputs(store, 86400) == [str(shared)]
    assert not shared.exists()
    assert store.get_experiment(root)["outputs_path"] is None and store.get_experiment(clone)["outputs_path"] is None


def test_deploy_generate_and_check(tmp_path, monkeypatch, capsys):
    import json as _json

    from polyaxon_amd.cli.main import main
    from polyaxon_amd.conf import Settings
    from polyaxon_amd.deploy import DeployConfig, preflight

    monkeypatch.setenv("PLX_CONFIG", str(tmp_path / "c.yaml"))
    out_dir = tmp_path / "dep"
    assert main(["deploy", "generate", "--root", str(tmp_path / "root"), "--port", "8123", "--gpus", "8",
                 "--out", str(out_dir)]) == 0
    res = _json.loads(capsys.readouterr().out)
    assert res["files"] == ["deploy.json", "plx.env", "polyaxon-mi355x.service", "settings.yaml"]
    st = Settings.load(env={}, files=[str(out_dir / "settings.yaml")])
    assert st["api.port"] == 8123 and st["scheduler.gpus"] == 8 and st["root"] == str(tmp_path / "root")
    tok = st["api.admin_token"]
    assert f"PLX_TOKEN={tok}" in (out_dir / "plx.env").read_text()
    assert oct((out_dir / "plx.env").stat().st_mode & 0o777) == "0o600"
    unit = (out_dir / "polyaxon-mi355x.service").read_text()
    assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in unit and "--port 8123" in unit
    names = {c.name for c in preflight(DeployConfig(root=str(tmp_path), port=0, host="127.0.0.1"))}
    assert {"dev_kfd", "gfx950_agents", "rccl", "port", "disk", "root_writable"} <= names
