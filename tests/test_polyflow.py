"""polyflow scheduler on CPU: trials are real subprocesses; devices are a fake pool (no GPU needed).

Covers the reference's lifecycle tests (tests/test_experiments/test_models.py,
tests/test_experiment_groups/test_models.py) with a real process backend instead of mocked spawners."""
import json
import os
import sys
import textwrap
import time

import pytest

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow

PY = sys.executable


def _flow(tmp_path, n_gpus=2, grace=2.0):
    alloc = DeviceAllocator([Device(i) for i in range(n_gpus)])
    return Polyflow(str(tmp_path / "plx"), allocator=alloc, stop_grace_s=grace).start()


def _xp(cmd, **env):
    d = {"version": 1, "kind": "experiment", "run": {"cmd": cmd}}
    if env:
        d["environment"] = env
    return d


def test_experiment_success_env_contract_and_logs(tmp_path):
    flow = _flow(tmp_path)
    try:
        script = ("import os,json; print('HIP', os.environ['HIP_VISIBLE_DEVICES']); "
                  "print('DECL', os.environ['POLYAXON_DECLARATIONS']); print('OUT', os.environ['POLYAXON_RUN_OUTPUTS_PATH']);"
                  "print('TASK', os.environ['POLYAXON_TASK_INFO'])")
        spec = _xp(f"{PY} -c \"{script}\"", resources={"gpu": {"limits": 1}})
        spec["declarations"] = {"lr": 0.5}
        r = flow.submit(spec, project="p")
        assert flow.wait("experiment", r["id"], timeout=30) == "succeeded"
        logs = flow.logs("experiment", r["id"])
        assert "master.0 -- HIP 0" in logs and '"lr": 0.5' in logs and '"type": "master"' in logs
        x = flow.store.get_experiment(r["id"])
        assert os.path.isdir(x["outputs_path"]) and "/root/p/experiments/" in x["outputs_path"]
        sts = [s["status"] for s in flow.store.experiment_statuses(r["id"])]
        assert sts == ["created", "scheduled", "starting", "running", "succeeded"]
        jobs = flow.store.experiment_jobs(r["id"])
        assert [j["status"] for j in jobs] == ["succeeded"] and jobs[0]["devices"] == [0]
    finally:
        flow.shutdown()


def test_failure_and_stop(tmp_path):
    flow = _flow(tmp_path)
    try:
        bad = flow.submit(_xp("exit 3"))
        assert flow.wait("experiment", bad["id"], timeout=30) == "failed"
        j = flow.store.experiment_jobs(bad["id"])[0]
        assert j["exit_code"] == 3 and j["status"] == "failed"
        slow = flow.submit(_xp("sleep 60"))
        deadline = time.time() + 10
        while flow.store.get_experiment(slow["id"])["status"] != "running" and time.time() < deadline:
            time.sleep(0.02)
        assert flow.stop_experiment(slow["id"])
        assert flow.wait("experiment", slow["id"], timeout=15) == "stopped"
    finally:
        flow.shutdown()


def test_distributed_pytorch_master_done_wins(tmp_path):
    flow = _flow(tmp_path, n_gpus=4)
    try:
        script = ("import os,sys,time; print(os.environ['RANK'], os.environ['WORLD_SIZE'], os.environ['MASTER_ADDR'],"
                  " os.environ['HIP_VISIBLE_DEVICES'], flush=True); "
                  "time.sleep(1 if os.environ['RANK']=='0' else 30)")
        spec = _xp(f"{PY} -c \"{script}\"", resources={"gpu": {"limits": 1}},
                   pytorch={"n_workers": 2, "default_worker": {"resources": {"gpu": {"limits": 1}}}})
        r = flow.submit(spec)
        assert flow.wait("experiment", r["id"], timeout=30) == "succeeded"
        jobs = flow.store.experiment_jobs(r["id"])
        assert [(j["role"], j["idx"]) for j in jobs] == [("master", 0), ("worker", 0), ("worker", 1)]
        assert all(j["status"] == "succeeded" for j in jobs)  # "Master is done."
        assert sorted(d for j in jobs for d in j["devices"]) == [0, 1, 2]
        logs = flow.logs("experiment", r["id"])
        assert "master.0 -- 0 3 127.0.0.1" in logs and "worker.1 -- 2 3 127.0.0.1" in logs
    finally:
        flow.shutdown()


def test_distributed_worker_failure_fails_experiment(tmp_path):
    flow = _flow(tmp_path, n_gpus=2)
    try:
        script = "import os,sys,time; sys.exit(5) if os.environ['RANK']=='1' else time.sleep(30)"
        r = flow.submit(_xp(f"{PY} -c \"{script}\"", pytorch={"n_workers": 1}))
        assert flow.wait("experiment", r["id"], timeout=30) == "failed"
        st = {j["role"]: j["status"] for j in flow.store.experiment_jobs(r["id"])}
        assert st == {"master": "stopped", "worker": "failed"}
    finally:
        flow.shutdown()


def test_gang_allocation_waits_for_devices(tmp_path):
    flow = _flow(tmp_path, n_gpus=2)
    try:
        a = flow.submit(_xp("sleep 0.5", resources={"gpu": {"limits": 1}}))
        b = flow.submit(_xp("true", resources={"gpu": {"limits": 2}}))
        assert flow.wait("experiment", b["id"], timeout=30) == "succeeded"
        xa, xb = flow.store.get_experiment(a["id"]), flow.store.get_experiment(b["id"])
        assert xb["started_at"] >= xa["finished_at"] - 0.05
        too_big = flow.submit(_xp("true", resources={"gpu": {"limits": 3}}))
        assert flow.wait("experiment", too_big["id"], timeout=10) == "failed"
    finally:
        flow.shutdown()


def _group(algo_block, matrix, cmd, concurrency=2, extra=None):
    d = {"version": 1, "kind": "group", "hptuning": {"concurrency": concurrency, "matrix": matrix, **algo_block},
         "run": {"cmd": cmd}}
    if extra:
        d.update(extra)
    return d


TRIAL = ("from polyaxon_amd.client import Experiment, get_declarations; import time; d = get_declarations(); "
         "e = Experiment(); time.sleep(float(d.get('sleep', 0.05))); "
         "e.log_metrics(step=1, loss=(d['lr'] - 0.3) ** 2 + 1.0 / float(d.get('steps', 1))); e.close()")


def _trial_cmd():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return f"PYTHONPATH={root} {PY} -c \"{TRIAL}\""


def test_grid_group_concurrency_and_metrics(tmp_path):
    flow = _flow(tmp_path, n_gpus=1)
    try:
        spec = _group({}, {"lr": {"values": [0.1, 0.2, 0.3]}, "sleep": {"values": [0.3, 0.31]}}, _trial_cmd(),
                      concurrency=2, extra={"environment": {"resources": {"gpu": {"limits": 0.25}}}})
        g = flow.submit(spec)
        assert flow.wait("group", g["id"], timeout=60) == "succeeded"
        xps = flow.store.list_experiments(group_id=g["id"], sort="metric.loss")
        assert len(xps) == 6 and all(x["status"] == "succeeded" for x in xps)
        assert xps[0]["declarations"]["lr"] == 0.3
        # never more than `concurrency` trials overlapping
        spans = sorted((x["started_at"], x["finished_at"]) for x in xps)
        for t, _ in spans:
            assert sum(1 for s, f in spans if s <= t < f) <= 2
        assert [s["status"] for s in flow.store.group_statuses(g["id"])] == ["created", "running", "succeeded"]
    finally:
        flow.shutdown()


def test_hyperband_group_promotions(tmp_path):
    flow = _flow(tmp_path, n_gpus=1)
    try:
        hb = {"hyperband": {"max_iter": 3, "eta": 3, "resource": {"name": "steps", "type": "int"},
                            "metric": {"name": "loss", "optimization": "minimize"}, "resume": True}, "seed": 1}
        spec = _group(hb, {"lr": {"values": [0.1, 0.2, 0.3, 0.4, 0.5]}}, _trial_cmd(), concurrency=3)
        g = flow.submit(spec)
        assert flow.wait("group", g["id"], timeout=120) == "succeeded"
        its = flow.store.iterations(g["id"])
        # max_iter=3, eta=3: s_max=1; bracket 1: 3 configs -> keep 1; bracket 0: 2 configs -> keep int(2/3)=0... +1
        seq = [(i["data"]["iteration"], i["data"]["bracket_iteration"]) for i in its]
        assert seq[0] == (0, 0) and (0, 1) in seq and (1, 0) in seq
        promoted = [x for x in flow.store.list_experiments(group_id=g["id"]) if x["cloning_strategy"] == "resume"]
        assert promoted and all(x["declarations"]["steps"] == 3 for x in promoted)
        orig = flow.store.get_experiment(promoted[0]["original_experiment_id"])
        assert promoted[0]["outputs_path"] == orig["outputs_path"]  # RESUME reuses the outputs
    finally:
        flow.shutdown()


def _reference_hyperband_schedule(max_iter, eta):
    """(iteration, bracket_iteration) pairs the reference's create_iteration visits
    (hpsearch/iteration_managers/hyperband.py:14-50): reschedule first, then reduce."""
    from polyaxon_amd.polytune.managers import HyperbandSearchManager
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    m = HyperbandSearchManager(HPTuningConfig.from_dict(
        {"hyperband": {"max_iter": max_iter, "eta": eta, "resource": {"name": "steps", "type": "int"},
                       "metric": {"name": "loss", "optimization": "minimize"}},
         "matrix": {"lr": {"uniform": [0, 1]}}}))
    seq, it = [], m.next_iteration(None)
    while True:
        seq.append((it.iteration, it.bracket_iteration))
        if m.is_done(it):
            return m, seq
        it = m.next_iteration(it)


def test_hyperband_brackets_end_where_the_reference_reschedules(tmp_path):
    """max_iter 8, eta 2: bracket 2's rung 1 has both should_reduce and should_reschedule true; the reference moves
    to the next bracket there (no third rung at 16 units > max_iter), only the last bracket keeps reducing."""
    m, ref = _reference_hyperband_schedule(8, 2)
    assert (2, 1) in ref and (2, 2) not in ref and (3, 1) in ref
    flow = _flow(tmp_path, n_gpus=8)
    try:
        hb = {"hyperband": {"max_iter": 8, "eta": 2, "resource": {"name": "steps", "type": "int"},
                            "metric": {"name": "loss", "optimization": "minimize"}, "resume": True}, "seed": 4}
        spec = _group(hb, {"lr": {"uniform": [0.0, 1.0]}, "sleep": {"values": [0.01]}}, _trial_cmd(), concurrency=8)
        g = flow.submit(spec)
        assert flow.wait("group", g["id"], timeout=180) == "succeeded"
        its = flow.store.iterations(g["id"])
        assert sorted((i["data"]["iteration"], i["data"]["bracket_iteration"]) for i in its) == sorted(ref)
        for i in its:
            d = i["data"]
            want = int(m.get_n_resources_for_iteration(d["iteration"], d["bracket_iteration"]))
            got = {flow.store.get_experiment(x)["declarations"]["steps"] for x in d["experiment_ids"]}
            assert got == {want}
        assert max(x["declarations"]["steps"] for x in flow.store.list_experiments(group_id=g["id"])) <= 2 * 8
    finally:
        flow.shutdown()


def test_random_group_early_stopping(tmp_path):
    flow = _flow(tmp_path, n_gpus=1)
    try:
        spec = _group({"random_search": {"n_experiments": 6}, "seed": 2,
                       "early_stopping": [{"metric": "loss", "value": 10.0, "optimization": "minimize"}]},
                      {"lr": {"uniform": [0.0, 1.0]}}, _trial_cmd(), concurrency=1)
        g = flow.submit(spec)
        assert flow.wait("group", g["id"], timeout=60) in ("stopped", "succeeded")
        xps = flow.store.list_experiments(group_id=g["id"])
        assert len(xps) == 6
        assert sum(x["status"] == "succeeded" for x in xps) == 1
        assert sum(x["status"] == "stopped" for x in xps) == 5
    finally:
        flow.shutdown()


def test_bo_and_asha_groups(tmp_path):
    flow = _flow(tmp_path, n_gpus=1)
    try:
        bo = {"bo": {"n_iterations": 2, "n_initial_trials": 3, "metric": {"name": "loss", "optimization": "minimize"},
                     "utility_function": {"acquisition_function": "ucb", "kappa": 1.0,
                                          "gaussian_process": {"kernel": "matern", "nu": 2.5}}}, "seed": 3}
        g = flow.submit(_group(bo, {"lr": {"uniform": [0.0, 1.0]}}, _trial_cmd(), concurrency=3))
        assert flow.wait("group", g["id"], timeout=120) == "succeeded"
        assert len(flow.store.list_experiments(group_id=g["id"])) == 3 + 2
        asha = {"asha": {"min_resource": 1, "max_resource": 9, "eta": 3, "n_experiments": 6,
                         "resource": {"name": "steps", "type": "int"},
                         "metric": {"name": "loss", "optimization": "minimize"}}, "seed": 4}
        g2 = flow.submit(_group(asha, {"lr": {"uniform": [0.0, 1.0]}}, _trial_cmd(), concurrency=2))
        assert flow.wait("group", g2["id"], timeout=120) == "succeeded"
        xps = flow.store.list_experiments(group_id=g2["id"])
        assert len([x for x in xps if x["declarations"]["steps"] == 1]) == 6
        assert any(x["declarations"]["steps"] == 3 for x in xps)
    finally:
        flow.shutdown()


def test_clone_strategies(tmp_path):
    flow = _flow(tmp_path)
    try:
        r = flow.submit(_xp("echo hi > $POLYAXON_RUN_OUTPUTS_PATH/ckpt.txt"))
        assert flow.wait("experiment", r["id"], timeout=30) == "succeeded"
        orig = flow.store.get_experiment(r["id"])
        res = flow.clone_experiment(r["id"], "resume")
        cp = flow.clone_experiment(r["id"], "copy")
        rs = flow.clone_experiment(r["id"], "restart", declarations={"lr": 1})
        for x in (res, cp, rs):
            flow.wait("experiment", x, timeout=30)
        assert flow.store.get_experiment(res)["outputs_path"] == orig["outputs_path"]
        cpx = flow.store.get_experiment(cp)
        assert cpx["outputs_path"] != orig["outputs_path"] and os.path.exists(os.path.join(cpx["outputs_path"], "ckpt.txt"))
        assert flow.store.get_experiment(rs)["declarations"]["lr"] == 1
        assert flow.store.get_experiment(rs)["original_experiment_id"] == r["id"]
    finally:
        flow.shutdown()


def test_trial_to_trial_gap_is_small(tmp_path):
    flow = _flow(tmp_path, n_gpus=1)
    try:
        g = flow.submit(_group({}, {"i": {"range": [0, 8, 1]}}, "true", concurrency=1))
        assert flow.wait("group", g["id"], timeout=60) == "succeeded"
        gaps = flow.stats["gaps_ms"]
        assert len(gaps) >= 7
        assert sorted(gaps)[len(gaps) // 2] < 100.0  # SURVEY.md §7.3 acceptance: < 100 ms
    finally:
        flow.shutdown()


def test_jobs_and_builds(tmp_path):
    flow = _flow(tmp_path)
    try:
        j = flow.submit({"version": 1, "kind": "job", "run": {"cmd": "echo job-ran"}})
        assert flow.wait("job", j["id"], timeout=30) == "succeeded"
        assert "job-ran" in flow.logs("job", j["id"])
        spec = _xp("test -n \"$PLX_BUILD_DIR\" && cat $PLX_BUILD_DIR/marker")
        spec["build"] = {"image": "rocm/pytorch", "build_steps": ["echo built > $PLX_BUILD_DIR/marker"]}
        x1 = flow.submit(spec)
        assert flow.wait("experiment", x1["id"], timeout=30) == "succeeded"
        x2 = flow.submit(spec)
        assert flow.wait("experiment", x2["id"], timeout=30) == "succeeded"
        builds = flow.store.list_jobs(kind="build")
        assert len(builds) == 1  # second experiment reused the build (6 h window)
        assert "built" in flow.logs("experiment", x2["id"])
        # the rendered Dockerfile lands in the build's environment directory (reproducible as an image)
        dockerfile = open(os.path.join(builds[0]["outputs_path"], "Dockerfile")).read()
        assert dockerfile.startswith("FROM rocm/pytorch\n")
        assert "RUN echo built > $PLX_BUILD_DIR/marker" in dockerfile
    finally:
        flow.shutdown()


def test_dockerfile_and_image_naming(tmp_path):
    from polyaxon_amd.polyflow import dockerizer

    (tmp_path / "requirements.txt").write_text("numpy\n")
    text = dockerizer.render_dockerfile("rocm/pytorch:latest", ["pip install -r requirements.txt", "make"],
                                        [["LR", "0.1"], ["MSG", "two words"]], context=str(tmp_path))
    lines = text.splitlines()
    assert lines[0] == "FROM rocm/pytorch:latest"
    assert "ENV LR=0.1" in lines and 'ENV MSG="two words"' in lines
    # manifests are copied before the steps (cache-friendly), the code after them
    assert lines.index("COPY requirements.txt /code/") < lines.index("RUN pip install -r requirements.txt")
    assert lines.index("RUN make") < lines.index("COPY . /code")
    assert dockerizer.tagged_image("MyProj", 7, "abc") == "localhost:5000/myproj_7:abc"
    assert dockerizer.resolve_backend("native") == "native"
    with pytest.raises(ValueError):
        dockerizer.resolve_backend("kaniko")
    with pytest.raises(ValueError):
        dockerizer.render_dockerfile("", [])


def test_container_build_backend(tmp_path, monkeypatch):
    """build.backend=container: the scheduler builds the rendered Dockerfile with the engine on PATH (a fake
    docker here that records its argv) and records the tagged image on the build job."""
    bindir = tmp_path / "bin"
    bindir.mkdir()
    argv_log = tmp_path / "docker_argv"
    fake = bindir / "docker"
    fake.write_text(f"#!/bin/sh\necho \"$@\" >> {argv_log}\n")
    fake.chmod(0o755)
    monkeypatch.setenv("PATH", f"{bindir}:{os.environ['PATH']}")
    from polyaxon_amd.polyflow import dockerizer

    assert dockerizer.resolve_backend("auto") == "container"
    flow = _flow(tmp_path)
    flow.build_backend, flow.build_push = "container", True
    try:
        spec = _xp("true")
        spec["build"] = {"image": "rocm/pytorch", "build_steps": ["pip install einops"], "nocache": True}
        x = flow.submit(spec)
        assert flow.wait("experiment", x["id"], timeout=30) == "succeeded"
        b = flow.store.list_jobs(kind="build")[0]
        assert b["image"].startswith("localhost:5000/") and ":" in b["image"].split("/", 1)[1]
        calls = argv_log.read_text().splitlines()
        assert calls[0].startswith(f"build -t {b['image']} -f ") and "--no-cache" in calls[0]
        assert calls[0].split(" -f ")[1].split()[0].endswith("Dockerfile")
        assert calls[1] == f"push {b['image']}"
    finally:
        flow.shutdown()


def test_pipeline_dag_triggers_and_retries(tmp_path):
    from polyaxon_amd.polyflow.pipelines import sort_topologically, trigger_satisfied

    assert sort_topologically({"a": {"b", "c"}, "b": {"d"}, "c": {"d"}, "d": set()}) == ["a", "b", "c", "d"]
    with pytest.raises(ValueError):
        sort_topologically({"a": {"b"}, "b": {"a"}})
    assert trigger_satisfied("all_succeeded", ["succeeded", "running"]) is None
    assert trigger_satisfied("all_succeeded", ["succeeded", "failed"]) is False
    assert trigger_satisfied("one_failed", ["failed", "running"]) is True
    assert trigger_satisfied("all_done", ["failed", "stopped"]) is True

    flow = _flow(tmp_path)
    try:
        counter = tmp_path / "count"
        flaky = f"n=$(cat {counter} 2>/dev/null || echo 0); echo $((n+1)) > {counter}; test $n -ge 1"
        job = lambda cmd: {"version": 1, "kind": "job", "run": {"cmd": cmd}}  # noqa: E731
        spec = {"version": 1, "kind": "pipeline", "concurrency": 2, "ops": [
            {"name": "prep", "template": job("true")},
            {"name": "flaky", "upstream": ["prep"], "max_retries": 2, "retry_delay": 0.05,
             "template": job(flaky)},
            {"name": "never", "upstream": ["prep"], "template": job("exit 1")},
            {"name": "after_fail", "upstream": ["never"], "trigger": "all_succeeded", "template": job("true")},
            {"name": "cleanup", "upstream": ["flaky", "never"], "trigger": "all_done", "template": job("true")}]}
        r = flow.submit(spec)
        assert flow.wait("pipeline_run", r["run_id"], timeout=60) == "finished"
        ops = {o["name"]: o for o in flow.store.operation_runs(r["run_id"])}
        assert ops["prep"]["status"] == "succeeded"
        assert ops["flaky"]["status"] == "succeeded" and ops["flaky"]["retries"] == 1
        assert ops["never"]["status"] == "failed"
        assert ops["after_fail"]["status"] == "upstream_failed"
        assert ops["cleanup"]["status"] == "succeeded"
    finally:
        flow.shutdown()


def test_process_mode_hyperband_runs_brackets_concurrently(tmp_path):
    """examples/resnet50_hyperband.yml (max_iter 9, eta 3, concurrency 8) in process mode with stub trials on 8
    virtual devices: the three brackets share the slots, so while any trial waits in the group's queue all 8 devices
    are busy (the reference runs the brackets one after another: bracket 0's 3-config rung 1 would idle 5 GPUs)."""
    import yaml

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = yaml.safe_load(open(os.path.join(root, "examples", "resnet50_hyperband.yml")))
    stub = TRIAL.replace("d.get('steps', 1)", "d['units']").replace("float(d.get('sleep', 0.05))", "0.4")
    stub = stub.replace("(d['lr'] - 0.3) ** 2", "abs(d['lr'] - 0.3)")
    spec["run"]["cmd"] = f"PYTHONPATH={root} {PY} -c \"{stub}\""
    flow = _flow(tmp_path, n_gpus=8)
    try:
        g = flow.submit(spec)
        gid = g["id"]
        samples = []
        end = time.time() + 120
        while time.time() < end:
            st = flow.store.group_status_counts(gid)
            running = sum(st.get(k, 0) for k in ("scheduled", "starting", "running"))
            queued = st.get("created", 0)
            samples.append((running, queued))
            if flow.store.get_group(gid)["status"] in ("succeeded", "failed", "stopped"):
                break
            time.sleep(0.02)
        assert flow.store.get_group(gid)["status"] == "succeeded"
        xs = flow.store.list_experiments(group_id=gid)
        assert len(xs) == 9 + 5 + 3 + 3 + 1 + 1 + 1  # reference bracket arithmetic (incl. the s=0 reduction)
        busy = [r for r, q in samples if q > 0]
        assert busy and max(r for r, _ in samples) == 8
        assert sum(1 for r in busy if r == 8) >= 0.8 * len(busy), samples
        its = flow.store.iterations(gid)
        assert sorted((i["data"]["iteration"], i["data"]["bracket_iteration"]) for i in its) == [
            (0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (2, 0), (2, 1)]
    finally:
        flow.shutdown()
