"""Resident executors inside polyflow (polyflow/resident.py, pool.py, groups.ResidentHyperbandDriver) on CPU.

The reference runs every Hyperband trial as a pod and reduces rungs with a Python sort after a 30 s poll
(polyaxon/hpsearch/tasks/hyperband.py:7-83, iteration_managers/hyperband.py:52-113).  These tests check that the
resident path keeps the reference's observable semantics -- same suggestions, same bracket/rung arithmetic,
promotions = top-k of the rung, RESUME clones, FSM history per trial, iteration rows -- while running brackets
concurrently on warm executors.
"""
import math
import os
import socket
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _hp(seed=3, max_iter=9, eta=3, resume=True, concurrency=2, early=None):
    hp = {"seed": seed, "concurrency": concurrency,
          "hyperband": {"max_iter": max_iter, "eta": eta, "resource": {"name": "units", "type": "int"},
                        "metric": {"name": "loss", "optimization": "minimize"}, "resume": resume},
          "matrix": {"lr": {"loguniform": [-4, -1]}, "momentum": {"uniform": [0.8, 0.95]}}}
    if early:
        hp["early_stopping"] = early
    return hp


TINY = {"unit_steps": 1, "batch": 4, "image": 16, "grid": 4}


def _group(**kw):
    params = kw.pop("params", TINY)
    return {"version": 1, "kind": "group", "project": "rt", "hptuning": _hp(**kw),
            "environment": {"resources": {"gpu": 1},
                            "executor": {"kind": "resident", "program": "resnet_tiny", "params": params}}}


def test_channel_roundtrip():
    from polyaxon_amd.polyflow.resident import Channel, ChannelClosed

    a, b = socket.socketpair()
    ca, cb = Channel(a), Channel(b)
    assert cb.recv(timeout=0) is None
    big = {"x": list(range(20000)), "s": "é" * 100, "nan": float("nan")}
    ca.send({"op": "ping"})
    ca.send(big)
    assert cb.recv() == {"op": "ping"}
    got = cb.recv()
    assert got["x"] == big["x"] and got["s"] == big["s"] and math.isnan(got["nan"])
    ca.close()
    with pytest.raises(ChannelClosed):
        cb.recv()


def test_bracket_units_follow_reference_arithmetic():
    from polyaxon_amd.polyflow.programs import bracket_units
    from polyaxon_amd.polytune.managers import HyperbandSearchManager
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    for max_iter, eta, resume in ((9, 3, True), (9, 3, False), (81, 3, True), (10, 3, False), (27, 3, True),
                                  (8, 2, True), (16, 2, False)):
        m = HyperbandSearchManager(HPTuningConfig.from_dict(_hp(max_iter=max_iter, eta=eta, resume=resume)))
        totals, prev, n = {}, {}, {}
        cur = m.next_iteration(None)
        while True:  # walk the reference state machine (reschedule before reduce)
            it, rung = cur.iteration, cur.bracket_iteration
            cnt = m.get_n_configs(m.get_bracket(it)) if rung == 0 else n[it]
            r = m.get_n_resources_for_iteration(it, rung)
            totals[it] = totals.get(it, 0.0) + cnt * ((r - prev[it]) if (resume and rung) else r)
            prev[it], n[it] = r, m.get_n_config_to_keep_for_iteration(it, rung)
            if m.is_done(cur):
                break
            cur = m.next_iteration(cur)
        for it in range(m.s_max + 1):
            assert bracket_units(max_iter, eta, it, resume) == pytest.approx(totals[it])


def _worker_thread(program="resnet_tiny", params=TINY, max_active=8):
    from polyaxon_amd.polyflow.resident import Channel, ResidentWorker, serve_forever

    a, b = socket.socketpair()
    sched, wchan = Channel(a), Channel(b)
    w = ResidentWorker(program, device="cpu", max_active=max_active)
    t = threading.Thread(target=serve_forever, args=(w, wchan), daemon=True)
    t.start()
    sched.send({"op": "init", "program": program, "params": params, "max_active": max_active})
    ready = sched.recv(timeout=120)
    assert ready["ev"] == "ready", ready
    return w, sched, t


def _collect(sched, n_brackets, timeout=300):  # generous: CPU training slows under a loaded parallel run
    evs = []
    done = 0
    end = time.time() + timeout
    while done < n_brackets:
        m = sched.recv(timeout=max(0.1, end - time.time()))
        assert m is not None, "worker stalled"
        evs.append(m)
        if m["ev"] == "bracket_done":
            done += 1
        assert m["ev"] != "error", m
    return evs


def test_worker_brackets_end_where_the_reference_reschedules():
    """eta 2 / max_iter 8: each bracket runs exactly the rungs of the reference state machine
    (hpsearch/iteration_managers/hyperband.py:25-36: reschedule before reduce)."""
    from polyaxon_amd.polytune.managers import HyperbandIterationConfig, HyperbandSearchManager
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    hp = _hp(max_iter=8, eta=2)
    m = HyperbandSearchManager(HPTuningConfig.from_dict(hp))
    ref, it = {}, m.next_iteration(None)
    while True:
        ref.setdefault(it.iteration, []).append(it.bracket_iteration)
        if m.is_done(it):
            break
        it = m.next_iteration(it)
    assert ref[2] == [0, 1]  # the case the concurrent driver used to extend to a third rung
    w, sched, t = _worker_thread()
    for it in range(m.s_max + 1):
        sugg = m.get_suggestions(HyperbandIterationConfig(iteration=it))
        sched.send({"op": "bracket", "key": f"b{it}", "hptuning": hp, "iteration": it, "seed": 5,
                    "configs": [{"cid": i, "params": {k: v for k, v in s.items() if k != "units"}}
                                for i, s in enumerate(sugg)]})
    evs = _collect(sched, m.s_max + 1)
    ran = {}
    for e in evs:
        if e["ev"] == "trial_start":
            ran.setdefault(int(e["key"][1:]), set()).add(e["rung"])
    assert {k: sorted(v) for k, v in ran.items()} == ref


def test_worker_runs_concurrent_brackets_with_reference_promotions():
    from polyaxon_amd.polytune.managers import HyperbandIterationConfig, HyperbandSearchManager
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    hp = _hp()
    m = HyperbandSearchManager(HPTuningConfig.from_dict(hp))
    w, sched, t = _worker_thread()
    for it in range(m.s_max + 1):
        sugg = m.get_suggestions(HyperbandIterationConfig(iteration=it))
        sched.send({"op": "bracket", "key": f"b{it}", "hptuning": hp, "iteration": it, "seed": 5,
                    "configs": [{"cid": i, "params": {k: v for k, v in s.items() if k != "units"}}
                                for i, s in enumerate(sugg)]})
    evs = _collect(sched, m.s_max + 1)
    starts = [e for e in evs if e["ev"] == "trial_start"]
    ends = [e for e in evs if e["ev"] == "trial_end"]
    rungs = [e for e in evs if e["ev"] == "rung_done"]
    assert len(starts) == len(ends) == 23  # 13 + 6 + 4 trials (reference arithmetic, incl. the s=0 reduction)
    for e in rungs:
        it = int(e["key"][1:])
        keep = m.get_n_config_to_keep_for_iteration(it, e["rung"])
        ranked = [c for c, v in sorted(e["metrics"], key=lambda cv: (cv[1], cv[0]))]
        assert e["promoted"] == ranked[:keep]  # device top-k == reference sort + keep
        # resources follow the reference schedule
        res = {s["params"]["units"] for s in starts if s["key"] == e["key"] and s["rung"] == e["rung"]}
        assert res == {int(m.get_n_resources_for_iteration(it, e["rung"]))}
    # the brackets were interleaved: one decision launch per round covered all of them
    assert w.stats["rounds"] < len(rungs)
    assert w.stats["topk_launches"] == w.stats["rounds"]
    # resumed trials train only the additional resource
    by = {(e["key"], e["rung"], e["cid"]): e for e in ends}
    for (key, rung, cid), e in by.items():
        if rung:
            it = int(key[1:])
            extra = m.get_n_resources_for_iteration(it, rung) - m.get_n_resources_for_iteration(it, rung - 1)
            assert e["steps"] == int(extra) * TINY["unit_steps"]
    sched.send({"op": "shutdown"})
    t.join(10)


def test_worker_stop_bracket_and_pause():
    from polyaxon_amd.polytune.managers import HyperbandIterationConfig, HyperbandSearchManager
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    hp = _hp()
    m = HyperbandSearchManager(HPTuningConfig.from_dict(hp))
    w, sched, t = _worker_thread(max_active=1)
    for it in range(2):
        sugg = m.get_suggestions(HyperbandIterationConfig(iteration=it))
        sched.send({"op": "bracket", "key": f"b{it}", "hptuning": hp, "iteration": it, "seed": 1,
                    "configs": [{"cid": i, "params": {"lr": s["lr"], "momentum": s["momentum"]}}
                                for i, s in enumerate(sugg)]})
    sched.send({"op": "stop_bracket", "key": "b1"})  # still queued (max_active=1): stopped without running
    sched.send({"op": "pause", "tag": "p"})
    evs = _collect(sched, 2)
    done = {e["key"]: e["status"] for e in evs if e["ev"] == "bracket_done"}
    assert done == {"b0": "succeeded", "b1": "stopped"}
    assert not any(e["ev"] == "trial_start" and e["key"] == "b1" for e in evs)
    paused = sched.recv(timeout=30)
    assert paused["ev"] == "paused" and paused["tag"] == "p"
    sched.send({"op": "shutdown"})
    t.join(10)


def test_worker_early_stopping_on_device_metric():
    from polyaxon_amd.polytune.managers import HyperbandIterationConfig, HyperbandSearchManager
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    hp = _hp(early=[{"metric": "loss", "value": 100.0, "optimization": "minimize"}])  # trips on the first rung
    m = HyperbandSearchManager(HPTuningConfig.from_dict(hp))
    w, sched, t = _worker_thread()
    sugg = m.get_suggestions(HyperbandIterationConfig(iteration=0))
    sched.send({"op": "bracket", "key": "b0", "hptuning": hp, "iteration": 0, "seed": 1,
                "early_stopping": hp["early_stopping"],
                "configs": [{"cid": i, "params": {"lr": s["lr"]}} for i, s in enumerate(sugg)]})
    evs = _collect(sched, 1)
    rung = [e for e in evs if e["ev"] == "rung_done"]
    assert len(rung) == 1 and rung[0]["early_stop"] and rung[0]["promoted"] == []
    assert [e["status"] for e in evs if e["ev"] == "bracket_done"] == ["stopped"]
    assert w.stats["early_stop_launches"] == 1
    sched.send({"op": "shutdown"})
    t.join(10)


@pytest.fixture
def cpu_pool_env(monkeypatch):
    monkeypatch.setenv("PLX_NUM_GPUS", "2")
    monkeypatch.setenv("PLX_CPU_ONLY", "1")
    monkeypatch.setenv("OMP_NUM_THREADS", "2")


def test_polyflow_resident_group_end_to_end(tmp_path, cpu_pool_env):
    from polyaxon_amd.polyflow.scheduler import Polyflow

    with Polyflow(str(tmp_path), reconcile_s=0) as flow:
        r = flow.submit(_group())
        assert flow.wait("group", r["id"], timeout=300) == "succeeded"
        st = flow.store
        xs = st.list_experiments(group_id=r["id"])
        assert len(xs) == 23 and {x["status"] for x in xs} == {"succeeded"}
        for x in xs:
            assert [s["status"] for s in st.experiment_statuses(x["id"])] == [
                "created", "scheduled", "starting", "running", "succeeded"]
            assert "loss" in x["last_metric"] and x["started_at"] <= x["finished_at"]
            jobs = st.experiment_jobs(x["id"])
            assert len(jobs) == 1 and jobs[0]["status"] == "succeeded" and jobs[0]["devices"] in ([0], [1])
        resumed = [x for x in xs if x["cloning_strategy"] == "resume"]
        assert len(resumed) == 6
        for x in resumed:  # RESUME: same outputs as the root, one more resource level
            orig = st.get_experiment(x["original_experiment_id"])
            assert x["declarations"]["units"] > orig["declarations"]["units"]
            assert x["outputs_path"] == orig["outputs_path"] or orig["cloning_strategy"] == "resume"
            assert x["declarations"]["lr"] == orig["declarations"]["lr"]
        its = st.iterations(r["id"])
        assert len(its) == 7  # 3 + 2 + 2 rungs
        for it in its:
            d = it["data"]
            vals = dict((int(a), b) for a, b in d["experiments_metrics"])
            keep = len(d["promoted"])
            assert d["promoted"] == sorted(vals, key=lambda k: vals[k])[:keep]
        # both executors were used (brackets run concurrently) and stay warm for the next group
        pool = flow.call(lambda: flow.resident_pool().snapshot())
        assert len(pool) == 2 and all(p["ready"] and p["alive"] for p in pool)
        assert {tuple(j["devices"]) for x in xs for j in st.experiment_jobs(x["id"])} == {(0,), (1,)}
        # a second group reuses the warm executors (no new processes)
        pids = {p["pid"] for p in pool}
        r2 = flow.submit(_group(seed=11, concurrency=1))
        assert flow.wait("group", r2["id"], timeout=300) == "succeeded"
        pool2 = flow.call(lambda: flow.resident_pool().snapshot())
        assert {p["pid"] for p in pool2} == pids
        used = {tuple(j["devices"]) for x in st.list_experiments(group_id=r2["id"]) for j in st.experiment_jobs(x["id"])}
        assert len(used) == 1  # concurrency: 1 -> one executor
    # shutdown released every device
    assert flow.alloc.allocations == {}


def _kill_when_running(flow, gid, n_ready=1, timeout=120, exclude=()):
    end = time.time() + timeout
    while time.time() < end:
        snap = [p for p in flow.call(lambda: flow.resident_pool().snapshot()) if p["alive"] and p["pid"] not in exclude]
        running = flow.store.list_experiments(group_id=gid)
        if len(snap) >= n_ready and snap[0]["ready"] and any(x["status"] == "running" for x in running):
            os.kill(snap[0]["pid"], 9)
            return snap[0]["pid"]
        time.sleep(0.05)
    raise AssertionError("no running resident trial to interrupt")


def test_resident_executor_crash_redispatches_brackets(tmp_path, cpu_pool_env):
    """A lost executor's unfinished brackets go to a replacement executor (spawned on the freed device) and continue
    after their last completed rung; the trials that were running fail, the group still completes every bracket."""
    from polyaxon_amd.polyflow.scheduler import Polyflow

    params = dict(TINY, unit_steps=3)
    with Polyflow(str(tmp_path), reconcile_s=0) as flow:
        r = flow.submit(_group(concurrency=1, params=params))
        pid = _kill_when_running(flow, r["id"])
        assert flow.wait("group", r["id"], timeout=300) == "succeeded"
        xs = flow.store.list_experiments(group_id=r["id"])
        assert any(x["status"] == "failed" for x in xs)
        assert all(x["status"] in ("succeeded", "failed") for x in xs)
        ev = flow.store.cluster_events()
        assert any(e["kind"] == "resident_executor" and "gone" in e["message"] for e in ev)
        assert any(e["kind"] == "resident_executor" and "re-dispatched" in e["message"] for e in ev)
        # every bracket reached its last rung: 3 + 2 + 2 rung decisions (more if a rung was redone)
        its = flow.store.iterations(r["id"])
        last = {}
        for it in its:
            d = it["data"]
            last[d["iteration"]] = max(last.get(d["iteration"], -1), d["bracket_iteration"])
        assert last == {0: 2, 1: 1, 2: 1}
        # the dead executor's device was released; the replacement holds one
        snap = flow.call(lambda: flow.resident_pool().snapshot())
        assert any(p["alive"] and p["pid"] != pid for p in snap)
        assert not any(p["alive"] and p["pid"] == pid for p in snap)
        owners = [o for o in flow.alloc.allocations if o.startswith("resident:")]
        assert owners and "resident:1" not in owners


def test_resident_group_fails_when_no_executor_can_be_placed(tmp_path, cpu_pool_env):
    from polyaxon_amd.polyflow.scheduler import Polyflow

    g = _group()
    g["environment"]["resources"] = {"gpu": 1, "hbm": 100000}
    with Polyflow(str(tmp_path), reconcile_s=0) as flow:
        r = flow.submit(g)
        assert flow.wait("group", r["id"], timeout=30) == "failed"
        assert "placed" in (flow.store.group_statuses(r["id"])[-1].get("message") or "")


def _asha_group(n=14, seed=5, concurrency=1, shards=1, params=None, min_r=1, max_r=9, eta=3):
    return {"version": 1, "kind": "group", "project": "rt",
            "hptuning": {"seed": seed, "concurrency": concurrency,
                         "asha": {"min_resource": min_r, "max_resource": max_r, "eta": eta, "n_experiments": n,
                                  "resource": {"name": "units", "type": "int"},
                                  "metric": {"name": "loss", "optimization": "minimize"}, "resume": True},
                         "matrix": {"lr": {"loguniform": [-4, -1]}, "momentum": {"uniform": [0.8, 0.95]}}},
            "environment": {"resources": {"gpu": 1},
                            "executor": {"kind": "resident", "program": "resnet_tiny", "params": params or TINY,
                                         "shards": shards}}}


def test_worker_runs_asha_shard_asynchronously():
    """One ASHA shard on a worker: every round runs one job; a config enters rung k+1 only from the top
    floor(n_k / eta) of rung k's results at decision time; promoted jobs resume (train only the extra resource)."""
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    g = _asha_group(n=10)
    hp = HPTuningConfig.from_dict(g["hptuning"])
    w, sched, t = _worker_thread()
    from polyaxon_amd.polytune.managers import AshaSearchManager

    sugg = AshaSearchManager(hp).get_suggestions()
    sched.send({"op": "asha", "key": "a0", "hptuning": g["hptuning"], "iteration": 0, "seed": 3,
                "configs": [{"cid": i, "params": {k: v for k, v in p.items() if k != "units"}}
                            for i, p in enumerate(sugg)]})
    evs = _collect(sched, 1)
    starts = [e for e in evs if e["ev"] == "trial_start"]
    ends = [e for e in evs if e["ev"] == "trial_end"]
    assert len(starts) == len(ends) and w.stats["asha_jobs"] == len(ends)
    assert sum(1 for e in ends if e["rung"] == 0) == 10
    # replay the decisions: at each promotion the config was in the top floor(n/eta) of its rung so far
    seen = {0: {}, 1: {}, 2: {}}
    for e in evs:
        if e["ev"] == "trial_start" and e["rung"] > 0:
            prev = seen[e["rung"] - 1]
            k = int(len(prev) / 3)
            top = sorted(prev, key=lambda c: (prev[c], c))[:k]
            assert e["cid"] in top, (e, prev)
            assert e["resumed"] is True
            assert e["params"]["units"] == 3 ** e["rung"]
        if e["ev"] == "trial_end" and e["metric"] is not None:
            seen[e["rung"]][e["cid"]] = e["metric"]
    for e in ends:
        if e["rung"] > 0:
            assert e["steps"] == (3 ** e["rung"] - 3 ** (e["rung"] - 1)) * TINY["unit_steps"]
    assert any(e["rung"] == 2 for e in ends)  # promotions reached the top rung
    rungs = [e for e in evs if e["ev"] == "rung_done"]
    assert [r["rung"] for r in rungs] == [0, 1, 2]
    assert [e["status"] for e in evs if e["ev"] == "bracket_done"] == ["succeeded"]
    assert not any(k[0] == "a0" for k in w.program.executor.snapshots if isinstance(k, tuple))
    sched.send({"op": "shutdown"})
    t.join(10)


def test_polyflow_resident_asha_group_end_to_end(tmp_path, cpu_pool_env):
    from polyaxon_amd.polyflow.scheduler import Polyflow

    with Polyflow(str(tmp_path), reconcile_s=0) as flow:
        r = flow.submit(_asha_group(n=12, concurrency=2, shards=2))
        assert flow.wait("group", r["id"], timeout=300) == "succeeded"
        st = flow.store
        xs = st.list_experiments(group_id=r["id"])
        assert sum(1 for x in xs if x["declarations"]["units"] == 1) == 12
        assert {x["status"] for x in xs} == {"succeeded"}
        for x in xs:
            assert [s["status"] for s in st.experiment_statuses(x["id"])] == [
                "created", "scheduled", "starting", "running", "succeeded"]
        resumed = [x for x in xs if x["cloning_strategy"] == "resume"]
        assert resumed
        for x in resumed:  # RESUME lineage: same config, one rung lower, same outputs
            orig = st.get_experiment(x["original_experiment_id"])
            assert x["declarations"]["units"] == 3 * orig["declarations"]["units"]
            assert x["declarations"]["lr"] == orig["declarations"]["lr"]
            assert x["outputs_path"] == orig["outputs_path"]
        its = st.iterations(r["id"])
        assert {it["data"]["unit"] for it in its} == {"asha"}
        # two shards on two executors
        assert {tuple(j["devices"]) for x in xs for j in st.experiment_jobs(x["id"])} == {(0,), (1,)}


def test_resident_asha_shard_survives_executor_loss(tmp_path, cpu_pool_env):
    from polyaxon_amd.polyflow.scheduler import Polyflow

    with Polyflow(str(tmp_path), reconcile_s=0) as flow:
        r = flow.submit(_asha_group(n=9, params=dict(TINY, unit_steps=3)))
        _kill_when_running(flow, r["id"])
        assert flow.wait("group", r["id"], timeout=300) == "succeeded"
        xs = flow.store.list_experiments(group_id=r["id"])
        done0 = {x["declarations"]["lr"] for x in xs if x["declarations"]["units"] == 1 and x["status"] == "succeeded"}
        assert len(done0) == 9  # every config was evaluated at rung 0 despite the crash
        ev = flow.store.cluster_events()
        assert any("re-dispatched" in e["message"] for e in ev)


def test_resident_spec_validation():
    from polyaxon_amd.spec import specification_for
    from polyaxon_amd.spec.specification import PolyaxonfileError

    spec = specification_for(_group())
    assert spec.environment.executor.resident and spec.environment.executor.program == "resnet_tiny"
    assert spec.environment.to_dict()["executor"]["kind"] == "resident"
    bad = _group()
    bad["environment"]["executor"] = {"kind": "resident"}
    with pytest.raises(PolyaxonfileError):
        specification_for(bad)
    bad = _group()
    bad["environment"]["executor"]["kind"] = "magic"
    with pytest.raises(PolyaxonfileError):
        specification_for(bad)
    bad = _group()
    bad["environment"]["resources"] = {"gpu": 1.5}
    with pytest.raises(PolyaxonfileError):
        specification_for(bad)
    # a standalone experiment cannot name a resident executor (only a group's trials are trained by one)
    xp = {"version": 1, "kind": "experiment", "environment": _group()["environment"]}
    with pytest.raises(PolyaxonfileError):
        specification_for(xp)
    # ... while the group's own trial specs (no run section) still parse
    assert specification_for(_group()).get_experiment_spec({"lr": 0.01, "momentum": 0.9, "units": 1}).run is None


def test_resident_rejects_grid_random(tmp_path, cpu_pool_env):
    from polyaxon_amd.polyflow.scheduler import Polyflow
    from polyaxon_amd.spec.specification import PolyaxonfileError

    g = _group()
    del g["hptuning"]["hyperband"]
    g["hptuning"]["random_search"] = {"n_experiments": 3}
    with Polyflow(str(tmp_path), reconcile_s=0) as flow:
        with pytest.raises(PolyaxonfileError):
            flow.submit(g)
        assert flow.store.list_groups() == []


def test_bench_cpu_two_ranks_complete_sweeps():
    """bench.py --gpus 2 spawns its own two ranks, times whole sweeps through polyflow and reports n_gpus: 2."""
    import json

    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2", "--steps", "1",
                          "--warmup", "0"], capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["steps"] == 1
    assert res["config"]["sweeps"] == 2 and res["config"]["brackets"] == 6
    assert res["trials"] == 46 and res["trials_succeeded"] == 46
    assert res["store_fsm_history_ok"] is True
    assert res["value"] > 0 and res["ms_per_step"] > 0


def _bench(*extra, threads="1", timeout=900):
    import json

    env = dict(os.environ, OMP_NUM_THREADS=threads)
    env.pop("WORLD_SIZE", None)
    env.pop("PLX_BENCH_CONTROL", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", *extra], capture_output=True,
                         text=True, timeout=timeout, env=env, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])


def test_bench_cpu_four_ranks_scheduler_off_the_ranks():
    """The scheduler runs in the launcher (no GPU, no rank): its PID is none of the ranks'; per-rank times, trials
    and executor loads are reported, and the brackets are balanced to within one bracket of the mean load."""
    from polyaxon_amd.polyflow.programs import bracket_units

    res = _bench("--gpus", "4", "--steps", "2", "--warmup", "0")
    assert res["n_gpus"] == 4 and res["trials"] == 8 * 23
    ranks = res["per_rank"]
    assert len(ranks) == 4 and res["control_pid"] not in {r["pid"] for r in ranks}
    assert sum(r["trials"] for r in ranks) == res["trials"]
    assert all(r["elapsed_s"] > 0 for r in ranks)
    loads = [e["load_units"] for e in res["executors"]]
    assert len(loads) == 4 and sum(loads) == pytest.approx(8 * 87)
    biggest = max(bracket_units(9, 3, it, True) for it in range(3))
    mean = sum(loads) / 4
    assert all(abs(x - mean) <= biggest for x in loads), loads


def test_bench_cpu_single_rank_control_process_and_asha():
    """--gpus 1 (and torchrun's rank 0) start the scheduler as a process of its own; --search asha times whole
    asynchronous successive-halving sweeps through the same resident path."""
    res = _bench("--gpus", "1", "--steps", "1", "--warmup", "0", "--search", "asha", "--asha-n", "12", threads="2")
    assert res["n_gpus"] == 1 and res["control_pid"] != res["per_rank"][0]["pid"]
    assert res["config"]["search"].startswith("asha") and res["trials_succeeded"] == res["trials"]
    assert res["trials"] > 12 and res["trials_resumed"] > 0  # promotions happened and resumed


def test_bench_cpu_under_torchrun_like_the_driver():
    """The driver's multi-GPU launch, rehearsed on CPU: ``python -m torch.distributed.run --nproc-per-node 2
    --master-addr 127.0.0.1 bench.py --gpus 2``; rank 0 prints the one JSON line with the whole-job value."""
    import json
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PLX_BENCH_CONTROL"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2", "--steps", "1", "--warmup", "0"],
                         capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 1 and res["warmup"] == 0
    assert res["trials"] == 46 and res["trials_succeeded"] == 46 and res["store_fsm_history_ok"] is True
    assert res["value"] > 0 and res["higher_is_better"] is True and res["scaling"] == "weak"


def test_idle_resident_executors_yield_to_a_waiting_gang(tmp_path, monkeypatch):
    """A DP=8 experiment submitted while a resident Hyperband group holds executors on 2 of 8 (virtual) devices waits
    for devices; the moment the group's last bracket ends, its idle executors are released (not after the 300 s idle
    timeout) and the gang starts within a reconcile tick (reference: concurrency is counted against the cluster for
    every run, polyaxon/db/models/experiment_groups.py:193-197)."""
    from polyaxon_amd.polyflow.scheduler import Polyflow

    monkeypatch.setenv("PLX_NUM_GPUS", "8")
    monkeypatch.setenv("PLX_CPU_ONLY", "1")
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    gang = {"version": 1, "kind": "experiment", "run": {"cmd": f"{sys.executable} -c \"print('dp8 up')\""},
            "environment": {"pytorch": {"n_workers": 7}, "resources": {"gpu": 1}}}
    with Polyflow(str(tmp_path), reconcile_s=1.0) as flow:
        g = flow.submit(_group(concurrency=2))
        end = time.time() + 120
        while time.time() < end and not any(x["status"] == "running" for x in flow.store.list_experiments(group_id=g["id"])):
            time.sleep(0.05)
        # the executors hold 2 devices: a DP=8 gang cannot start yet, and waits behind them
        x = flow.submit(gang, project="dp")
        time.sleep(0.5)
        assert flow.store.get_experiment(x["id"])["status"] == "created"
        assert flow.wait("group", g["id"], timeout=300) == "succeeded"
        t_group = time.time()
        assert flow.wait("experiment", x["id"], timeout=60) == "succeeded", flow.logs("experiment", x["id"])[-2000:]
        st = {s["status"]: s["created_at"] for s in flow.store.experiment_statuses(x["id"])}
        started = st.get("scheduled") or st.get("starting")
        assert started is not None and started - t_group < 10.0, (started, t_group)
        jobs = flow.store.experiment_jobs(x["id"])
        assert len(jobs) == 8 and sorted(d for j in jobs for d in j["devices"]) == list(range(8))
        acts = [a["event_type"] for a in flow.store.activity_logs(limit=500)] if hasattr(flow.store, "activity_logs") \
            else []
        assert not acts or "resident_executor.yielded" in acts


def _bo_group(concurrency=2, n_initial=3, n_iterations=2, trial_units=3):
    hp = {"seed": 5, "concurrency": concurrency,
          "bo": {"n_initial_trials": n_initial, "n_iterations": n_iterations,
                 "metric": {"name": "loss", "optimization": "minimize"},
                 "utility_function": {"acquisition_function": "ucb", "kappa": 1.5,
                                      "gaussian_process": {"kernel": "matern", "length_scale": 1.0, "nu": 1.5},
                                      "n_warmup": 100, "n_iter": 3}},
          "matrix": {"lr": {"loguniform": [-9, -3]}, "weight_decay": {"uniform": [0.0, 0.2]}}}
    return {"version": 1, "kind": "group", "project": "rbo", "hptuning": hp,
            "environment": {"resources": {"gpu": 1},
                            "executor": {"kind": "resident", "program": "gpt2_tiny",
                                         "params": {"batch": 2, "seq": 32, "unit_steps": 2,
                                                    "trial_units": trial_units}}}}


def test_polyflow_resident_bo_group_over_gpt2(tmp_path, cpu_pool_env):
    """BO (BASELINE config 4) on resident GPT-2 executors: the initial random batch, then GP batches of
    ``concurrency`` constant-liar suggestions, every trial an experiment with its FSM history and metric, one
    iteration row per BO iteration with the metrics the GP was fitted on, both executors used."""
    from polyaxon_amd.polyflow.scheduler import Polyflow

    with Polyflow(str(tmp_path), reconcile_s=0) as flow:
        r = flow.submit(_bo_group())
        assert flow.wait("group", r["id"], timeout=300) == "succeeded"
        st = flow.store
        xs = st.list_experiments(group_id=r["id"])
        assert len(xs) == 3 + 2 * 2  # n_initial + n_iterations x max(n_suggestions, concurrency)
        for x in xs:
            assert x["status"] == "succeeded"
            assert [s["status"] for s in st.experiment_statuses(x["id"])] == [
                "created", "scheduled", "starting", "running", "succeeded"]
            assert x["declarations"]["units"] == 3 and "lr" in x["declarations"]
            assert x["last_metric"]["loss"] > 0
        its = sorted(st.iterations(r["id"]), key=lambda i: i["data"]["iteration"])
        assert [i["data"]["iteration"] for i in its] == [0, 1, 2]
        assert [len(i["data"]["experiment_ids"]) for i in its] == [3, 2, 2]
        assert all(len(i["data"]["experiments_metrics"]) == len(i["data"]["experiment_ids"]) for i in its)
        # GP suggestions after the random batch: new points, not repeats of the initial ones
        first = {round(x["declarations"]["lr"], 12) for x in xs if x["id"] in its[0]["data"]["experiment_ids"]}
        later = {round(x["declarations"]["lr"], 12) for x in xs if x["id"] in its[1]["data"]["experiment_ids"]}
        assert not (first & later)
        assert {tuple(j["devices"]) for x in xs for j in st.experiment_jobs(x["id"])} == {(0,), (1,)}
        # the GP of every BO iteration ran on an executor (numpy on these CPU executors, the HIP kernels on a GPU),
        # never in the scheduler process, which stays free of device work
        assert [i["data"]["suggest"]["where"].startswith("executor") for i in its[1:]] == [True, True], its
        assert "suggest" not in its[0]["data"]  # the initial batch is random


def test_polyflow_resident_bo_group_on_a_dp2_gang(tmp_path, cpu_pool_env):
    """BASELINE config 4's shape on CPU: a BO group whose trials are DP=2 (``resources.gpu: 2``) runs on ONE resident
    executor spanning a 2-rank gang (gloo; polyflow wires the ranks): every trial trains data-parallel (FlatDDP), the
    ranks follow rank 0's control stream and decide from the cross-rank mean metric, each trial is an experiment with
    its FSM history whose job holds both devices, and the gang stays warm for the whole group."""
    from polyaxon_amd.polyflow.scheduler import Polyflow

    g = _bo_group(concurrency=1, n_initial=2, n_iterations=2)
    g["environment"]["resources"] = {"gpu": 2}
    with Polyflow(str(tmp_path), reconcile_s=0) as flow:
        r = flow.submit(g)
        assert flow.wait("group", r["id"], timeout=300) == "succeeded", flow.store.get_group(r["id"])
        st = flow.store
        xs = st.list_experiments(group_id=r["id"])
        assert len(xs) == 2 + 2 * 1
        for x in xs:
            assert [s["status"] for s in st.experiment_statuses(x["id"])] == [
                "created", "scheduled", "starting", "running", "succeeded"]
            jobs = st.experiment_jobs(x["id"])
            assert len(jobs) == 1 and sorted(jobs[0]["devices"]) == [0, 1]
            assert x["last_metric"]["loss"] > 0
        pool = flow.call(lambda: flow.resident_pool().snapshot())
        assert len(pool) == 1 and sorted(pool[0]["devices"]) == [0, 1]
        wid = pool[0]["wid"]
        info = flow.call(lambda: dict(flow.resident_pool().workers[wid].info))
        assert info.get("dp_world") == 2
    assert flow.alloc.allocations == {}


def test_asha_drops_snapshots_of_configs_that_can_no_longer_be_promoted():
    """once rung 0 is final (nothing pending) the configs below its top floor(n/eta) lose their HBM snapshot;
    rung 1 becomes final when rung 0's whole top set was promoted, and so on; the top sets keep theirs."""
    from polyaxon_amd.polyflow.resident import ResidentWorker, _AshaShard

    class Ex:
        def __init__(self):
            self.snapshots = {}

        def drop(self, key):
            self.snapshots.pop(key, None)

    class Prog:
        executor = Ex()

    w = ResidentWorker("resnet_tiny", device="cpu")
    w.program = Prog()
    sh = _AshaShard(key="s", configs={i: {} for i in range(9)}, pending=[], n_rungs=3, eta=3.0, min_r=1, max_r=9,
                    resource_name="units", resource=None, maximize=False, resume=True, seed=0)
    sh.results = [{i: float(i) for i in range(9)}, {0: 0.5, 1: 0.7, 2: 0.1}, {}]
    sh.order = [list(range(9)), [2, 0, 1], []]
    sh.promoted = [{0, 1, 2}, set(), set()]
    for cid in range(9):
        sh.snap_rung[cid] = 0
        Prog.executor.snapshots[("s", cid)] = object()
    for cid in (0, 1, 2):  # the promoted ones were re-snapshotted at rung 1
        sh.snap_rung[cid] = 1
    w._drop_hopeless_snapshots(sh)
    # rung 0 final: 3..8 are below its top 3 -> dropped; rung 1 final (top 3 of rung 0 promoted): top 1 of 3 = {2}
    assert sorted(sh.snap_rung) == [2]
    assert set(Prog.executor.snapshots) == {("s", 2)}
    # with configs still pending nothing is final: nothing is dropped
    sh2 = _AshaShard(key="t", configs={0: {}, 1: {}}, pending=[1], n_rungs=2, eta=3.0, min_r=1, max_r=3,
                     resource_name="units", resource=None, maximize=False, resume=True, seed=0)
    sh2.results, sh2.order, sh2.promoted = [{0: 1.0}, {}], [[0], []], [set(), set()]
    sh2.snap_rung[0] = 0
    w._drop_hopeless_snapshots(sh2)
    assert sh2.snap_rung == {0: 0}


def test_bench_cpu_config4_trials_are_dp2_gangs():
    """BASELINE config 4 ("each trial DP=2 on RCCL over xGMI") through bench.py: ``--config gpt2_bo --gpus 4
    --trial-gpus 2`` builds two resident DP gangs of two ranks; every trial's job holds 2 devices, every rank launched
    FlatDDP bucket collectives on the framework communicator (the gloo shim here, RCCL on the GPU), the two ranks of
    a gang end with identical weights (the gangs differ), and the scheduler process stays device-free."""
    res = _bench("--config", "gpt2_bo", "--gpus", "4", "--trial-gpus", "2", "--steps", "1", "--warmup", "0",
                 threads="2")
    assert res["config"]["per_trial_world"] == 2 and "dp2" in res["config"]["parallelism"]
    assert res["trials"] == res["trials_succeeded"] > 0
    assert res["trial_devices"] == {"2": res["trials"]}, res["trial_devices"]
    ranks = res["per_rank"]
    assert [r["gang"] for r in ranks] == [0, 0, 1, 1]
    assert all(r["ddp_collectives"] > 0 and r["ddp_on_framework_comm"] for r in ranks), ranks
    assert ranks[0]["weights_fingerprint"] == ranks[1]["weights_fingerprint"]
    assert ranks[2]["weights_fingerprint"] == ranks[3]["weights_fingerprint"]
    assert ranks[0]["weights_fingerprint"] != ranks[2]["weights_fingerprint"]
    assert len(res["executors"]) == 2 and all(len(e["devices"]) == 2 for e in res["executors"])
    fp = res["control_device_footprint"]
    assert not fp["torch_imported"] and not fp["hip_mapped"] and not fp["kfd_open"], fp
