"""Lifecycle FSM golden behaviour (reference constants/*.py) and the tracking store / query DSL."""
import time

import pytest

from polyaxon_amd.fsm import (ExperimentGroupLifeCycle, ExperimentLifeCycle, JobLifeCycle, OperationLifeCycle,
                              PipelineLifeCycle, S)
from polyaxon_amd.store import QueryError, Store


def test_experiment_transitions():
    X = ExperimentLifeCycle
    assert X.can_transition(None, S.CREATED)
    assert not X.can_transition(S.CREATED, S.RUNNING)
    assert X.can_transition(S.CREATED, S.SCHEDULED) and X.can_transition(S.SCHEDULED, S.STARTING)
    assert X.can_transition(S.STARTING, S.RUNNING) and X.can_transition(S.RUNNING, S.SUCCEEDED)
    assert X.can_transition(S.SUCCEEDED, S.RESUMING) and X.can_transition(S.STOPPED, S.RESUMING)
    assert not X.can_transition(S.FAILED, S.RESUMING)
    assert X.can_transition(S.RUNNING, S.STOPPED) and not X.can_transition(S.STOPPED, S.STOPPED)
    assert all(X.can_transition(v, S.UNKNOWN) for v in X.VALUES)
    assert not X.can_transition(S.CREATED, S.SUCCEEDED)
    assert X.is_done(S.FAILED) and X.is_running(S.BUILDING) and X.is_pending(S.RESUMING)


def test_jobs_status_precedence():
    X = ExperimentLifeCycle
    assert X.jobs_status([]) is None
    assert X.jobs_status([S.RUNNING, S.UNKNOWN, S.STOPPED]) == S.UNKNOWN
    assert X.jobs_status([S.RUNNING, S.STOPPED, S.FAILED]) == S.STOPPED
    assert X.jobs_status([S.SUCCEEDED, S.SUCCEEDED]) == S.SUCCEEDED
    assert X.jobs_status([S.SUCCEEDED, S.FAILED]) == S.FAILED
    assert X.jobs_status([S.CREATED, S.RUNNING]) == S.STARTING
    assert X.jobs_status([S.SCHEDULED, S.RUNNING]) == S.RUNNING


def test_other_lifecycles():
    assert JobLifeCycle.can_transition(None, S.BUILDING) and JobLifeCycle.can_transition(S.SCHEDULED, S.BUILDING)
    assert not JobLifeCycle.can_transition(S.SUCCEEDED, S.RUNNING)
    G = ExperimentGroupLifeCycle
    assert G.can_transition(S.STOPPED, S.RUNNING) and not G.can_transition(S.CREATED, S.SUCCEEDED)
    assert PipelineLifeCycle.can_transition(S.STOPPED, S.SKIPPED)
    O = OperationLifeCycle
    assert O.can_transition(S.RETRYING, S.SCHEDULED) and O.can_transition(S.FAILED, S.RETRYING)
    assert O.can_transition(S.SUCCEEDED, S.UPSTREAM_FAILED) and O.failed(S.UPSTREAM_FAILED)


@pytest.fixture(params=["memory", "file"])
def store(request, tmp_path):
    return Store(":memory:" if request.param == "memory" else str(tmp_path / "db.sqlite"))


def test_experiment_lifecycle_in_store(store):
    p = store.create_project("proj")
    x = store.create_experiment(p["id"], {"run": {"cmd": "x"}}, declarations={"lr": 0.1})
    for st in ("scheduled", "starting", "running", "succeeded"):
        assert store.set_experiment_status(x, st)
    assert not store.set_experiment_status(x, "running")
    e = store.get_experiment(x)
    assert e["status"] == "succeeded" and e["started_at"] and e["finished_at"] >= e["started_at"]
    assert [s["status"] for s in store.experiment_statuses(x)] == ["created", "scheduled", "starting", "running",
                                                                   "succeeded"]


def test_metrics_last_metric_merge(store):
    p = store.create_project("proj")
    x = store.create_experiment(p["id"])
    store.add_metrics(x, {"loss": 1.0, "acc": 0.1}, step=1)
    store.add_metrics_batch([(x, {"loss": 0.5}, 2, None), (x, {"loss": 0.25}, 3, None)])
    assert store.get_experiment(x)["last_metric"] == {"loss": 0.25, "acc": 0.1}
    assert [m["values"]["loss"] for m in store.get_metrics(x)] == [1.0, 0.5, 0.25]
    assert store.experiments_metrics([x], "loss") == [(x, 0.25)]


def test_non_finite_metrics_keep_metric_queries_working(store):
    """A diverged trial's NaN / inf loss is stored as valid JSON ("NaN" / "Infinity"): metric sorts and filters over
    its group still run (bare NaN made SQLite reject the document as malformed JSON), the value sorts last in both
    directions and ranks nothing for the search managers."""
    p = store.create_project("proj")
    g = store.create_group(p["id"], {}, {})
    xs = [store.create_experiment(p["id"], group_id=g) for _ in range(4)]
    store.add_metrics(xs[0], {"loss": 0.5}, step=1)
    store.add_metrics(xs[1], {"loss": float("nan")}, step=1)
    store.add_metrics_batch([(xs[2], {"loss": float("inf")}, 1, None), (xs[3], {"loss": 0.25}, 1, None)])
    asc = [x["id"] for x in store.list_experiments(group_id=g, sort="metric.loss")]
    desc = [x["id"] for x in store.list_experiments(group_id=g, sort="-metric.loss")]
    assert asc[:2] == [xs[3], xs[0]] and set(asc[2:]) == {xs[1], xs[2]}
    assert desc[:2] == [xs[0], xs[3]] and set(desc[2:]) == {xs[1], xs[2]}
    assert [x["id"] for x in store.list_experiments(group_id=g, query="metric.loss:<0.4")] == [xs[3]]
    assert store.get_experiment(xs[1])["last_metric"] == {"loss": "NaN"}
    assert store.get_metrics(xs[2])[0]["values"] == {"loss": "Infinity"}
    assert dict(store.experiments_metrics(xs, "loss")) == {xs[0]: 0.5, xs[1]: None, xs[2]: None, xs[3]: 0.25}


def test_query_dsl(store):
    p = store.create_project("proj")
    g = store.create_group(p["id"], {}, {})
    ids = []
    for i in range(6):
        x = store.create_experiment(p["id"], group_id=g if i % 2 else None, declarations={"opt": "sgd" if i < 3 else
                                    "adam", "lr": i / 10}, tags=["a"] if i < 2 else ["b"])
        store.add_metrics(x, {"loss": 1.0 / (i + 1)})
        ids.append(x)
    store.set_experiment_status(ids[0], "scheduled")
    q = lambda s, sort=None: [e["id"] for e in store.list_experiments(query=s, sort=sort)]  # noqa: E731
    assert q("metric.loss:<0.3") == ids[3:]
    assert q("metric.loss:~<0.3") == ids[:3]
    assert q("metric.loss:>=0.25, metric.loss:<=0.5") == ids[1:4]
    assert q("declarations.opt:adam") == ids[3:]
    assert q("declarations.opt:~adam") == ids[:3]
    assert q("status:created|scheduled") == ids
    assert q("status:~created") == [ids[0]]
    assert q("tags:a") == ids[:2] and q("tags:~a") == ids[2:]
    assert q("independent:true") == ids[0::2]
    assert q(f"group:{g}") == ids[1::2]
    assert q("project:proj") == ids and q("project:other") == []
    assert q("", sort="-metric.loss") == ids
    assert q("", sort="metric.loss") == list(reversed(ids))
    today = time.strftime("%Y-%m-%d", time.gmtime())
    assert q(f"created_at:{today}") == ids
    assert q("created_at:2001-01-01 .. 2002-01-01") == []
    with pytest.raises(QueryError):
        q("bogus:1")
    with pytest.raises(QueryError):
        q("metric.loss:abc")


def test_groups_iterations_jobs_kv(store):
    p = store.create_project("proj")
    g = store.create_group(p["id"], {"a": 1}, {"matrix": {}}, search_algorithm="grid_search", concurrency=2)
    assert store.set_group_status(g, "running") and store.set_group_status(g, "succeeded")
    it = store.create_iteration(g, {"iteration": 0})
    store.update_iteration(it, {"iteration": 0, "experiment_ids": [1]})
    assert store.last_iteration(g)["data"]["experiment_ids"] == [1]
    j = store.create_job("build", p["id"], {"build": {"image": "x"}}, image_hash="abc")
    assert store.set_job_status(j, "running") and store.set_job_status(j, "succeeded")
    assert store.last_build_for_hash("abc", 3600)["id"] == j
    store.kv_set("k", {"v": 1}, ttl=100)
    assert store.kv_get("k") == {"v": 1}
    store.kv_set("t", 1, ttl=-1)
    assert store.kv_get("t") is None
