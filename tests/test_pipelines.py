"""Pipelines DAG engine: DAG helpers, the full trigger-policy matrix, and scheduling behaviour (concurrency,
timeouts, exponential retry backoff, no-op nodes, stop).

DAG cases follow the reference's tests/test_pipelines/test_dags.py (pipelines/dags.py:6-76); trigger and
retry semantics follow db/models/pipelines.py:233-258,502-523 and constants/pipelines.py:4-97."""
import time

import pytest

from polyaxon_amd.fsm import OperationLifeCycle
from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.pipelines import (get_dag, get_independent_nodes, get_orphan_nodes, has_dependencies,
                                             sort_topologically, trigger_satisfied)
from polyaxon_amd.polyflow.scheduler import Polyflow

DAG1 = {1: [2, 3, 4], 2: [3], 5: [3], 4: [], 6: []}
DAG2 = {1: [2, 3, 4], 2: [3], 3: [], 5: [], 6: [7, 8], 7: [10], 9: [10, 11]}
DAG3 = {1: [2, 3, 4, 5], 2: [6, 7], 3: [8], 4: [9], 5: [10], 6: [11], 7: [], 8: [12, 13], 9: [14], 10: [15],
        11: [], 12: []}
DAG4 = {0: [1, 2], 1: [2, 3], 2: [3, 5], 3: [4], 5: [], 7: [6]}
CYCLE1 = {1: [2], 2: [3], 3: [4], 4: [1]}
CYCLE2 = {1: [2, 3, 4, 5], 2: [3, 1], 5: [2], 6: [7, 8], 7: [10], 9: [10, 11]}


def test_orphan_and_independent_nodes():
    assert get_orphan_nodes(DAG1) == {6}
    assert get_orphan_nodes(DAG2) == {5}
    assert get_orphan_nodes(DAG3) == set() and get_orphan_nodes(DAG4) == set()
    assert get_orphan_nodes(CYCLE1) == set() and get_orphan_nodes(CYCLE2) == set()
    assert get_independent_nodes(DAG1) == {1, 5, 6}
    assert get_independent_nodes(DAG2) == {1, 5, 6, 9}
    assert get_independent_nodes(DAG3) == {1}
    assert get_independent_nodes(DAG4) == {0, 7}
    assert get_independent_nodes(CYCLE1) == set()
    assert get_independent_nodes(CYCLE2) == {6, 9}


def test_has_dependencies():
    assert has_dependencies(3, DAG1) and not has_dependencies(1, DAG1)
    assert has_dependencies(10, DAG2) and not has_dependencies(9, DAG2)
    assert all(has_dependencies(n, CYCLE1) for n in CYCLE1)


def test_get_dag_from_objects():
    class Op:
        def __init__(self, i, down):
            self.id, self.down = i, down

    ops = [Op(1, [2]), Op(2, []), Op(3, [2])]
    dag, by_id = get_dag(ops, lambda o: o.down)
    assert dag == {1: {2}, 2: set(), 3: {2}} and by_id[3] is ops[2]
    assert sort_topologically(dag) == [1, 3, 2]


def test_topological_sort():
    order = sort_topologically({k: set(v) for k, v in DAG4.items()})
    pos = {n: i for i, n in enumerate(order)}
    for n, ds in DAG4.items():
        for d in ds:
            if d in pos:
                assert pos[n] < pos[d]
    full3 = {k: set(v) for k, v in DAG3.items()}
    for n in range(13, 16):
        full3[n] = set()
    order3 = sort_topologically(full3)
    assert order3[0] == 1 and len(order3) == 15
    for cyc in (CYCLE1, CYCLE2):
        with pytest.raises(ValueError):
            sort_topologically({k: set(v) for k, v in cyc.items()})


S, F, ST, R, UF, SK = "succeeded", "failed", "stopped", "running", "upstream_failed", "skipped"


@pytest.mark.parametrize("policy,ups,expected", [
    ("all_succeeded", [S, S], True), ("all_succeeded", [S, R], None), ("all_succeeded", [S, F], False),
    ("all_succeeded", [S, SK], False), ("all_succeeded", [], True),
    ("all_failed", [F, F], True), ("all_failed", [F, UF], True), ("all_failed", [F, S], False),
    ("all_failed", [F, R], None),
    ("all_done", [S, F], True), ("all_done", [ST, SK], True), ("all_done", [S, R], None),
    ("one_succeeded", [S, R], True), ("one_succeeded", [F, R], None), ("one_succeeded", [F, ST], False),
    ("one_failed", [F, R], True), ("one_failed", [S, R], None), ("one_failed", [S, S], False),
    ("one_failed", [UF, R], True),
    ("one_done", [S, R], True), ("one_done", [F, R], True), ("one_done", [R, R], None),
])
def test_trigger_policy_matrix(policy, ups, expected):
    assert trigger_satisfied(policy, ups) is expected


def test_unknown_trigger_policy():
    with pytest.raises(ValueError):
        trigger_satisfied("sometimes", [S])


def test_operation_lifecycle_done_states():
    for s in (S, F, ST, UF, SK):
        assert OperationLifeCycle.is_done(s)
    assert not OperationLifeCycle.is_done(R)


def _job(cmd):
    return {"version": 1, "kind": "job", "run": {"cmd": cmd}}


@pytest.fixture
def flow(tmp_path):
    f = Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0), Device(1)]), stop_grace_s=1.0).start()
    yield f
    f.shutdown()


def test_concurrency_one_serialises_independent_ops(flow, tmp_path):
    log = tmp_path / "spans"
    cmd = f"echo start $(date +%s.%N) >> {log}; sleep 0.3; echo end $(date +%s.%N) >> {log}"
    spec = {"version": 1, "kind": "pipeline", "concurrency": 1,
            "ops": [{"name": f"op{i}", "template": _job(cmd)} for i in range(3)]}
    r = flow.submit(spec)
    assert flow.wait("pipeline_run", r["run_id"], timeout=60) == "finished"
    events = [(float(t), kind) for kind, t in (line.split() for line in log.read_text().splitlines())]
    depth, peak = 0, 0
    for _, kind in sorted(events):
        depth += 1 if kind == "start" else -1
        peak = max(peak, depth)
    assert peak == 1 and len(events) == 6


def test_timeout_stops_operation_and_downstream_is_upstream_failed(flow):
    spec = {"version": 1, "kind": "pipeline", "ops": [
        {"name": "slow", "timeout": 0.5, "template": _job("sleep 30")},
        {"name": "next", "upstream": ["slow"], "template": _job("true")},
        {"name": "marker", "upstream": ["slow"], "trigger": "all_done"}]}  # no template: a no-op node
    t0 = time.time()
    r = flow.submit(spec)
    assert flow.wait("pipeline_run", r["run_id"], timeout=60) == "finished"
    assert time.time() - t0 < 20
    ops = {o["name"]: o for o in flow.store.operation_runs(r["run_id"])}
    assert ops["slow"]["status"] == "stopped"
    assert ops["next"]["status"] == "upstream_failed"
    assert ops["marker"]["status"] == "succeeded"


def test_exponential_backoff_retries(flow, tmp_path):
    stamps = tmp_path / "stamps"
    cmd = f"date +%s.%N >> {stamps}; exit 1"
    spec = {"version": 1, "kind": "pipeline", "ops": [
        {"name": "bad", "max_retries": 3, "retry_delay": 0.2, "retry_exponential_backoff": True,
         "max_retry_delay": 0.5, "template": _job(cmd)}]}
    r = flow.submit(spec)
    assert flow.wait("pipeline_run", r["run_id"], timeout=60) == "finished"
    op = flow.store.operation_runs(r["run_id"])[0]
    assert op["status"] == "failed" and op["retries"] == 3
    t = [float(x) for x in stamps.read_text().split()]
    gaps = [b - a for a, b in zip(t, t[1:])]
    assert len(gaps) == 3
    # delays 0.2, 0.4, then capped at 0.5 (plus process start-up)
    assert gaps[0] >= 0.18 and gaps[1] >= 0.38 and gaps[2] >= 0.48
    assert gaps[2] < gaps[1] + 0.5
