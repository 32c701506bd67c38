"""Hyperband golden vectors (reference tests/test_experiment_groups/test_search_managers.py:184-530)."""
import pytest

from polyaxon_amd.polytune.managers import (HyperbandIterationConfig, HyperbandSearchManager,
                                            get_search_algorithm_manager)
from polyaxon_amd.spec.hptuning import HPTuningConfig


def _mgr(max_iter, rtype, n_features=3, name="steps"):
    matrix = {"feature1": {"values": [1, 2, 3]}, "feature2": {"linspace": [1, 2, 5]},
              "feature3": {"range": [1, 5, 1]}}
    if n_features == 4:
        matrix["feature4"] = {"range": [1, 5, 1]}
    return HyperbandSearchManager(HPTuningConfig.from_dict({
        "concurrency": 2,
        "hyperband": {"max_iter": max_iter, "eta": 3, "resource": {"name": name, "type": rtype},
                      "resume": False, "metric": {"name": "loss", "optimization": "minimize"}},
        "matrix": matrix}))


@pytest.fixture
def m1():
    return _mgr(10, "float")


@pytest.fixture
def m2():
    return _mgr(81, "int", 4, name="size")


def test_properties(m1, m2):
    assert (m1.max_iter, m1.eta, m1.s_max, m1.B) == (10, 3, 2, 30)
    assert (m2.max_iter, m2.eta, m2.s_max, m2.B) == (81, 3, 4, 405)


def test_brackets_and_configs(m1, m2):
    assert [m1.get_bracket(i) for i in range(3)] == [2, 1, 0]
    assert [m2.get_bracket(i) for i in range(5)] == [4, 3, 2, 1, 0]
    assert [m1.get_n_configs(b) for b in (2, 1, 0)] == [9, 5, 3]
    assert [m2.get_n_configs(b) for b in (4, 3, 2, 1, 0)] == [81, 34, 15, 8, 5]


@pytest.mark.parametrize("n,expected", [(9, [3, 1, 0]), (5, [1, 0]), (3, [1])])
def test_keep_m1(m1, n, expected):
    assert [m1.get_n_config_to_keep(n, i) for i in range(len(expected))] == expected


@pytest.mark.parametrize("n,expected", [(81, [27, 9, 3, 1, 0]), (34, [11, 3, 1, 0]), (15, [5, 1, 0]), (8, [2, 0]),
                                        (5, [1])])
def test_keep_m2(m2, n, expected):
    assert [m2.get_n_config_to_keep(n, i) for i in range(len(expected))] == expected


def test_keep_for_iteration(m1, m2):
    assert [m1.get_n_config_to_keep_for_iteration(0, i) for i in range(3)] == [3, 1, 0]
    assert [m1.get_n_config_to_keep_for_iteration(1, i) for i in range(2)] == [1, 0]
    assert m1.get_n_config_to_keep_for_iteration(2, 0) == 1
    assert [m2.get_n_config_to_keep_for_iteration(0, i) for i in range(5)] == [27, 9, 3, 1, 0]
    assert [m2.get_n_config_to_keep_for_iteration(3, i) for i in range(2)] == [2, 0]


def test_resources(m1, m2):
    for b, v in ((2, 1.11), (1, 3.33), (0, 10)):
        assert m1.get_resources(b) == pytest.approx(v, abs=0.02)
    for it, v in enumerate((1, 3, 9, 27, 81)):
        assert m2.get_resources_for_iteration(it) == pytest.approx(v, abs=0.02)
    for i, v in enumerate((1.11, 3.33, 9.99)):
        assert m1.get_n_resources_for_iteration(0, i) == pytest.approx(v, abs=0.02)
    for i, v in enumerate((3, 9, 27, 81)):
        assert m2.get_n_resources_for_iteration(1, i) == pytest.approx(v, abs=0.02)


def test_should_reschedule_and_reduce(m1):
    resched = {(0, 0): False, (0, 1): False, (0, 2): True, (0, 3): True, (1, 0): False, (1, 1): True,
               (1, 2): True, (2, 0): False, (2, 1): False, (5, 0): False}
    reduce = {(0, 0): True, (0, 1): True, (0, 2): False, (0, 3): False, (1, 0): True, (1, 1): False,
              (1, 2): False, (2, 0): True, (2, 1): False, (5, 0): False}
    for (it, bi), v in resched.items():
        assert m1.should_reschedule(it, bi) is v, (it, bi)
    for (it, bi), v in reduce.items():
        assert m1.should_reduce_configs(it, bi) is v, (it, bi)


def test_get_suggestions(m1, m2):
    with pytest.raises(ValueError):
        m1.get_suggestions()
    with pytest.raises(ValueError):
        m1.get_suggestions(1)
    s = m1.get_suggestions(HyperbandIterationConfig(iteration=0, bracket_iteration=0))
    assert len(s) == 9
    assert all(x["steps"] == pytest.approx(1.11, abs=0.02) for x in s)
    s = m2.get_suggestions(HyperbandIterationConfig(iteration=2, bracket_iteration=1))
    assert len(s) == 15 and all(x["size"] == 27 for x in s)
    assert len({tuple(sorted(x.items())) for x in s}) == 15  # de-duplicated


def test_iteration_state_machine_visits_reference_schedule(m1):
    seq, it = [], m1.next_iteration(None)
    while True:
        seq.append((it.iteration, it.bracket_iteration))
        if m1.is_done(it):
            break
        it = m1.next_iteration(it)
    assert seq == [(0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (2, 0), (2, 1)]


def test_reduce_keeps_top(m1):
    it = HyperbandIterationConfig(iteration=0, bracket_iteration=0,
                                  experiments_metrics=[(i, v) for i, v in enumerate([5, 1, 4, 2, 9, 3, 8, 7, 6])])
    assert m1.reduce(it) == [1, 3, 5]


def test_factory_dispatch(m1):
    assert isinstance(get_search_algorithm_manager(m1.hptuning_config), HyperbandSearchManager)
