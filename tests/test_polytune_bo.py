"""Bayesian optimisation: search space (reference test_search_managers.py:631-1010), GP math parity with
sklearn, and the BO manager on every backend available on CPU."""
import numpy as np
import pytest

from polyaxon_amd.polytune.bo import (BOIterationConfig, BOOptimizer, BOSearchManager, SearchSpace, acquisition_np,
                                      fit_gp, kernel_np, predict_np)
from polyaxon_amd.spec.hptuning import HPTuningConfig


def _cfg1():
    return HPTuningConfig.from_dict({
        "concurrency": 2,
        "bo": {"n_iterations": 5, "n_initial_trials": 5, "metric": {"name": "loss", "optimization": "minimize"},
               "utility_function": {"acquisition_function": "ucb", "kappa": 1.2,
                                    "gaussian_process": {"kernel": "matern", "length_scale": 1.0, "nu": 1.9,
                                                         "n_restarts_optimizer": 0}}},
        "matrix": {"feature1": {"values": [1, 2, 3]}, "feature2": {"linspace": [1, 2, 5]},
                   "feature3": {"range": [1, 5, 1]}}})


def _cfg2():
    return HPTuningConfig.from_dict({
        "concurrency": 2,
        "bo": {"n_iterations": 4, "n_initial_trials": 4, "metric": {"name": "accuracy", "optimization": "maximize"},
               "utility_function": {"acquisition_function": "ei", "eps": 1.2,
                                    "gaussian_process": {"kernel": "matern", "length_scale": 1.0, "nu": 1.9,
                                                         "n_restarts_optimizer": 0}}},
        "matrix": {"feature1": {"values": [1, 2, 3, 4, 5]}, "feature2": {"linspace": [1, 5, 5]},
                   "feature3": {"range": [1, 6, 1]}, "feature4": {"uniform": [1, 5]},
                   "feature5": {"values": ["a", "b", "c"]}}})


def test_initial_suggestions():
    assert len(BOSearchManager(_cfg1()).get_suggestions()) == 5
    assert len(BOSearchManager(_cfg2()).get_suggestions()) == 4


def test_space_bounds_and_features():
    s1 = SearchSpace(_cfg1())
    assert s1.dim == 3 and len(s1.bounds) == 3 and len(s1.discrete_features) == 3 and not s1.categorical_features
    b = dict(zip(s1.features, s1.bounds.tolist()))
    assert b == {"feature1": [1, 3], "feature2": [1, 2], "feature3": [1, 4]}
    np.testing.assert_allclose(s1.discrete_features["feature2"]["values"], [1., 1.25, 1.5, 1.75, 2.])
    s2 = SearchSpace(_cfg2())
    assert s2.dim == 7 and len(s2.bounds) == 7 and len(s2.discrete_features) == 3
    assert len(s2.categorical_features) == 1 and len(s2.features) == 5
    assert s2.categorical_features["feature5"]["number"] == 3


def test_space_parse_and_snap():
    s2 = SearchSpace(_cfg2())
    configs = [{"feature1": 1, "feature2": 1, "feature3": 1, "feature4": 1, "feature5": "a"},
               {"feature1": 2, "feature2": 1.2, "feature3": 2, "feature4": 4, "feature5": "c"}]
    s2.add_observations(configs, [1, 2])
    np.testing.assert_array_equal(s2.x, [[1, 1, 1, 1, 1, 0, 0], [2, 1.2, 2, 4, 0, 0, 1]])
    np.testing.assert_array_equal(s2.y, [1, 2])  # maximize: not negated
    s1 = SearchSpace(_cfg1())
    s1.add_observations([{"feature1": 1, "feature2": 1, "feature3": 1}], [3])
    assert s1.y.tolist() == [-3]  # minimize: negated
    sug = s2.get_suggestion(np.array([1.2, 1.1, 2.9, 3.3, 0.1, 0.9, 0.2]))
    assert sug == {"feature1": 1, "feature2": 1.0, "feature3": 3, "feature4": 3.3, "feature5": "b"}


@pytest.mark.parametrize("kernel,nu", [("rbf", 1.5), ("matern", 0.5), ("matern", 1.5), ("matern", 2.5),
                                       ("matern", 1.9)])
def test_gp_matches_sklearn_posterior(kernel, nu):
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import RBF, Matern

    rng = np.random.RandomState(0)
    X = rng.uniform(0, 3, size=(20, 3))
    y = np.sin(X).sum(1)
    gp = fit_gp(X, y, kernel=kernel, nu=nu, length_scale=1.0, optimize=False)
    k = RBF(1.0) if kernel == "rbf" else Matern(1.0, nu=nu)
    sk = GaussianProcessRegressor(kernel=k, optimizer=None).fit(X, y)
    Xc = rng.uniform(0, 3, size=(50, 3))
    m1, s1 = predict_np(gp, Xc)
    m2, s2 = sk.predict(Xc, return_std=True)
    np.testing.assert_allclose(m1, m2, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(s1, s2, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(kernel_np(X, X, gp.kind, 1.0, nu), k(X), rtol=1e-6, atol=1e-8)


def test_lml_length_scale_fit_close_to_sklearn():
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import Matern

    rng = np.random.RandomState(1)
    X = rng.uniform(0, 10, size=(30, 2))
    y = np.sin(X[:, 0] / 2) + np.cos(X[:, 1] / 3)
    gp = fit_gp(X, y, kernel="matern", nu=2.5, length_scale=1.0)
    sk = GaussianProcessRegressor(kernel=Matern(1.0, nu=2.5), random_state=0).fit(X, y)
    assert gp.lml >= sk.log_marginal_likelihood_value_ - 1e-3
    assert gp.ls == pytest.approx(sk.kernel_.length_scale, rel=0.05)


def test_acquisitions():
    mean, std = np.array([0.0, 1.0, 2.0]), np.array([1.0, 0.5, 0.0])
    np.testing.assert_allclose(acquisition_np(mean, std, "ucb", 0, 2.0, 0), [2.0, 2.0, 2.0])
    ei = acquisition_np(mean, std, "ei", 1.0, 0, 0.0)
    assert ei[2] == pytest.approx(1.0) and ei[0] > 0
    poi = acquisition_np(mean, std, "poi", 1.0, 0, 0.0)
    assert poi[1] == pytest.approx(0.5)


@pytest.mark.parametrize("backend", ["reference", "numpy"])
def test_optimizer_concrete_example(backend):
    """Suggestions improve on a known 1-D objective (reference test_concrete_example shape)."""
    cfg = HPTuningConfig.from_dict({
        "seed": 3,
        "bo": {"n_iterations": 3, "n_initial_trials": 3, "metric": {"name": "loss", "optimization": "minimize"},
               "utility_function": {"acquisition_function": "ucb", "kappa": 1.0,
                                    "gaussian_process": {"kernel": "matern", "length_scale": 1.0, "nu": 1.9}}},
        "matrix": {"x": {"uniform": [-3, 3]}, "y": {"values": [1, 2, 3]}}})
    opt = BOOptimizer(cfg, backend=backend)
    configs = [{"x": -2.0, "y": 1}, {"x": 0.5, "y": 2}, {"x": 2.5, "y": 3}]
    metrics = [(c["x"] - 0.3) ** 2 + 0.1 * c["y"] for c in configs]
    opt.add_observations(configs, metrics)
    s = opt.get_suggestion()
    assert set(s) == {"x", "y"} and -3 <= s["x"] <= 3 and s["y"] in (1, 2, 3)


def test_manager_iteration_uses_combined_observations():
    m = BOSearchManager(_cfg1(), backend="numpy")
    it = BOIterationConfig(iteration=2, old_experiment_ids=[1, 2, 3],
                           old_experiments_configs=[(1, {"feature1": 1, "feature2": 1, "feature3": 1}),
                                                    (2, {"feature1": 2, "feature2": 1.25, "feature3": 2}),
                                                    (3, {"feature1": 3, "feature2": 1.5, "feature3": 3})],
                           old_experiments_metrics=[(1, 1), (2, 2), (3, 3)], experiment_ids=[4],
                           experiments_configs=[(4, {"feature1": 2, "feature2": 1.5, "feature3": 4})],
                           experiments_metrics=[(4, 4)])
    s = m.get_suggestions(it)
    assert len(s) == 1 and s[0]["feature1"] in (1, 2, 3) and s[0]["feature3"] in (1, 2, 3, 4)
    assert it.combined_experiment_ids == [1, 2, 3, 4] and len(it.old_experiment_ids) == 3  # no aliasing


def test_batch_suggestions_constant_liar():
    cfg = _cfg1()
    cfg.bo.n_suggestions = 3
    opt = BOOptimizer(cfg, backend="numpy")
    opt.add_observations([{"feature1": 1, "feature2": 1.0, "feature3": 1},
                          {"feature1": 3, "feature2": 2.0, "feature3": 4}], [1.0, 0.2])
    assert len(opt.get_suggestions(3)) == 3


def test_unit_space_maps_log_dimensions_and_roundtrips():
    """bo.space: unit -- log-distributed dimensions in log space, every continuous one scaled to [0, 1]: a config
    maps into the unit box and back, and a BO search over a learning rate spanning decades finds the optimum of a
    bowl in log-lr (the raw space's bounds are dominated by the large learning rates)."""
    import math

    import numpy as np

    from polyaxon_amd.polytune.bo import BOSearchManager, BOIterationConfig, SearchSpace
    from polyaxon_amd.spec.hptuning import HPTuningConfig

    def cfg(space):
        return HPTuningConfig.from_dict({
            "seed": 3, "matrix": {"lr": {"loguniform": [math.log(1e-5), math.log(3e-3)]},
                                  "wd": {"uniform": [0.0, 0.2]}},
            "bo": {"n_initial_trials": 4, "n_iterations": 6, "space": space,
                   "metric": {"name": "loss", "optimization": "minimize"},
                   "utility_function": {"acquisition_function": "ucb", "kappa": 1.0,
                                        "gaussian_process": {"kernel": "matern", "length_scale": 0.3, "nu": 2.5},
                                        "n_warmup": 2000, "n_iter": 4}}})

    sp = SearchSpace(cfg("unit"))
    x = sp.parse_x([{"lr": 1e-4, "wd": 0.1}])[0]
    assert np.all((x >= 0) & (x <= 1)) and abs(sp.get_suggestion(x)["lr"] - 1e-4) < 1e-12
    assert sp.to_dict() if hasattr(sp, "to_dict") else True

    def loss(p):
        return (math.log10(p["lr"]) + 4.0) ** 2 + 0.1 * p["wd"]

    best = {}
    for space in ("raw", "unit"):
        m = BOSearchManager(cfg(space), backend="numpy")
        configs = list(enumerate(m.get_suggestions()))
        metrics = [(i, loss(c)) for i, c in configs]
        for it in range(1, 4):
            sugg = m.get_suggestions(BOIterationConfig(iteration=it, old_experiments_configs=configs,
                                                       old_experiments_metrics=metrics), n=2)
            for c in sugg:
                i = len(configs)
                assert 1e-5 * 0.999 <= c["lr"] <= 3e-3 * 1.001
                configs.append((i, c))
                metrics.append((i, loss(c)))
        best[space] = min(v for _, v in metrics)
    assert best["unit"] < 0.05 and best["unit"] <= best["raw"], best
