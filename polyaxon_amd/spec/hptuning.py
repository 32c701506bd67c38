"""``hptuning`` section schema: seed, concurrency, matrix, search algorithm, early stopping.

Contract re-created from docs/templates/polyaxonfile_specification/sections.md:41-290 and the attribute
accesses of the reference search managers (polyaxon/hpsearch/search_managers/*.py) — the schema package
itself (polyaxon_schemas.hptuning) is not in the reference tree.  Grid search is the default algorithm
(sections.md:209-220; polyaxon/signals/experiment_groups.py:40-41).

New algorithm beyond the reference: ``asha`` (asynchronous successive halving, no rung barrier), and
``bo.n_suggestions`` (> 1 = batch BO via constant-liar; reference behaviour is 1 — SURVEY.md §3.3).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from polyaxon_amd.spec.matrix import MatrixConfig, MatrixValidationError, parse_matrix


class SearchAlgorithms:
    GRID = "grid_search"
    RANDOM = "random_search"
    HYPERBAND = "hyperband"
    BO = "bo"
    ASHA = "asha"
    VALUES = (GRID, RANDOM, HYPERBAND, BO, ASHA)


class Optimization:
    MAXIMIZE = "maximize"
    MINIMIZE = "minimize"
    VALUES = (MAXIMIZE, MINIMIZE)

    @staticmethod
    def maximize(value: str) -> bool:
        return value == Optimization.MAXIMIZE

    @staticmethod
    def minimize(value: str) -> bool:
        return value == Optimization.MINIMIZE


def _check_opt(v: str) -> str:
    if v not in Optimization.VALUES:
        raise MatrixValidationError(f"optimization must be one of {Optimization.VALUES}, got {v!r}")
    return v


@dataclass
class SearchMetricConfig:
    name: str
    optimization: str = Optimization.MINIMIZE

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "SearchMetricConfig":
        return cls(name=d["name"], optimization=_check_opt(d.get("optimization", Optimization.MINIMIZE)))

    def to_dict(self):
        return {"name": self.name, "optimization": self.optimization}


@dataclass
class EarlyStoppingMetricConfig:
    metric: str
    value: float
    optimization: str = Optimization.MAXIMIZE

    @classmethod
    def from_dict(cls, d):
        return cls(metric=d["metric"], value=float(d["value"]),
                   optimization=_check_opt(d.get("optimization", Optimization.MAXIMIZE)))

    def to_dict(self):
        return {"metric": self.metric, "value": self.value, "optimization": self.optimization}


@dataclass
class ResourceConfig:
    name: str
    type: str = "float"

    @classmethod
    def from_dict(cls, d):
        t = d.get("type", "float")
        if t not in ("int", "float"):
            raise MatrixValidationError(f"resource type must be int or float, got {t!r}")
        return cls(name=d["name"], type=t)

    def cast_value(self, value):
        return int(value) if self.type == "int" else float(value)

    def to_dict(self):
        return {"name": self.name, "type": self.type}


@dataclass
class GridSearchConfig:
    n_experiments: Optional[int] = None

    @classmethod
    def from_dict(cls, d):
        return cls(n_experiments=(d or {}).get("n_experiments"))

    def to_dict(self):
        return {"n_experiments": self.n_experiments}


@dataclass
class RandomSearchConfig:
    n_experiments: int
    # "numpy": the reference's sequential RandomState stream (default, parity); "device": the counter-based
    # Philox stream of polytune/sampler.py (one kernel launch for any n, same suggestions on any device)
    sampler: str = "numpy"

    @classmethod
    def from_dict(cls, d):
        if not d or not d.get("n_experiments"):
            raise MatrixValidationError("random_search requires `n_experiments`")
        sampler = str(d.get("sampler", "numpy"))
        if sampler not in ("numpy", "device"):
            raise MatrixValidationError("random_search.sampler must be `numpy` or `device`")
        return cls(n_experiments=int(d["n_experiments"]), sampler=sampler)

    def to_dict(self):
        out = {"n_experiments": self.n_experiments}
        if self.sampler != "numpy":
            out["sampler"] = self.sampler
        return out


@dataclass
class HyperbandConfig:
    max_iter: int
    eta: float
    resource: ResourceConfig
    metric: SearchMetricConfig
    resume: bool = False

    @classmethod
    def from_dict(cls, d):
        return cls(max_iter=int(d["max_iter"]), eta=d.get("eta", 3), resource=ResourceConfig.from_dict(d["resource"]),
                   metric=SearchMetricConfig.from_dict(d["metric"]), resume=bool(d.get("resume", False)))

    def to_dict(self):
        return {"max_iter": self.max_iter, "eta": self.eta, "resource": self.resource.to_dict(),
                "metric": self.metric.to_dict(), "resume": self.resume}


@dataclass
class AshaConfig:
    """Asynchronous successive halving: promote as soon as a config is in the top 1/eta of its rung."""
    min_resource: float
    max_resource: float
    eta: float
    resource: ResourceConfig
    metric: SearchMetricConfig
    n_experiments: int
    resume: bool = True

    @classmethod
    def from_dict(cls, d):
        return cls(min_resource=float(d.get("min_resource", 1)), max_resource=float(d["max_resource"]),
                   eta=float(d.get("eta", 3)), resource=ResourceConfig.from_dict(d["resource"]),
                   metric=SearchMetricConfig.from_dict(d["metric"]), n_experiments=int(d["n_experiments"]),
                   resume=bool(d.get("resume", True)))

    def to_dict(self):
        return {"min_resource": self.min_resource, "max_resource": self.max_resource, "eta": self.eta,
                "resource": self.resource.to_dict(), "metric": self.metric.to_dict(),
                "n_experiments": self.n_experiments, "resume": self.resume}


@dataclass
class GaussianProcessConfig:
    kernel: str = "matern"
    length_scale: float = 1.0
    nu: float = 1.5
    n_restarts_optimizer: int = 0

    @classmethod
    def from_dict(cls, d):
        d = d or {}
        k = d.get("kernel", "matern")
        if k not in ("matern", "rbf"):
            raise MatrixValidationError(f"gaussian_process.kernel must be matern or rbf, got {k!r}")
        return cls(kernel=k, length_scale=float(d.get("length_scale", 1.0)), nu=float(d.get("nu", 1.5)),
                   n_restarts_optimizer=int(d.get("n_restarts_optimizer", 0)))

    def to_dict(self):
        return dict(kernel=self.kernel, length_scale=self.length_scale, nu=self.nu,
                    n_restarts_optimizer=self.n_restarts_optimizer)


@dataclass
class UtilityFunctionConfig:
    acquisition_function: str = "ucb"
    gaussian_process: GaussianProcessConfig = field(default_factory=GaussianProcessConfig)
    kappa: Optional[float] = None
    eps: Optional[float] = None
    n_warmup: Optional[int] = None
    n_iter: Optional[int] = None

    @classmethod
    def from_dict(cls, d):
        d = d or {}
        acq = d.get("acquisition_function", "ucb")
        if acq not in ("ucb", "ei", "poi"):
            raise MatrixValidationError(f"acquisition_function must be ucb, ei or poi, got {acq!r}")
        if acq == "ucb" and d.get("kappa") is None:
            raise MatrixValidationError("ucb requires `kappa`")
        if acq in ("ei", "poi") and d.get("eps") is None:
            raise MatrixValidationError(f"{acq} requires `eps`")
        return cls(acquisition_function=acq, gaussian_process=GaussianProcessConfig.from_dict(d.get("gaussian_process")),
                   kappa=d.get("kappa"), eps=d.get("eps"), n_warmup=d.get("n_warmup"), n_iter=d.get("n_iter"))

    def to_dict(self):
        return dict(acquisition_function=self.acquisition_function, gaussian_process=self.gaussian_process.to_dict(),
                    kappa=self.kappa, eps=self.eps, n_warmup=self.n_warmup, n_iter=self.n_iter)


@dataclass
class BOConfig:
    n_iterations: int
    n_initial_trials: int
    metric: SearchMetricConfig
    utility_function: UtilityFunctionConfig
    n_suggestions: int = 1
    # the GP's input space: "raw" (the reference's: every continuous dimension in its own units), or "unit" (our
    # addition): log-distributed dimensions (loguniform, qloguniform, lognormal, qlognormal) in log space, then every
    # continuous / discrete dimension min-max scaled to [0, 1], so one isotropic length scale fits a learning rate
    # over decades beside a beta2 over [0.9, 0.999]
    space: str = "raw"

    @classmethod
    def from_dict(cls, d):
        space = d.get("space", "raw")
        if space not in ("raw", "unit"):
            raise MatrixValidationError(f"bo.space must be raw or unit, got {space!r}")
        return cls(n_iterations=int(d["n_iterations"]), n_initial_trials=int(d["n_initial_trials"]),
                   metric=SearchMetricConfig.from_dict(d["metric"]),
                   utility_function=UtilityFunctionConfig.from_dict(d.get("utility_function")),
                   n_suggestions=int(d.get("n_suggestions", 1)), space=space)

    def to_dict(self):
        out = dict(n_iterations=self.n_iterations, n_initial_trials=self.n_initial_trials,
                   metric=self.metric.to_dict(), utility_function=self.utility_function.to_dict(),
                   n_suggestions=self.n_suggestions)
        if self.space != "raw":
            out["space"] = self.space
        return out


@dataclass
class HPTuningConfig:
    matrix: Dict[str, MatrixConfig]
    seed: Optional[int] = None
    concurrency: int = 1
    grid_search: Optional[GridSearchConfig] = None
    random_search: Optional[RandomSearchConfig] = None
    hyperband: Optional[HyperbandConfig] = None
    bo: Optional[BOConfig] = None
    asha: Optional[AshaConfig] = None
    early_stopping: List[EarlyStoppingMetricConfig] = field(default_factory=list)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "HPTuningConfig":
        if not isinstance(d, dict):
            raise MatrixValidationError("hptuning must be a mapping")
        algos = [a for a in SearchAlgorithms.VALUES if d.get(a) is not None]
        if len(algos) > 1:
            raise MatrixValidationError(f"hptuning defines more than one search algorithm: {algos}")
        matrix = parse_matrix(d.get("matrix") or {})
        cfg = cls(
            matrix=matrix,
            seed=d.get("seed"),
            concurrency=int(d.get("concurrency", 1) or 1),
            grid_search=GridSearchConfig.from_dict(d["grid_search"]) if d.get("grid_search") is not None else None,
            random_search=RandomSearchConfig.from_dict(d["random_search"]) if d.get("random_search") else None,
            hyperband=HyperbandConfig.from_dict(d["hyperband"]) if d.get("hyperband") else None,
            bo=BOConfig.from_dict(d["bo"]) if d.get("bo") else None,
            asha=AshaConfig.from_dict(d["asha"]) if d.get("asha") else None,
            early_stopping=[EarlyStoppingMetricConfig.from_dict(e) for e in d.get("early_stopping") or []],
        )
        if cfg.search_algorithm == SearchAlgorithms.GRID:
            cont = [k for k, v in matrix.items() if v.is_continuous]
            if cont:
                raise MatrixValidationError(f"grid search requires discrete matrix values; continuous: {cont}")
        return cfg

    @property
    def search_algorithm(self) -> str:
        for a in (SearchAlgorithms.RANDOM, SearchAlgorithms.HYPERBAND, SearchAlgorithms.BO, SearchAlgorithms.ASHA):
            if getattr(self, a) is not None:
                return a
        return SearchAlgorithms.GRID

    def to_dict(self) -> Dict[str, Any]:
        out: Dict[str, Any] = {"matrix": {k: v.to_dict() for k, v in self.matrix.items()},
                               "concurrency": self.concurrency}
        if self.seed is not None:
            out["seed"] = self.seed
        for a in SearchAlgorithms.VALUES:
            v = getattr(self, a)
            if v is not None:
                out[a] = v.to_dict()
        if self.early_stopping:
            out["early_stopping"] = [e.to_dict() for e in self.early_stopping]
        return out
