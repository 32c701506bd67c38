"""Search-algorithm managers: grid, random, Hyperband (reference-exact) and ASHA (new, asynchronous).

Reference: polyaxon/hpsearch/search_managers/{__init__,base,grid,random,hyperband}.py.  Formulas and
their floating-point quirks are kept bit-for-bit: ``s_max = int(log(R)/log(eta))``,
``B = (s_max+1)·R``, ``n = ceil((B/R)·eta^s/(s+1))``, ``r = R·eta^-s``, ``keep = int(n·eta^-i/eta)``,
and the same seed reused for every bracket's random suggestions (§8.6).

BO lives in :mod:`polyaxon_amd.polytune.bo` (GP + acquisition on the HIP kernels).
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from polyaxon_amd.polytune.utils import get_random_suggestions
from polyaxon_amd.spec.hptuning import HPTuningConfig, Optimization, SearchAlgorithms


class BaseSearchAlgorithmManager:
    NAME: Optional[str] = None

    def __init__(self, hptuning_config: HPTuningConfig):
        self.hptuning_config = hptuning_config

    def get_suggestions(self, iteration_config=None) -> List[Dict[str, Any]]:
        raise NotImplementedError


class GridSearchManager(BaseSearchAlgorithmManager):
    """Cartesian product of the (discrete) matrix, capped by ``grid_search.n_experiments``
    (reference grid.py:12-31)."""

    NAME = SearchAlgorithms.GRID

    def get_suggestions(self, iteration_config=None):
        matrix = self.hptuning_config.matrix
        keys = list(matrix.keys())
        n = None
        if self.hptuning_config.grid_search is not None:
            n = self.hptuning_config.grid_search.n_experiments
        out = []
        for combo in itertools.product(*[matrix[k].to_numpy() for k in keys]):
            out.append({k: (v.item() if hasattr(v, "item") else v) for k, v in zip(keys, combo)})
            if n and len(out) >= n:
                break
        return out


class RandomSearchManager(BaseSearchAlgorithmManager):
    NAME = SearchAlgorithms.RANDOM

    def get_suggestions(self, iteration_config=None):
        cfg = self.hptuning_config
        if cfg.random_search.sampler == "device":
            from polyaxon_amd.polytune.sampler import philox_random_suggestions

            return philox_random_suggestions(cfg.matrix, cfg.random_search.n_experiments, seed=cfg.seed)
        return get_random_suggestions(cfg.matrix, cfg.random_search.n_experiments, seed=cfg.seed)


@dataclass
class HyperbandIterationConfig:
    """State of one (iteration = bracket index, bracket_iteration = rung) step
    (reference hpsearch/schemas/hyperband.py:25-32)."""
    iteration: int
    bracket_iteration: int = 0
    experiment_ids: List[int] = field(default_factory=list)
    experiments_metrics: List[Tuple[int, float]] = field(default_factory=list)

    def to_dict(self):
        return {"iteration": self.iteration, "bracket_iteration": self.bracket_iteration,
                "experiment_ids": list(self.experiment_ids),
                "experiments_metrics": [list(m) for m in self.experiments_metrics]}

    @classmethod
    def from_dict(cls, d):
        return cls(iteration=d["iteration"], bracket_iteration=d.get("bracket_iteration", 0),
                   experiment_ids=list(d.get("experiment_ids") or []),
                   experiments_metrics=[tuple(m) for m in d.get("experiments_metrics") or []])


class HyperbandSearchManager(BaseSearchAlgorithmManager):
    NAME = SearchAlgorithms.HYPERBAND

    def __init__(self, hptuning_config: HPTuningConfig):
        super().__init__(hptuning_config)
        hb = hptuning_config.hyperband
        self.max_iter = hb.max_iter
        self.eta = hb.eta
        self.s_max = int(math.log(self.max_iter) / math.log(self.eta))
        self.B = (self.s_max + 1) * self.max_iter

    def get_bracket(self, iteration: int) -> int:
        return self.s_max - iteration

    def get_n_configs(self, bracket: int) -> int:
        return int(math.ceil((self.B / self.max_iter) * (self.eta ** bracket) / (bracket + 1)))

    def get_resources(self, bracket: int) -> float:
        return self.max_iter * (self.eta ** (-bracket))

    def get_resources_for_iteration(self, iteration: int) -> float:
        return self.get_resources(self.get_bracket(iteration))

    def get_n_config_to_keep(self, n_suggestions: int, bracket_iteration: int) -> int:
        return int(n_suggestions * (self.eta ** -bracket_iteration) / self.eta)

    def get_n_config_to_keep_for_iteration(self, iteration: int, bracket_iteration: int) -> int:
        bracket = self.get_bracket(iteration)
        if bracket_iteration == bracket + 1:
            return 0
        return self.get_n_config_to_keep(self.get_n_configs(bracket), bracket_iteration)

    def get_n_resources(self, n_resources: float, bracket_iteration: int) -> float:
        return n_resources * self.eta ** bracket_iteration

    def get_n_resources_for_iteration(self, iteration: int, bracket_iteration: int) -> float:
        return self.get_n_resources(self.get_resources_for_iteration(iteration), bracket_iteration)

    def get_suggestions(self, iteration_config=None):
        if not isinstance(iteration_config, HyperbandIterationConfig):
            raise ValueError("Hyperband get suggestions requires an iteration.")
        cfg = self.hptuning_config
        bracket = self.get_bracket(iteration_config.iteration)
        n_configs = self.get_n_configs(bracket)
        r = self.get_n_resources_for_iteration(iteration_config.iteration, iteration_config.bracket_iteration)
        r = cfg.hyperband.resource.cast_value(r)
        return get_random_suggestions(cfg.matrix, n_configs, {cfg.hyperband.resource.name: r}, seed=cfg.seed)

    def should_reschedule(self, iteration: int, bracket_iteration: int) -> bool:
        if bracket_iteration < self.get_bracket(iteration):
            return False
        return self.get_bracket(iteration + 1) >= 0

    def should_reduce_configs(self, iteration: int, bracket_iteration: int) -> bool:
        return self.get_n_config_to_keep_for_iteration(iteration, bracket_iteration) > 0

    # ---------------------------------------------------------------- iteration state machine
    def next_iteration(self, current: Optional[HyperbandIterationConfig]) -> HyperbandIterationConfig:
        """Reference HyperbandIterationManager.create_iteration (iteration_managers/hyperband.py:14-50)."""
        if current is None:
            return HyperbandIterationConfig(iteration=0, bracket_iteration=0)
        if self.should_reschedule(current.iteration, current.bracket_iteration):
            return HyperbandIterationConfig(iteration=current.iteration + 1, bracket_iteration=0)
        if self.should_reduce_configs(current.iteration, current.bracket_iteration):
            return HyperbandIterationConfig(iteration=current.iteration, bracket_iteration=current.bracket_iteration + 1)
        raise ValueError("Hyperband create iteration failed: could not reschedule or reduce configs")

    def reduce(self, current: HyperbandIterationConfig, select=None) -> List[int]:
        """Ids to promote: the top ``keep`` of the rung by metric (reference get_reduced_configs :52-77).
        ``select`` may be a device top-k (polyaxon_amd.polytune.kernels.select_top) with the same ordering."""
        keep = self.get_n_config_to_keep_for_iteration(current.iteration, current.bracket_iteration)
        maximize = Optimization.maximize(self.hptuning_config.hyperband.metric.optimization)
        metrics = [m for m in current.experiments_metrics if m[1] is not None]
        if select is not None:
            return select(metrics, keep, maximize)
        ordered = sorted(metrics, key=lambda x: x[1], reverse=maximize)
        return [m[0] for m in ordered[:keep]]

    def is_done(self, current: HyperbandIterationConfig) -> bool:
        return (not self.should_reschedule(current.iteration, current.bracket_iteration)
                and not self.should_reduce_configs(current.iteration, current.bracket_iteration))


class AshaSearchManager(BaseSearchAlgorithmManager):
    """Asynchronous successive halving (Li et al. 2018) — the reference has only the synchronous rung
    barrier (hpsearch/tasks/hyperband.py:57-60, 30 s poll).  Rungs k = 0..K with resource
    ``r_k = min_resource · eta^k`` (≤ max_resource).  Whenever a worker frees up, ``next_job`` promotes the
    best config of the highest rung that has one in its top ``floor(n_rung/eta)`` not yet promoted, else
    starts a new random config at rung 0 (until ``n_experiments`` configs were started)."""

    NAME = SearchAlgorithms.ASHA

    def __init__(self, hptuning_config: HPTuningConfig):
        super().__init__(hptuning_config)
        a = hptuning_config.asha
        self.eta = a.eta
        self.min_r = a.min_resource
        self.max_r = a.max_resource
        self.n_rungs = int(math.floor(math.log(self.max_r / self.min_r) / math.log(self.eta) + 1e-9)) + 1
        self.maximize = Optimization.maximize(a.metric.optimization)
        self.rungs: List[Dict[int, float]] = [dict() for _ in range(self.n_rungs)]
        self.promoted: List[set] = [set() for _ in range(self.n_rungs)]
        self.configs: Dict[int, Dict[str, Any]] = {}
        self._pending = get_random_suggestions(hptuning_config.matrix, a.n_experiments, seed=hptuning_config.seed)
        self._next_id = 0

    def resource(self, rung: int):
        return self.hptuning_config.asha.resource.cast_value(min(self.min_r * self.eta ** rung, self.max_r))

    def report(self, config_id: int, rung: int, metric: float) -> None:
        self.rungs[rung][config_id] = metric

    def _top(self, rung: int) -> List[int]:
        entries = sorted(self.rungs[rung].items(), key=lambda kv: kv[1], reverse=self.maximize)
        k = int(len(entries) / self.eta)
        return [cid for cid, _ in entries[:k]]

    def next_job(self) -> Optional[Tuple[int, int, Dict[str, Any]]]:
        """(config_id, rung, params) to run next, or None if nothing is runnable right now."""
        for rung in range(self.n_rungs - 2, -1, -1):
            for cid in self._top(rung):
                if cid not in self.promoted[rung]:
                    self.promoted[rung].add(cid)
                    params = dict(self.configs[cid])
                    params[self.hptuning_config.asha.resource.name] = self.resource(rung + 1)
                    return cid, rung + 1, params
        if self._pending:
            params = self._pending.pop(0)
            cid = self._next_id
            self._next_id += 1
            self.configs[cid] = params
            p = dict(params)
            p[self.hptuning_config.asha.resource.name] = self.resource(0)
            return cid, 0, p
        return None

    def get_suggestions(self, iteration_config=None):
        return list(self._pending)


def get_search_algorithm_manager(hptuning_config: HPTuningConfig) -> BaseSearchAlgorithmManager:
    """Reference hpsearch/search_managers/__init__.py:8-21."""
    algo = hptuning_config.search_algorithm
    if algo == SearchAlgorithms.GRID:
        return GridSearchManager(hptuning_config)
    if algo == SearchAlgorithms.RANDOM:
        return RandomSearchManager(hptuning_config)
    if algo == SearchAlgorithms.HYPERBAND:
        return HyperbandSearchManager(hptuning_config)
    if algo == SearchAlgorithms.ASHA:
        return AshaSearchManager(hptuning_config)
    if algo == SearchAlgorithms.BO:
        from polyaxon_amd.polytune.bo import BOSearchManager
        return BOSearchManager(hptuning_config)
    raise ValueError(f"Search algorithm `{algo}` is not supported")
