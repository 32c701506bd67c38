"""Hyper-parameter matrix distributions (the ``hptuning.matrix`` section of a Polyaxonfile).

Re-implements the contract of the external ``polyaxon_schemas.matrix.MatrixConfig`` that the reference
imports (polyaxon/schemas/hptuning.py:1-19) from its documentation
(docs/templates/polyaxonfile_specification/sections.md:68-200) and its call sites:
``is_continuous/is_discrete/is_categorical/is_uniform``, ``min/max``, ``to_numpy()`` and
``sample(rand_generator=...)`` (polyaxon/hpsearch/search_managers/utils.py:41-64,
polyaxon/hpsearch/search_managers/bayesian_optimization/space.py:67-93).

Accepted value syntaxes for every option: a list ``[a, b, c]``, a mapping (``{start, stop, step}``,
``{start, stop, num}``, ``{low, high[, q]}``, ``{loc, scale[, q]}``) or a colon string ``'a:b:c'``.
The log-family distributions follow hyperopt conventions (the reference's schema package was modelled on
them): ``loguniform(low, high) = exp(uniform(low, high))``, ``lognormal(loc, scale) = exp(normal(...))``,
and every ``q*`` variant is ``round(x / q) * q``.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

DISCRETE = ("values", "range", "linspace", "logspace", "geomspace")
CONTINUOUS = ("uniform", "quniform", "loguniform", "qloguniform", "normal", "qnormal", "lognormal",
              "qlognormal")
DISTRIBUTIONS = ("pvalues",) + CONTINUOUS
ALL = DISCRETE + DISTRIBUTIONS

_KEYS = {
    "range": ("start", "stop", "step"),
    "linspace": ("start", "stop", "num"),
    "logspace": ("start", "stop", "num"),
    "geomspace": ("start", "stop", "num"),
    "uniform": ("low", "high"),
    "quniform": ("low", "high", "q"),
    "loguniform": ("low", "high"),
    "qloguniform": ("low", "high", "q"),
    "normal": ("loc", "scale"),
    "qnormal": ("loc", "scale", "q"),
    "lognormal": ("loc", "scale"),
    "qlognormal": ("loc", "scale", "q"),
}


class MatrixValidationError(ValueError):
    pass


def _num(x: Any):
    """Numeric literal from YAML/JSON/colon-string; ints stay ints so ``range`` yields ints."""
    if isinstance(x, str):
        x = x.strip()
        try:
            return int(x)
        except ValueError:
            return float(x)
    if isinstance(x, bool) or not _is_number(x):
        raise MatrixValidationError(f"expected a number, got {x!r}")
    return x


def _parse_args(option: str, raw: Any) -> List[float]:
    keys = _KEYS[option]
    if isinstance(raw, str):
        parts = [p for p in raw.split(":")]
        vals = [_num(p) for p in parts]
    elif isinstance(raw, dict):
        missing = [k for k in keys[:2] if k not in raw]
        if missing:
            raise MatrixValidationError(f"`{option}` needs keys {keys}, missing {missing}")
        vals = [_num(raw[k]) for k in keys if k in raw]
    elif isinstance(raw, (list, tuple)):
        vals = [_num(v) for v in raw]
    else:
        raise MatrixValidationError(f"`{option}` got an unsupported value {raw!r}")
    if len(vals) != len(keys):
        raise MatrixValidationError(f"`{option}` expects {len(keys)} values {keys}, got {vals}")
    return vals


def _is_number(v: Any) -> bool:
    return isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool)


class MatrixConfig:
    """One matrix entry, e.g. ``{'logspace': '0.01:0.1:5'}``."""

    def __init__(self, option: str, value: Any):
        if option not in ALL:
            raise MatrixValidationError(f"unknown matrix option `{option}`; expected one of {ALL}")
        self.option = option
        self.raw = value
        if option == "values":
            if not isinstance(value, (list, tuple)) or not value:
                raise MatrixValidationError("`values` expects a non-empty list")
            self.values = list(value)
        elif option == "pvalues":
            pairs = []
            for item in value:
                if isinstance(item, dict):
                    pairs.append((item["value"], float(item["prob"])))
                else:
                    v, p = item
                    pairs.append((v, float(p)))
            total = sum(p for _, p in pairs)
            if not pairs or abs(total - 1.0) > 1e-6:
                raise MatrixValidationError(f"`pvalues` probabilities must sum to 1, got {total}")
            self.values = [v for v, _ in pairs]
            self.probs = [p for _, p in pairs]
        else:
            self.args = _parse_args(option, value)
            if option in ("uniform", "quniform", "loguniform", "qloguniform") and self.args[0] >= self.args[1]:
                raise MatrixValidationError(f"`{option}` needs low < high, got {self.args}")
            if option in ("normal", "qnormal", "lognormal", "qlognormal") and self.args[1] <= 0:
                raise MatrixValidationError(f"`{option}` needs scale > 0, got {self.args}")

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "MatrixConfig":
        if isinstance(data, MatrixConfig):
            return data
        if not isinstance(data, dict) or len(data) != 1:
            raise MatrixValidationError(f"a matrix entry needs exactly one option, got {data!r}")
        (option, value), = data.items()
        return cls(option, value)

    def to_dict(self) -> Dict[str, Any]:
        return {self.option: self.raw}

    # ------------------------------------------------------------------ classification
    @property
    def is_distribution(self) -> bool:
        return self.option in DISTRIBUTIONS

    @property
    def is_continuous(self) -> bool:
        return self.option in CONTINUOUS

    @property
    def is_discrete(self) -> bool:
        return not self.is_continuous

    @property
    def is_categorical(self) -> bool:
        return self.option in ("values", "pvalues") and any(not _is_number(v) for v in self.values)

    @property
    def is_range(self) -> bool:
        return self.option == "range"

    @property
    def is_uniform(self) -> bool:
        """Continuous with a bounded box usable by the BO search space."""
        return self.option in CONTINUOUS

    # ------------------------------------------------------------------ values
    def to_numpy(self) -> np.ndarray:
        o = self.option
        if o in ("values", "pvalues"):
            return np.asarray(self.values)
        if o == "range":
            return np.arange(*self.args)
        if o == "linspace":
            a, b, n = self.args
            return np.linspace(a, b, int(n))
        if o == "logspace":
            a, b, n = self.args
            return np.logspace(a, b, int(n))
        if o == "geomspace":
            a, b, n = self.args
            return np.geomspace(a, b, int(n))
        raise MatrixValidationError(f"`{o}` is a continuous distribution and has no finite value list")

    @property
    def length(self) -> int:
        return len(self.to_numpy())

    @property
    def min(self) -> Optional[float]:
        o = self.option
        if self.is_categorical:
            return None
        if self.is_discrete:
            return float(np.min(self.to_numpy())) if o != "range" else self.to_numpy().min()
        return self._box()[0]

    @property
    def max(self) -> Optional[float]:
        o = self.option
        if self.is_categorical:
            return None
        if self.is_discrete:
            return float(np.max(self.to_numpy())) if o != "range" else self.to_numpy().max()
        return self._box()[1]

    def _box(self):
        o, a = self.option, self.args
        if o in ("uniform", "quniform"):
            return float(a[0]), float(a[1])
        if o in ("loguniform", "qloguniform"):
            return math.exp(a[0]), math.exp(a[1])
        if o in ("normal", "qnormal"):
            return a[0] - 3 * a[1], a[0] + 3 * a[1]
        return math.exp(a[0] - 3 * a[1]), math.exp(a[0] + 3 * a[1])

    def sample(self, size: Optional[int] = None, rand_generator=None):
        rng = rand_generator if rand_generator is not None else np.random
        o = self.option
        if o == "pvalues":
            idx = rng.choice(len(self.values), size=size, p=self.probs)
            return self.values[idx] if size is None else [self.values[i] for i in idx]
        if self.is_discrete:
            vals = self.to_numpy()
            idx = rng.randint(0, len(vals), size=size)
            out = vals[idx]
            return out.item() if size is None and hasattr(out, "item") else out
        a = self.args
        if o in ("uniform", "quniform", "loguniform", "qloguniform"):
            x = rng.uniform(a[0], a[1], size=size)
        else:
            x = rng.normal(a[0], a[1], size=size)
        if o in ("loguniform", "qloguniform", "lognormal", "qlognormal"):
            x = np.exp(x)
        if o.startswith("q"):
            q = a[2]
            x = np.round(x / q) * q
        return float(x) if size is None else x

    def __repr__(self) -> str:
        return f"MatrixConfig({self.option}={self.raw!r})"


def parse_matrix(matrix: Dict[str, Any]) -> Dict[str, MatrixConfig]:
    if not isinstance(matrix, dict) or not matrix:
        raise MatrixValidationError("`matrix` must be a non-empty mapping")
    return {k: MatrixConfig.from_dict(v) for k, v in matrix.items()}


def space_size(matrix: Dict[str, MatrixConfig]) -> Optional[int]:
    """Cardinality of an all-discrete matrix (None if any entry is continuous)."""
    n = 1
    for v in matrix.values():
        if v.is_continuous:
            return None
        n *= v.length
    return n


def ensure_seq(x) -> Sequence:
    return x if isinstance(x, (list, tuple)) else [x]
