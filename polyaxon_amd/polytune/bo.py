"""Bayesian optimisation: search space, Gaussian process, acquisition maximisation, BO search manager.

Reference: polyaxon/hpsearch/search_managers/bayesian_optimization/{space,acquisition_function,optimizer,
manager}.py and hpsearch/schemas/bayesian_optimization.py.

Two execution paths, same semantics:

* ``backend="reference"`` — sklearn ``GaussianProcessRegressor`` (Matern/RBF, alpha=1e-10, LML fit of the
  length scale with ``n_restarts_optimizer``) + random warm-up + scipy L-BFGS-B restarts, with the
  reference defaults ``n_warmup or 5``, ``n_iter or 10`` (optimizer.py:13-14).  Used for parity tests.
* ``backend="hip"`` (default on a GPU) — the GP posterior and the acquisition are evaluated by the HIP
  kernels in csrc/gp_kernels.hip: Gram matrix via MFMA + fused Matern epilogue (general nu included),
  single-workgroup fp64 LDS Cholesky, fused predict+UCB/EI/POI+argmax over every candidate in one launch.
  Because a candidate costs nanoseconds there, acquisition maximisation evaluates the docstring's intended
  effort (1e5 random candidates, acquisition_function.py:75) plus rounds of batched local refinement around
  the best points instead of sequential scipy restarts.  The length scale is fit by maximising the log
  marginal likelihood on the device too: batched Gram kernels + one batched fp64 Cholesky per zoom round
  (``HipGP.fit_length_scale``), so an n ~ 1000 suggestion is not bound by host O(n^3) factorisations.
* ``backend="numpy"`` — the same math as the HIP path in numpy (CPU-only hosts, and the kernels' parity
  reference).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from polyaxon_amd.polytune.managers import BaseSearchAlgorithmManager
from polyaxon_amd.polytune.utils import get_random_generator, get_random_suggestions
from polyaxon_amd.spec.hptuning import HPTuningConfig, Optimization, SearchAlgorithms

# May this process run the GP on the GPU?  The scheduler (control) process says no at start: it stays HIP-free (no
# device context outside the allocator's accounting), like the reference's hpsearch workers, which run on their own
# CPU queue apart from the trial pods (/root/reference/polyaxon/polyaxon/config_settings/celery_settings.py:398-419).
_DEVICE_ALLOWED = True


def set_device_allowed(allowed: bool) -> None:
    global _DEVICE_ALLOWED
    _DEVICE_ALLOWED = bool(allowed)


def device_allowed() -> bool:
    return _DEVICE_ALLOWED

KIND_IDS = {"rbf": 0, "matern05": 1, "matern15": 2, "matern25": 3, "matern_nu": 4}


# ================================================================================ search space
class SearchSpace:
    """Feature encoding of the matrix (reference space.py:9-164): sorted keys, one-hot categoricals,
    discrete values snapped back to the nearest feasible value, continuous bounds."""

    def __init__(self, hptuning_config: HPTuningConfig):
        self.hptuning_config = hptuning_config
        self.features: List[str] = []
        self.discrete_features: Dict[str, Dict] = {}
        self.categorical_features: Dict[str, Dict] = {}
        self.dim = 0
        self.x = np.zeros((0, 0))
        self.y = np.zeros(0)
        bounds = []
        bo = hptuning_config.bo
        unit = bo is not None and getattr(bo, "space", "raw") == "unit"
        self.scale: Dict[str, Tuple[bool, float, float]] = {}  # unit space: feature -> (log, lo, hi) in model units
        for key in sorted(hptuning_config.matrix):
            v = hptuning_config.matrix[key]
            self.features.append(key)
            if v.is_categorical:
                values = v.to_numpy()
                for _ in range(len(values)):
                    bounds.append((0, 1))
                self.categorical_features[key] = {"values": values, "number": len(values)}
                self.dim += len(values)
                continue
            lo, hi = float(v.min), float(v.max)
            if v.is_discrete:
                self.discrete_features[key] = {"values": v.to_numpy()}
            if unit:
                log = getattr(v, "option", None) in ("loguniform", "qloguniform", "lognormal", "qlognormal") and lo > 0
                if log:
                    lo, hi = math.log(lo), math.log(hi)
                self.scale[key] = (log, lo, hi if hi > lo else lo + 1.0)
                bounds.append((0.0, 1.0))
            else:
                bounds.append((lo, hi) if not v.is_discrete else (v.min, v.max))
            self.dim += 1
        self.bounds = np.asarray(bounds, dtype=np.float64)

    def _to_model(self, f: str, val: float) -> float:
        if f not in self.scale:
            return val
        log, lo, hi = self.scale[f]
        x = math.log(val) if log else float(val)
        return (x - lo) / (hi - lo)

    def _from_model(self, f: str, x: float) -> float:
        if f not in self.scale:
            return x
        log, lo, hi = self.scale[f]
        v = lo + float(x) * (hi - lo)
        return math.exp(v) if log else v

    def _maximize(self) -> bool:
        return Optimization.maximize(self.hptuning_config.bo.metric.optimization)

    def parse_y(self, metrics):
        if metrics is None or len(metrics) == 0:
            return metrics
        return np.array([float(v) if self._maximize() else -float(v) for v in metrics])

    def parse_x(self, configs):
        if configs is None or len(configs) == 0:
            return configs
        rows = []
        for cfg in configs:
            row = []
            for f in self.features:
                if f in self.categorical_features:
                    row += [1 if v == cfg[f] else 0 for v in self.categorical_features[f]["values"]]
                else:
                    row.append(self._to_model(f, cfg[f]))
            rows.append(row)
        return np.array(rows, dtype=np.float64)

    def add_observations(self, configs, metrics) -> None:
        self.x = self.parse_x(configs)
        self.y = self.parse_y(metrics)

    def is_observations_valid(self) -> bool:
        return self.x is not None and self.y is not None and len(self.x) == len(self.y) and len(self.x) > 0

    def get_suggestion(self, x) -> Optional[Dict[str, Any]]:
        if x is None:
            return None
        out, c = {}, 0
        for f in self.features:
            if f in self.discrete_features:
                vals = self.discrete_features[f]["values"]
                v = vals[int(np.argmin(np.abs(np.subtract(vals, self._from_model(f, x[c])))))]
                c += 1
            elif f in self.categorical_features:
                n = self.categorical_features[f]["number"]
                v = self.categorical_features[f]["values"][int(np.argmax(x[c:c + n]))]
                c += n
            else:
                v = self._from_model(f, x[c])
                c += 1
            out[f] = v.item() if hasattr(v, "item") else v
        return out


# ================================================================================ GP math (numpy)
def _kind(kernel: str, nu: float) -> str:
    if kernel == "rbf":
        return "rbf"
    for half, name in ((0.5, "matern05"), (1.5, "matern15"), (2.5, "matern25")):
        if abs(nu - half) < 1e-12:
            return name
    if math.isinf(nu):
        return "rbf"
    return "matern_nu"


def matern_c(nu: float) -> float:
    return 2.0 ** (1.0 - nu) / math.gamma(nu)


def kernel_np(A: np.ndarray, B: np.ndarray, kind: str, ls: float, nu: float) -> np.ndarray:
    sq = np.maximum((A * A).sum(1)[:, None] + (B * B).sum(1)[None, :] - 2.0 * A @ B.T, 0.0)
    r2 = sq / (ls * ls)
    if kind == "rbf":
        return np.exp(-0.5 * r2)
    r = np.sqrt(r2)
    if kind == "matern05":
        return np.exp(-r)
    if kind == "matern15":
        a = math.sqrt(3.0) * r
        return (1 + a) * np.exp(-a)
    if kind == "matern25":
        a = math.sqrt(5.0) * r
        return (1 + a + a * a / 3.0) * np.exp(-a)
    from scipy.special import kv

    s = math.sqrt(2.0 * nu) * r
    with np.errstate(invalid="ignore", divide="ignore"):
        K = matern_c(nu) * np.power(s, nu) * kv(nu, s)
    K[s < 1e-8] = 1.0
    return K


@dataclass
class GPState:
    X: np.ndarray
    y: np.ndarray
    ls: float
    kind: str
    nu: float
    L: np.ndarray
    alpha: np.ndarray
    lml: float


def fit_gp(X: np.ndarray, y: np.ndarray, kernel: str = "matern", nu: float = 1.5, length_scale: float = 1.0,
           alpha: float = 1e-10, optimize: bool = True, bounds=(1e-5, 1e5)) -> GPState:
    """GP fit with the length scale chosen by maximising the log marginal likelihood (like sklearn's
    default optimizer, here a bounded 1-D search on log ls since the kernel has one hyper-parameter)."""
    kind = _kind(kernel, nu)

    def factor(ls):
        K = kernel_np(X, X, kind, ls, nu) + alpha * np.eye(len(X))
        jitter = 0.0
        for _ in range(8):
            try:
                L = np.linalg.cholesky(K + jitter * np.eye(len(X)))
                break
            except np.linalg.LinAlgError:
                jitter = max(jitter * 10, 1e-10)
        else:
            return None
        a = np.linalg.solve(L.T, np.linalg.solve(L, y))
        lml = -0.5 * float(y @ a) - float(np.log(np.diag(L)).sum()) - 0.5 * len(X) * math.log(2 * math.pi)
        return L, a, lml

    ls = float(length_scale)
    if optimize and len(X) > 1:
        from scipy.optimize import minimize_scalar

        def neg(log_ls):
            f = factor(math.exp(log_ls))
            return 1e25 if f is None else -f[2]

        res = minimize_scalar(neg, bounds=(math.log(bounds[0]), math.log(bounds[1])), method="bounded",
                              options={"xatol": 1e-4})
        cand = [math.log(ls), res.x]
        ls = math.exp(min(cand, key=neg))
    L, a, lml = factor(ls)
    return GPState(X, y, ls, kind, nu, L, a, lml)


def predict_np(gp: GPState, Xc: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    Ks = kernel_np(Xc, gp.X, gp.kind, gp.ls, gp.nu)
    mean = Ks @ gp.alpha
    from scipy.linalg import solve_triangular

    v = solve_triangular(gp.L, Ks.T, lower=True)
    var = np.maximum(1.0 - (v * v).sum(0), 0.0)
    return mean, np.sqrt(var)


def acquisition_np(mean, std, acq: str, y_max: float, kappa: float, eps: float) -> np.ndarray:
    if acq == "ucb":
        return mean + kappa * std
    from scipy.stats import norm

    with np.errstate(divide="ignore", invalid="ignore"):
        z = np.where(std > 0, (mean - y_max - eps) / np.where(std > 0, std, 1), 0.0)
    if acq == "poi":
        return np.where(std > 0, norm.cdf(z), (mean - y_max - eps > 0).astype(float))
    return np.where(std > 0, (mean - y_max - eps) * norm.cdf(z) + std * norm.pdf(z),
                    np.maximum(mean - y_max - eps, 0.0))


# ================================================================================ HIP path
class HipGP:
    """GP posterior + acquisition on the MI355X kernels. Training data and factors stay on the device.

    Every factorisation is ours: the blocked fp64 Cholesky of csrc/gp_chol.hip, batched over length scales, with
    right-hand sides appended as extra rows (y -> z = L^-1 y for the LML; the identity -> L^-T for the posterior),
    so there is no host LAPACK and no rocSOLVER call at any n (torch's device Cholesky faulted the GPU at n = 1000
    on this ROCm build).  The posterior for m candidates is one MFMA cross-kernel launch, one GEMM with L^-T
    (V = K* L^-T, rows v_c = L^-1 k_c) and one fused mean/variance/acquisition epilogue; n <= 64 keeps the
    single fused predict+acquisition kernel."""

    FUSED_MAX = 64
    TABLE_NODES = 16384
    TABLE_SMAX = 50.0  # tabulate s = sqrt(2 nu) r up to 50: k < 1e-20 beyond

    _tables: Dict[Tuple[str, float], Tuple[Any, Any, float]] = {}

    def __init__(self, device=None):
        import torch

        self.torch = torch
        self.device = torch.device(device or "cuda")
        from polyaxon_amd.ops import _native

        self.lib = _native.lib("plx_gp")
        self._native = _native

    def table(self, kind: str, nu: float):
        """(t64 ptr, t32 ptr, rmax, nodes) of the Matern-nu lookup table (built once per device and nu by
        plx_gp_matern_table); null table for the closed-form kernels."""
        if kind != "matern_nu":
            return None, None, 0.0, 0
        key = (str(self.device), float(nu))
        if key not in HipGP._tables:
            t = self.torch
            n = self.TABLE_NODES
            rmax = self.TABLE_SMAX / math.sqrt(2.0 * nu)
            t64 = t.empty(2 * n, dtype=t.float64, device=self.device)
            t32 = t.empty(2 * n, dtype=t.float32, device=self.device)
            rc = self.lib.plx_gp_matern_table(float(nu), float(matern_c(nu)), rmax, n, t64.data_ptr(), t32.data_ptr(),
                                              self._stream())
            self._native.check(rc, "plx_gp_matern_table")
            HipGP._tables[key] = (t64, t32, rmax)
        t64, t32, rmax = HipGP._tables[key]
        return t64.data_ptr(), t32.data_ptr(), rmax, self.TABLE_NODES

    def _stream(self):
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def kmat(self, A, B, kind: str, ls: float, nu: float, diag: float = 0.0):
        t = self.torch
        A = t.as_tensor(A, dtype=t.float32, device=self.device).contiguous()
        B = t.as_tensor(B, dtype=t.float32, device=self.device).contiguous()
        K = t.empty((A.shape[0], B.shape[0]), dtype=t.float32, device=self.device)
        rc = self.lib.plx_gp_kmat(A.data_ptr(), B.data_ptr(), A.shape[0], B.shape[0], A.shape[1], K.data_ptr(),
                                  K.shape[1], KIND_IDS[kind], float(ls), float(nu),
                                  float(matern_c(nu)) if kind == "matern_nu" else 0.0, int(diag != 0.0), float(diag),
                                  *self.table(kind, nu), self._stream())
        self._native.check(rc, "plx_gp_kmat")
        return K

    def gram_f64(self, X, kind: str, nu: float, inv_ls2, rows: int, diag: float):
        """fp64 Gram matrices for every 1/ls^2 in ``inv_ls2`` (device fp64 [nb]) into rows [0, n) of a zeroed
        [nb, rows, n] buffer; rows [n, rows) are left for appended right-hand sides."""
        t = self.torch
        Xd = t.as_tensor(np.ascontiguousarray(X, dtype=np.float64), device=self.device)
        n, d = Xd.shape
        nb = int(inv_ls2.shape[0])
        A = t.zeros((nb, rows, n), dtype=t.float64, device=self.device)
        rc = self.lib.plx_gp_kmat_batch_f64(Xd.data_ptr(), n, d, inv_ls2.data_ptr(), nb, A.data_ptr(), n, rows * n,
                                            KIND_IDS[kind], float(nu),
                                            float(matern_c(nu)) if kind == "matern_nu" else 0.0, float(diag),
                                            *self.table(kind, nu), self._stream())
        self._native.check(rc, "plx_gp_kmat_batch_f64")
        return A

    def chol_aug(self, A, n: int):
        """In-place blocked fp64 Cholesky of A [nb, rows, n] (plx_gp_chol_aug_f64). Returns the device int32
        status per entry (0 = SPD, else the 1-based column of the first non-positive pivot)."""
        t = self.torch
        nb, rows = int(A.shape[0]), int(A.shape[1])
        assert A.dtype == t.float64 and A.is_contiguous() and A.shape[2] == n and rows >= n
        status = t.zeros(nb, dtype=t.int32, device=self.device)
        # per-matrix copy of the current diagonal block (the panel launch overwrites A11 in place, see gp_chol.hip)
        scratch = t.empty(nb * int(self.lib.plx_gp_chol_scratch_doubles()), dtype=t.float64, device=self.device)
        rc = self.lib.plx_gp_chol_aug_f64(A.data_ptr(), n, rows, n, rows * n, nb, status.data_ptr(),
                                          scratch.data_ptr(), self._stream())
        self._native.check(rc, "plx_gp_chol_aug_f64")
        return status

    def cholesky(self, K):
        """Lower Cholesky factor of one SPD matrix (fp32 in/out): the single-workgroup LDS kernel up to n = 128,
        the blocked fp64 kernel above."""
        t = self.torch
        n = K.shape[0]
        if n > 128:
            A = K.to(t.float64).contiguous()[None].clone()
            st = int(self.chol_aug(A, n)[0].item())
            if st != 0:
                raise np.linalg.LinAlgError(f"not positive definite at column {st}")
            return A[0].tril().to(t.float32)
        status = t.zeros(1, dtype=t.int32, device=self.device)
        out = K.clone()
        rc = self.lib.plx_gp_chol(out.data_ptr(), n, n, status.data_ptr(), self._stream())
        self._native.check(rc, "plx_gp_chol")
        if int(status.item()) != 0:
            raise np.linalg.LinAlgError(f"not positive definite at column {int(status.item())}")
        return out

    def lml_batch(self, X, y, kind: str, nu: float, log_ls, alpha: float = 1e-10):
        """Log marginal likelihood at every length scale exp(log_ls) with sklearn's semantics (fp64, alpha on the
        diagonal, -inf when not positive definite): one batched Gram launch, one batched blocked Cholesky with y
        appended (z = L^-1 y), one reduction launch; a single D2H of nb values."""
        t = self.torch
        n = len(X)
        nb = len(log_ls)
        inv = t.tensor([math.exp(-2.0 * float(l)) for l in log_ls], dtype=t.float64, device=self.device)
        A = self.gram_f64(X, kind, nu, inv, n + 1, alpha)
        A[:, n, :] = t.as_tensor(np.asarray(y, dtype=np.float64), device=self.device)
        status = self.chol_aug(A, n)
        out = t.empty(nb, dtype=t.float64, device=self.device)
        rc = self.lib.plx_gp_lml_f64(A.data_ptr(), n, n, (n + 1) * n, nb, status.data_ptr(), out.data_ptr(),
                                     self._stream())
        self._native.check(rc, "plx_gp_lml_f64")
        return out.cpu().numpy()

    def fit_length_scale(self, X, y, kind: str, nu: float, length_scale: float, alpha: float = 1e-10,
                         bounds=(1e-5, 1e5), coarse: int = 24, rounds: int = 2, zoom: int = 17) -> float:
        """Maximise the LML over log length scale on the device: a coarse batched grid over the bounds (plus the
        configured initial value, as sklearn always tries it), then batched zoom rounds around the best point.
        Replaces sklearn's L-BFGS-B on the LML, whose O(n^3) host factorisations dominate a suggestion at n ~ 1000.
        Each round is one batched factorisation (32 panel steps at n = 1000 whatever the batch), so the search uses
        few wide rounds: 25 points, then 2 zooms of 17 (final spacing 1/64 in log length scale)."""
        lo, hi = math.log(bounds[0]), math.log(bounds[1])
        grid = list(np.linspace(lo, hi, coarse)) + [math.log(length_scale)]
        vals = self.lml_batch(X, y, kind, nu, grid, alpha)
        best = int(np.argmax(vals))
        x_best, f_best = grid[best], vals[best]
        step = (hi - lo) / (coarse - 1)
        for _ in range(rounds):
            g = list(np.linspace(max(lo, x_best - step), min(hi, x_best + step), zoom))
            v = self.lml_batch(X, y, kind, nu, g, alpha)
            i = int(np.argmax(v))
            if v[i] > f_best:
                x_best, f_best = g[i], v[i]
            step = 2.0 * step / (zoom - 1)
        return math.exp(x_best) if math.isfinite(f_best) else float(length_scale)

    def fit(self, gp: GPState, alpha: float = 1e-10):
        """Device factors of a fitted GP: (X fp32, L fp32, alpha fp32, L^-T fp32, z fp32).

        One blocked fp64 Cholesky of [K; y^T; I] (2n + 1 rows): row n comes back as z = L^-1 y and rows n+1.. as
        L^-T, so alpha = L^-T z and the posterior needs only a GEMM.  A matrix that is not positive definite is
        retried with growing diagonal jitter (one status readback per attempt)."""
        t = self.torch
        n = len(gp.X)
        inv = t.tensor([1.0 / (gp.ls * gp.ls)], dtype=t.float64, device=self.device)
        yd = t.as_tensor(np.asarray(gp.y, dtype=np.float64), device=self.device)
        eye = t.eye(n, dtype=t.float64, device=self.device)
        jitter = 0.0
        for _ in range(8):
            A = self.gram_f64(gp.X, gp.kind, gp.nu, inv, 2 * n + 1, alpha + jitter)
            A[0, n] = yd
            A[0, n + 1:] = eye
            if int(self.chol_aug(A, n)[0].item()) == 0:
                break
            jitter = max(jitter * 10, 1e-8)
        else:
            raise np.linalg.LinAlgError("GP Gram matrix not positive definite")
        A = A[0]
        z = A[n]
        LinvT = A[n + 1:]
        a = LinvT @ z
        f32 = dict(dtype=t.float32)
        Xd = t.as_tensor(gp.X, dtype=t.float32, device=self.device).contiguous()
        return (Xd, A[:n].tril().to(**f32).contiguous(), a.to(**f32).contiguous(), LinvT.to(**f32).contiguous(),
                z.to(**f32).contiguous())

    def acq_dev(self, gp: GPState, dev_state, Xc, acq: str, y_max: float, kappa: float, eps: float,
                mean=None, std=None):
        """Acquisition of every candidate row of Xc (device fp32 [m, d]) as a device tensor; no host sync."""
        t = self.torch
        Xd, L, alpha, LinvT, z = dev_state
        m, n, d = Xc.shape[0], Xd.shape[0], Xd.shape[1]
        acq_id = {"ucb": 0, "ei": 1, "poi": 2}[acq]
        out = t.empty(m, dtype=t.float32, device=self.device)
        mp = mean.data_ptr() if mean is not None else None
        sp = std.data_ptr() if std is not None else None
        if n <= self.FUSED_MAX and d <= 16:
            rc = self.lib.plx_gp_predict_acq(
                Xc.data_ptr(), m, Xd.data_ptr(), n, d, L.data_ptr(), n, alpha.data_ptr(), KIND_IDS[gp.kind],
                float(gp.ls), float(gp.nu), float(matern_c(gp.nu)) if gp.kind == "matern_nu" else 0.0, 1.0, acq_id,
                float(kappa), float(eps), float(y_max), out.data_ptr(), mp, sp, None, None, *self.table(gp.kind, gp.nu),
                self._stream())
            self._native.check(rc, "plx_gp_predict_acq")
            return out
        Ks = self.kmat(Xc, Xd, gp.kind, gp.ls, gp.nu)  # MFMA cross-kernel, fused Matern epilogue
        V = Ks @ LinvT  # row c = (L^-1 k_c)^T
        rc = self.lib.plx_gp_acq_rows(V.data_ptr(), m, n, z.data_ptr(), 1.0, acq_id, float(kappa), float(eps),
                                      float(y_max), out.data_ptr(), mp, sp, self._stream())
        self._native.check(rc, "plx_gp_acq_rows")
        return out

    def fused(self, dev_state) -> bool:
        return dev_state[0].shape[0] <= self.FUSED_MAX and dev_state[0].shape[1] <= 16

    def ascent(self, gp: GPState, dev_state, xs, lo, hi, acq: str, y_max: float, kappa: float, eps: float,
               steps: int):
        """In-place multi-start ascent of the seeds xs (device fp32 [k, d]) in ONE launch (plx_gp_ascent, fused
        posterior, n <= 64); returns the device fp32 [k] acquisition values at the final points."""
        t = self.torch
        Xd, L, alpha, _, _ = dev_state
        k, d = xs.shape
        fx = t.empty(k, dtype=t.float32, device=self.device)
        rc = self.lib.plx_gp_ascent(xs.data_ptr(), fx.data_ptr(), k, lo.data_ptr(), hi.data_ptr(), Xd.data_ptr(),
                                    Xd.shape[0], d, L.data_ptr(), alpha.data_ptr(), KIND_IDS[gp.kind], float(gp.ls),
                                    float(gp.nu), float(matern_c(gp.nu)) if gp.kind == "matern_nu" else 0.0, 1.0,
                                    {"ucb": 0, "ei": 1, "poi": 2}[acq], float(kappa), float(eps), float(y_max),
                                    int(steps), *self.table(gp.kind, gp.nu), self._stream())
        self._native.check(rc, "plx_gp_ascent")
        return fx

    def predict_acq(self, gp: GPState, dev_state, Xc, acq: str, y_max: float, kappa: float, eps: float,
                    want_mean_std: bool = False):
        t = self.torch
        Xc = t.as_tensor(Xc, dtype=t.float32, device=self.device).contiguous()
        m = Xc.shape[0]
        mean = t.empty(m, dtype=t.float32, device=self.device) if want_mean_std else None
        std = t.empty(m, dtype=t.float32, device=self.device) if want_mean_std else None
        out = self.acq_dev(gp, dev_state, Xc, acq, y_max, kappa, eps, mean, std)
        return out, int(t.argmax(out).item()), mean, std


# ================================================================================ utility function / optimizer
class UtilityFunction:
    def __init__(self, config, seed: Optional[int] = None, backend: str = "auto"):
        self.config = config
        self.acquisition_function = config.acquisition_function
        self.kappa = config.kappa if config.kappa is not None else 2.576
        self.eps = config.eps if config.eps is not None else 0.0
        self.random_generator = get_random_generator(seed)
        self.backend = backend
        self.gp_config = config.gaussian_process
        self.gaussian_process = None
        self._gp: Optional[GPState] = None
        self._hip: Optional[HipGP] = None
        self._dev = None

    @staticmethod
    def resolve_backend(backend: str) -> str:
        """``auto``: the HIP kernels when this process may do device work and has a GPU, else numpy.  The polyflow
        scheduler process forbids device work (:func:`set_device_allowed`): it must never initialise HIP -- its
        GP work runs on a resident executor of the group (``bo_suggest``), or on numpy."""
        if backend != "auto":
            return backend
        if not device_allowed():
            return "numpy"
        try:
            import torch

            return "hip" if torch.cuda.is_available() else "numpy"
        except Exception:
            return "numpy"

    def fit(self, X: np.ndarray, y: np.ndarray) -> None:
        self.backend = self.resolve_backend(self.backend)
        g = self.gp_config
        if self.backend == "reference":
            from sklearn.gaussian_process import GaussianProcessRegressor
            from sklearn.gaussian_process.kernels import RBF, Matern

            kernel = RBF(length_scale=g.length_scale) if g.kernel == "rbf" else Matern(length_scale=g.length_scale,
                                                                                      nu=g.nu)
            self.gaussian_process = GaussianProcessRegressor(kernel=kernel,
                                                             n_restarts_optimizer=g.n_restarts_optimizer,
                                                             random_state=self.random_generator)
            self.gaussian_process.fit(X, y)
            return
        if self.backend == "hip":
            if self._hip is None:
                self._hip = HipGP()
            kind = _kind(g.kernel, g.nu)
            ls = self._hip.fit_length_scale(X, y, kind, g.nu, g.length_scale) if len(X) > 1 else float(g.length_scale)
            self._gp = GPState(np.asarray(X, dtype=np.float64), np.asarray(y, dtype=np.float64), ls, kind, g.nu,
                               None, None, float("nan"))
            self._dev = self._hip.fit(self._gp)
            return
        self._gp = fit_gp(X, y, kernel=g.kernel, nu=g.nu, length_scale=g.length_scale)

    def compute(self, x: np.ndarray, y_max: float) -> np.ndarray:
        acq = self.acquisition_function
        if self.backend == "reference":
            mean, std = self.gaussian_process.predict(x, return_std=True)
        elif self.backend == "hip":
            out, _, _, _ = self._hip.predict_acq(self._gp, self._dev, x, acq, y_max, self.kappa, self.eps)
            return out.cpu().numpy().astype(np.float64)
        else:
            mean, std = predict_np(self._gp, np.asarray(x, dtype=np.float64))
        return acquisition_np(mean, std, acq, y_max, self.kappa, self.eps)

    def max_compute(self, y_max: float, bounds: np.ndarray, n_warmup: int, n_iter: int) -> np.ndarray:
        rng = self.random_generator
        if self.backend in ("reference", "numpy") and not (self.backend == "numpy" and n_warmup > 5000):
            from scipy.optimize import minimize

            x_tries = rng.uniform(bounds[:, 0], bounds[:, 1], size=(n_warmup, bounds.shape[0]))
            ys = self.compute(x_tries, y_max)
            x_max, max_acq = x_tries[ys.argmax()], ys.max()
            for x_try in rng.uniform(bounds[:, 0], bounds[:, 1], size=(n_iter, bounds.shape[0])):
                res = minimize(lambda x: -float(self.compute(x.reshape(1, -1), y_max)[0]), x_try,
                               bounds=bounds, method="L-BFGS-B")
                if not res.success:
                    continue
                val = -float(np.ravel(res.fun)[0])
                if max_acq is None or val >= max_acq:
                    x_max, max_acq = res.x, val
            return np.clip(x_max, bounds[:, 0], bounds[:, 1])
        if self.backend == "hip":
            return self._max_compute_device(y_max, bounds, n_warmup, n_iter)
        # batched search (numpy backend with a large warm-up): one evaluation per round over all candidates
        d = bounds.shape[0]
        lo, hi = bounds[:, 0], bounds[:, 1]
        width = np.maximum(hi - lo, 1e-12)
        cand = rng.uniform(lo, hi, size=(max(n_warmup, 1), d))
        ys = self.compute(cand, y_max)
        order = np.argsort(-ys)[:max(1, min(64, len(cand)))]
        top, top_v = cand[order], ys[order]
        x_max, max_acq = top[0], top_v[0]
        scale = 0.1
        for _ in range(max(n_iter, 1)):
            pert = top[rng.randint(0, len(top), size=4096)] + rng.normal(0, 1, size=(4096, d)) * width * scale
            pert = np.clip(pert, lo, hi)
            yp = self.compute(pert, y_max)
            allx, allv = np.concatenate([top, pert]), np.concatenate([top_v, yp])
            keep = np.argsort(-allv)[:len(top)]
            top, top_v = allx[keep], allv[keep]
            if top_v[0] >= max_acq:
                x_max, max_acq = top[0], top_v[0]
            scale *= 0.7
        # batched multi-start projected gradient ascent (the reference's L-BFGS-B restarts, all seeds at once):
        # central differences for every seed and coordinate are ONE acquisition evaluation per step
        seeds = np.concatenate([x_max[None], top[1:16]])
        xs, fx = self._ascend(seeds, y_max, lo, hi, width)
        i = int(np.argmax(fx))
        if fx[i] >= max_acq:
            x_max = xs[i]
        return np.clip(x_max, lo, hi)

    def _ascend(self, xs: np.ndarray, y_max: float, lo, hi, width, steps: int = 25):
        k, d = xs.shape
        h = 1e-4 * width
        step = 0.05 * width
        fx = self.compute(xs, y_max)
        eye = np.eye(d)
        for _ in range(steps):
            probe = np.concatenate([(xs[:, None, :] + eye[None] * h), (xs[:, None, :] - eye[None] * h)], axis=1)
            fp = self.compute(np.clip(probe.reshape(-1, d), lo, hi), y_max).reshape(k, 2 * d)
            grad = (fp[:, :d] - fp[:, d:]) / (2 * h)
            gn = np.linalg.norm(grad / width, axis=1, keepdims=True)
            cand = np.clip(xs + step * grad / width / np.maximum(gn, 1e-30) * width, lo, hi)
            fc = self.compute(cand, y_max)
            better = fc > fx
            xs = np.where(better[:, None], cand, xs)
            fx = np.where(better, fc, fx)
            step = np.where(better[:, None], step * 1.2, step * 0.5)
        return xs, fx

    def _max_compute_device(self, y_max: float, bounds: np.ndarray, n_warmup: int, n_iter: int,
                            ascent_steps: int = 25) -> np.ndarray:
        """The same search as the batched numpy path, held on the device end to end: random warm-up, refinement
        rounds around the running top-64, then multi-start finite-difference ascent.  Candidates, acquisition
        values, top-k and the incumbent never leave HBM; the only host readback is the final argmax point."""
        import torch as t

        hip, gp, dev = self._hip, self._gp, self._dev
        device = hip.device
        acq, kappa, eps = self.acquisition_function, self.kappa, self.eps
        g = t.Generator(device=device)
        g.manual_seed(int(self.random_generator.randint(0, 2 ** 31 - 1)))
        d = bounds.shape[0]
        f32 = dict(dtype=t.float32, device=device)
        lo, hi = t.tensor(bounds[:, 0], **f32), t.tensor(bounds[:, 1], **f32)
        width = (hi - lo).clamp_min(1e-12)

        def f(x):
            return hip.acq_dev(gp, dev, x.contiguous(), acq, y_max, kappa, eps)

        cand = lo + width * t.rand((max(n_warmup, 1), d), generator=g, **f32)
        ys = f(cand)
        top_v, ti = t.topk(ys, min(64, ys.shape[0]))
        top = cand[ti]
        x_max, max_acq = top[0], top_v[0]
        scale = 0.1
        for _ in range(max(n_iter, 1)):
            idx = t.randint(0, top.shape[0], (4096,), generator=g, device=device)
            pert = t.minimum(t.maximum(top[idx] + t.randn((4096, d), generator=g, **f32) * width * scale, lo), hi)
            yp = f(pert)
            allv = t.cat([top_v, yp])
            top_v, keep = t.topk(allv, top.shape[0])
            top = t.cat([top, pert])[keep]
            x_max = t.where(top_v[0] >= max_acq, top[0], x_max)
            max_acq = t.maximum(max_acq, top_v[0])
            scale *= 0.7
        xs = t.cat([x_max[None], top[1:16]]).contiguous()
        k = xs.shape[0]
        if hip.fused(dev):  # the whole ascent in one launch
            fx = hip.ascent(gp, dev, xs, lo, hi, acq, y_max, kappa, eps, ascent_steps)
        else:
            fx = f(xs)
            h = 1e-4 * width
            step = (0.05 * width).expand(k, d).clone()
            eye = t.eye(d, **f32)
            for _ in range(ascent_steps):
                probe = t.cat([xs[:, None, :] + eye[None] * h, xs[:, None, :] - eye[None] * h], dim=1).reshape(-1, d)
                fp = f(t.minimum(t.maximum(probe, lo), hi)).reshape(k, 2 * d)
                grad = (fp[:, :d] - fp[:, d:]) / (2 * h)
                gn = (grad / width).norm(dim=1, keepdim=True).clamp_min(1e-30)
                c = t.minimum(t.maximum(xs + step * grad / gn, lo), hi)
                fc = f(c)
                better = fc > fx
                xs = t.where(better[:, None], c, xs)
                fx = t.where(better, fc, fx)
                step = t.where(better[:, None], step * 1.2, step * 0.5)
        i = t.argmax(fx)
        x_max = t.where(fx[i] >= max_acq, xs[i], x_max)
        return np.clip(x_max.double().cpu().numpy(), bounds[:, 0], bounds[:, 1])


class BOOptimizer:
    def __init__(self, hptuning_config: HPTuningConfig, backend: str = "auto"):
        self.hptuning_config = hptuning_config
        bo = hptuning_config.bo
        self.n_initial_trials = bo.n_initial_trials
        self.space = SearchSpace(hptuning_config)
        self.utility_function = UtilityFunction(bo.utility_function, seed=hptuning_config.seed, backend=backend)
        resolved = UtilityFunction.resolve_backend(backend)
        device_path = resolved == "hip"
        self.n_warmup = bo.utility_function.n_warmup or (100000 if device_path else 5)
        self.n_iter = bo.utility_function.n_iter or (8 if device_path else 10)

    def add_observations(self, configs, metrics) -> None:
        self.space.add_observations(configs, metrics)

    def _maximize(self, pending: Optional[Sequence] = None):
        if not self.space.is_observations_valid():
            return None
        X, y = self.space.x, self.space.y
        y_max = float(y.max())
        if pending is not None and len(pending):
            # constant liar: pretend pending points returned the current mean of y
            X = np.vstack([X, np.asarray(pending)])
            y = np.concatenate([y, np.full(len(pending), float(np.mean(self.space.y)))])
        self.utility_function.fit(X, y)
        return self.utility_function.max_compute(y_max, self.space.bounds, self.n_warmup, self.n_iter)

    def get_suggestion(self) -> Optional[Dict[str, Any]]:
        return self.space.get_suggestion(self._maximize())

    def get_suggestions(self, n: int) -> List[Dict[str, Any]]:
        out, pending = [], []
        for _ in range(n):
            x = self._maximize(pending)
            if x is None:
                break
            pending.append(x)
            out.append(self.space.get_suggestion(x))
        return out


@dataclass
class BOIterationConfig:
    """Reference hpsearch/schemas/bayesian_optimization.py:35-70 (``combined_*`` without its aliasing bug)."""
    iteration: int
    old_experiment_ids: List[int] = field(default_factory=list)
    old_experiments_configs: List[Tuple[int, Dict]] = field(default_factory=list)
    old_experiments_metrics: List[Tuple[int, float]] = field(default_factory=list)
    experiment_ids: List[int] = field(default_factory=list)
    experiments_configs: List[Tuple[int, Dict]] = field(default_factory=list)
    experiments_metrics: List[Tuple[int, float]] = field(default_factory=list)

    @property
    def combined_experiment_ids(self):
        return list(self.old_experiment_ids) + list(self.experiment_ids)

    @property
    def combined_experiments_configs(self):
        return list(self.old_experiments_configs) + list(self.experiments_configs)

    @property
    def combined_experiments_metrics(self):
        return list(self.old_experiments_metrics) + list(self.experiments_metrics)

    @classmethod
    def from_dict(cls, d):
        return cls(**{k: d.get(k, [] if k != "iteration" else 0) for k in cls.__dataclass_fields__})


class BOSearchManager(BaseSearchAlgorithmManager):
    NAME = SearchAlgorithms.BO

    def __init__(self, hptuning_config: HPTuningConfig, backend: str = "auto"):
        super().__init__(hptuning_config)
        self.n_initial_trials = hptuning_config.bo.n_initial_trials
        self.n_iterations = hptuning_config.bo.n_iterations
        self.backend = backend

    def get_suggestions(self, iteration_config=None, n: Optional[int] = None):
        """``n``: batch size of a BO iteration (default ``bo.n_suggestions``; a resident group asks for enough to
        fill its concurrency, constant liar)."""
        cfg = self.hptuning_config
        if not iteration_config:
            return get_random_suggestions(cfg.matrix, self.n_initial_trials, seed=cfg.seed)
        configs_by_id = dict(iteration_config.combined_experiments_configs)
        metrics_by_id = dict(iteration_config.combined_experiments_metrics)
        configs, metrics = [], []
        for key in metrics_by_id:
            configs.append(configs_by_id[key])
            metrics.append(metrics_by_id[key])
        return suggest(cfg, configs, metrics, n if n is not None else cfg.bo.n_suggestions, self.backend) or None

    def should_reschedule(self, iteration: int) -> bool:
        return iteration < self.n_iterations


def suggest(cfg: HPTuningConfig, configs: List[Dict[str, Any]], metrics: List[float], n: int,
            backend: str = "auto") -> List[Dict[str, Any]]:
    """One BO iteration's suggestions (``n`` > 1: a constant-liar batch) from the finished trials' configs and
    metrics -- what BOSearchManager.get_suggestions computes, callable where the GPU is (a resident executor's
    ``bo_suggest`` op)."""
    opt = BOOptimizer(cfg, backend=backend)
    opt.add_observations(configs, metrics)
    n = max(1, int(n))
    sugg = opt.get_suggestions(n) if n > 1 else [opt.get_suggestion()]
    return [s for s in sugg if s]
