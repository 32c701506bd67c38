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
        for key in sorted(hptuning_config.matrix):
            v = hptuning_config.matrix[key]
            self.features.append(key)
            if v.is_categorical:
                values = v.to_numpy()
                for _ in range(len(values)):
                    bounds.append((0, 1))
                self.categorical_features[key] = {"values": values, "number": len(values)}
                self.dim += len(values)
            elif v.is_discrete:
                bounds.append((v.min, v.max))
                self.discrete_features[key] = {"values": v.to_numpy()}
                self.dim += 1
            else:
                bounds.append((float(v.min), float(v.max)))
                self.dim += 1
        self.bounds = np.asarray(bounds, dtype=np.float64)

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
                    row.append(cfg[f])
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
                v = vals[int(np.argmin(np.abs(np.subtract(vals, x[c]))))]
                c += 1
            elif f in self.categorical_features:
                n = self.categorical_features[f]["number"]
                v = self.categorical_features[f]["values"][int(np.argmax(x[c:c + n]))]
                c += n
            else:
                v = x[c]
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

    Gram matrices are always built by our kernels; fp64 factorisations above ``DEVICE_FACTOR_MAX`` rows run
    through LAPACK on the host (a one-off D2H of the Gram): torch's device Cholesky faulted the GPU at n = 1000
    on this ROCm build (scripts/diag_bo1000.py), while n <= 128 goes through our LDS Cholesky or torch."""

    DEVICE_FACTOR_MAX = 128

    def __init__(self, device=None):
        import torch

        self.torch = torch
        self.device = torch.device(device or "cuda")
        from polyaxon_amd.ops import _native

        self.lib = _native.lib("plx_gp")
        self._native = _native

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
                                  self._stream())
        self._native.check(rc, "plx_gp_kmat")
        return K

    def cholesky(self, K):
        t = self.torch
        n = K.shape[0]
        if n > 128:
            try:
                L = np.linalg.cholesky(K.double().cpu().numpy())
            except np.linalg.LinAlgError as e:
                raise np.linalg.LinAlgError(str(e))
            return t.as_tensor(L, dtype=t.float32, device=self.device)
        status = t.zeros(1, dtype=t.int32, device=self.device)
        out = K.clone()
        rc = self.lib.plx_gp_chol(out.data_ptr(), n, n, status.data_ptr(), self._stream())
        self._native.check(rc, "plx_gp_chol")
        if int(status.item()) != 0:
            raise np.linalg.LinAlgError(f"not positive definite at column {int(status.item())}")
        return out

    def lml_batch(self, X, y, kind: str, nu: float, log_ls, alpha: float = 1e-10):
        """Log marginal likelihood at every length scale exp(log_ls): ONE fp64 Gram launch for the whole batch
        (plx_gp_kmat_batch_f64), fp64 Cholesky per scale, one batched solve."""
        t = self.torch
        Xd = t.as_tensor(np.ascontiguousarray(X, dtype=np.float64), device=self.device)
        yd = t.as_tensor(y, dtype=t.float64, device=self.device)
        n, d = Xd.shape
        nb = len(log_ls)
        inv = t.tensor([math.exp(-2.0 * float(l)) for l in log_ls], dtype=t.float64, device=self.device)
        Ks = t.empty((nb, n, n), dtype=t.float64, device=self.device)
        rc = self.lib.plx_gp_kmat_batch_f64(Xd.data_ptr(), n, d, inv.data_ptr(), nb, Ks.data_ptr(), KIND_IDS[kind],
                                            float(nu), float(matern_c(nu)) if kind == "matern_nu" else 0.0,
                                            float(alpha), self._stream())
        self._native.check(rc, "plx_gp_kmat_batch_f64")
        if n > self.DEVICE_FACTOR_MAX:
            return self._lml_host(Ks.cpu().numpy(), np.asarray(y, dtype=np.float64))
        # one factorisation per scale: a batched cholesky_ex on ROCm does not keep the other batch entries
        # valid once one of them is not positive definite (measured: wrong LMLs beside a failing entry)
        Ls, oks = [], []
        for b in range(nb):
            Lb, ib = t.linalg.cholesky_ex(Ks[b])
            Ls.append(Lb)
            oks.append(ib == 0)
        L, ok = t.stack(Ls), t.stack(oks)
        L = t.where(ok[:, None, None], L, t.eye(n, dtype=L.dtype, device=self.device).expand_as(L))
        a = t.cholesky_solve(yd[None, :, None].expand(nb, n, 1).contiguous(), L)[..., 0]
        lml = -0.5 * (a * yd[None]).sum(1) - t.log(t.diagonal(L, dim1=1, dim2=2)).sum(1) - 0.5 * n * math.log(2 * math.pi)
        lml = t.where(ok & t.isfinite(lml), lml, t.full_like(lml, -math.inf))
        return lml.cpu().numpy()

    @staticmethod
    def _lml_host(Ks: np.ndarray, y: np.ndarray) -> np.ndarray:
        """fp64 LAPACK factorisations of device-built Gram matrices (sklearn semantics: not PD -> -inf)."""
        out = np.full(Ks.shape[0], -np.inf)
        n = Ks.shape[1]
        for b in range(Ks.shape[0]):
            try:
                L = np.linalg.cholesky(Ks[b])
            except np.linalg.LinAlgError:
                continue
            from scipy.linalg import cho_solve

            a = cho_solve((L, True), y)
            v = -0.5 * float(y @ a) - float(np.log(np.diag(L)).sum()) - 0.5 * n * math.log(2 * math.pi)
            out[b] = v if math.isfinite(v) else -np.inf
        return out

    def fit_length_scale(self, X, y, kind: str, nu: float, length_scale: float, alpha: float = 1e-10,
                         bounds=(1e-5, 1e5), coarse: int = 24, rounds: int = 3) -> float:
        """Maximise the LML over log length scale on the device: a coarse batched grid over the bounds (plus the
        configured initial value, as sklearn always tries it), then batched zoom rounds around the best point.
        Replaces the host 1-D search, whose O(n^3) factorisations dominate a suggestion at n ~ 1000."""
        lo, hi = math.log(bounds[0]), math.log(bounds[1])
        grid = list(np.linspace(lo, hi, coarse)) + [math.log(length_scale)]
        vals = self.lml_batch(X, y, kind, nu, grid, alpha)
        best = int(np.argmax(vals))
        x_best, f_best = grid[best], vals[best]
        step = (hi - lo) / (coarse - 1)
        for _ in range(rounds):
            g = list(np.linspace(max(lo, x_best - step), min(hi, x_best + step), 9))
            v = self.lml_batch(X, y, kind, nu, g, alpha)
            i = int(np.argmax(v))
            if v[i] > f_best:
                x_best, f_best = g[i], v[i]
            step /= 4.0
        return math.exp(x_best) if math.isfinite(f_best) else float(length_scale)

    def fit(self, gp: GPState):
        """Device factors for a fitted GP (length scale from the LML search): (X, L, alpha, L^-1 or None).

        n <= DEVICE_FACTOR_MAX: our LDS Cholesky + device triangular solves.  Larger n: the Gram comes from our
        kernel, the fp64 factorisation, alpha and the explicit L^-1 from LAPACK; the posterior variance then
        needs only a GEMM (v = L^-1 k*^T) on the device instead of a triangular solve."""
        t = self.torch
        n = len(gp.X)
        K = self.kmat(gp.X, gp.X, gp.kind, gp.ls, gp.nu, diag=1e-10)
        Xd = t.as_tensor(gp.X, dtype=t.float32, device=self.device).contiguous()
        if n > self.DEVICE_FACTOR_MAX:
            from scipy.linalg import cho_solve, solve_triangular

            Kh = K.double().cpu().numpy()
            jitter = 0.0
            for _ in range(8):
                try:
                    Lh = np.linalg.cholesky(Kh + jitter * np.eye(n) if jitter else Kh)
                    break
                except np.linalg.LinAlgError:
                    jitter = max(jitter * 10, 1e-8)
            else:
                raise np.linalg.LinAlgError("GP Gram matrix not positive definite")
            ah = cho_solve((Lh, True), np.asarray(gp.y, dtype=np.float64))
            Linv = solve_triangular(Lh, np.eye(n), lower=True)
            f32 = dict(dtype=t.float32, device=self.device)
            return Xd, t.as_tensor(Lh, **f32).contiguous(), t.as_tensor(ah, **f32).contiguous(), \
                t.as_tensor(Linv, **f32).contiguous()
        jitter = 0.0
        for _ in range(6):
            try:
                L = self.cholesky(K if jitter == 0 else K + jitter * t.eye(K.shape[0], device=self.device))
                break
            except np.linalg.LinAlgError:
                jitter = max(jitter * 10, 1e-8)
        y = t.as_tensor(gp.y, dtype=t.float32, device=self.device)
        alpha = t.cholesky_solve(y[:, None], L)[:, 0]
        return Xd, L.contiguous(), alpha.contiguous(), None

    def predict_acq(self, gp: GPState, dev_state, Xc, acq: str, y_max: float, kappa: float, eps: float,
                    want_mean_std: bool = False):
        t = self.torch
        Xd, L, alpha, Linv = dev_state
        Xc = t.as_tensor(Xc, dtype=t.float32, device=self.device).contiguous()
        m, n, d = Xc.shape[0], Xd.shape[0], Xd.shape[1]
        acq_id = {"ucb": 0, "ei": 1, "poi": 2}[acq]
        out = t.empty(m, dtype=t.float32, device=self.device)
        mean = t.empty(m, dtype=t.float32, device=self.device) if want_mean_std else None
        std = t.empty(m, dtype=t.float32, device=self.device) if want_mean_std else None
        nblk = (m + 255) // 256
        bb = t.empty(nblk, dtype=t.float32, device=self.device)
        bi = t.empty(nblk, dtype=t.int32, device=self.device)
        if n <= 64 and d <= 16:
            rc = self.lib.plx_gp_predict_acq(
                Xc.data_ptr(), m, Xd.data_ptr(), n, d, L.data_ptr(), n, alpha.data_ptr(), KIND_IDS[gp.kind],
                float(gp.ls), float(gp.nu), float(matern_c(gp.nu)) if gp.kind == "matern_nu" else 0.0, 1.0, acq_id,
                float(kappa), float(eps), float(y_max), out.data_ptr(), mean.data_ptr() if mean is not None else None,
                std.data_ptr() if std is not None else None, bb.data_ptr(), bi.data_ptr(), self._stream())
            self._native.check(rc, "plx_gp_predict_acq")
            best = int(bi[int(t.argmax(bb))].item())
        else:  # large n: MFMA cross-kernel + TRSM, acquisition in torch
            Ks = self.kmat(Xc, Xd, gp.kind, gp.ls, gp.nu)
            mu = Ks @ alpha
            v = Linv @ Ks.T if Linv is not None else t.linalg.solve_triangular(L, Ks.T, upper=False)
            sd = (1.0 - (v * v).sum(0)).clamp_min(0).sqrt()
            out = self._acq_torch(mu, sd, acq, y_max, kappa, eps)
            best = int(t.argmax(out).item())
            mean, std = mu, sd
        return out, best, mean, std

    def _acq_torch(self, mu, sd, acq, y_max, kappa, eps):
        t = self.torch
        if acq == "ucb":
            return mu + kappa * sd
        z = t.where(sd > 0, (mu - y_max - eps) / sd.clamp_min(1e-30), t.zeros_like(sd))
        cdf = 0.5 * t.erfc(-z / math.sqrt(2))
        if acq == "poi":
            return cdf
        return (mu - y_max - eps) * cdf + sd * t.exp(-0.5 * z * z) / math.sqrt(2 * math.pi)


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
        if backend != "auto":
            return backend
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
        # batched device search: one kernel launch per round over all candidates
        d = bounds.shape[0]
        lo, hi = bounds[:, 0], bounds[:, 1]
        width = np.maximum(hi - lo, 1e-12)
        cand = rng.uniform(lo, hi, size=(max(n_warmup, 1), d))
        ys = self.compute(cand, y_max)
        best_i = int(np.argmax(ys))
        x_max, max_acq = cand[best_i], ys[best_i]
        top = cand[np.argsort(-ys)[:max(1, min(64, len(cand)))]]
        scale = 0.1
        for _ in range(max(n_iter, 1)):
            pert = top[rng.randint(0, len(top), size=4096)] + rng.normal(0, 1, size=(4096, d)) * width * scale
            pert = np.clip(pert, lo, hi)
            yp = self.compute(pert, y_max)
            order = np.argsort(-yp)
            if yp[order[0]] >= max_acq:
                x_max, max_acq = pert[order[0]], yp[order[0]]
            top = np.concatenate([top, pert[order[:64]]])[: 128]
            scale *= 0.7
        # batched multi-start projected gradient ascent (the reference's L-BFGS-B restarts, all seeds at once):
        # central differences for every seed and coordinate are ONE acquisition launch per step
        seeds = np.concatenate([x_max[None], top[:15]])
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

    def get_suggestions(self, iteration_config=None):
        cfg = self.hptuning_config
        if not iteration_config:
            return get_random_suggestions(cfg.matrix, self.n_initial_trials, seed=cfg.seed)
        configs_by_id = dict(iteration_config.combined_experiments_configs)
        metrics_by_id = dict(iteration_config.combined_experiments_metrics)
        configs, metrics = [], []
        for key in metrics_by_id:
            configs.append(configs_by_id[key])
            metrics.append(metrics_by_id[key])
        opt = BOOptimizer(cfg, backend=self.backend)
        opt.add_observations(configs, metrics)
        n = max(1, cfg.bo.n_suggestions)
        sugg = opt.get_suggestions(n) if n > 1 else [opt.get_suggestion()]
        sugg = [s for s in sugg if s]
        return sugg or None

    def should_reschedule(self, iteration: int) -> bool:
        return iteration < self.n_iterations
