"""Counter-based random-search sampler: Philox4x32-10 on the device (csrc/polytune_kernels.hip,
``plx_philox_sample``) with a bit-exact numpy twin on the host.

Reference behaviour: ``get_random_suggestions`` (polyaxon/hpsearch/search_managers/utils.py:41-64) draws every
matrix distribution from a seeded ``numpy.random.RandomState`` one suggestion at a time, de-duplicates, and caps
the count at the size of an all-discrete space.  That sequential stream is kept as the default (reference parity,
``polytune.utils.get_random_suggestions``).  This sampler is the SURVEY §2.2 alternative selected with
``hptuning.random_search.sampler: device``: suggestion ``r``, parameter ``p`` of seed ``s`` is
``Philox4x32-10(counter=(r, p, const), key=s)``, so a suggestion does not depend on how many were drawn before it
or on which device drew it -- a 10^6-suggestion search is one kernel launch, the host only de-duplicates.

Per-distribution mapping (same conventions as ``spec.matrix.MatrixConfig.sample``): uniform / loguniform draw a
53-bit uniform on [low, high) (then exp); normal / lognormal use Box-Muller on two 53-bit uniforms (then exp);
``q*`` variants round to the nearest multiple of q (half to even, like numpy); discrete options (values, range,
linspace, logspace, geomspace) draw an index uniformly; ``pvalues`` inverts the cumulative probabilities.
"""
from __future__ import annotations

import ctypes
import copy
from typing import Any, Dict, List, Optional

import numpy as np

from polyaxon_amd.spec.matrix import MatrixConfig, space_size

_M0, _M1 = np.uint32(0xD2511F53), np.uint32(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_TAG = 0x5A3E1E5


class _Desc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("log", ctypes.c_int), ("count", ctypes.c_int), ("cdf", ctypes.c_int),
                ("a", ctypes.c_double), ("b", ctypes.c_double), ("q", ctypes.c_double)]


def _mulhilo(m: np.uint32, x: np.ndarray):
    p = x.astype(np.uint64) * np.uint64(m)
    return (p >> np.uint64(32)).astype(np.uint32), (p & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11) on uint32 arrays; returns the four output words."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint32).copy() for c in (c0, c1, c2, c3))
    k0, k1 = np.uint32(k0 & 0xFFFFFFFF), np.uint32(k1 & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            hi0, lo0 = _mulhilo(_M0, c0)
            hi1, lo1 = _mulhilo(_M1, c2)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def _u53(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return (((a >> np.uint32(5)).astype(np.uint64) << np.uint64(26)) | (b >> np.uint32(6)).astype(np.uint64)) \
        .astype(np.float64) * (1.0 / 9007199254740992.0)


class PhiloxSampler:
    """Samples suggestion rows of a matrix; ``values(rows)`` maps the raw fp64 draws to parameter dicts."""

    def __init__(self, matrix: Dict[str, MatrixConfig]):
        self.keys = sorted(matrix)
        self.matrix = matrix
        self.descs: List[_Desc] = []
        cdf: List[float] = []
        self.tables: List[Optional[np.ndarray]] = []
        for k in self.keys:
            m = matrix[k]
            o = m.option
            if o == "pvalues":
                probs = np.asarray(m.probs, dtype=np.float64)
                c = np.cumsum(probs / probs.sum())
                c[-1] = 1.0
                self.descs.append(_Desc(3, 0, len(c), len(cdf), 0.0, 0.0, 0.0))
                cdf.extend(c.tolist())
                self.tables.append(np.asarray(m.values, dtype=object))
            elif m.is_discrete:
                vals = m.to_numpy()
                self.descs.append(_Desc(2, 0, len(vals), 0, 0.0, 0.0, 0.0))
                self.tables.append(vals)
            else:
                a = m.args
                kind = 0 if o in ("uniform", "quniform", "loguniform", "qloguniform") else 1
                log = int(o in ("loguniform", "qloguniform", "lognormal", "qlognormal"))
                q = float(a[2]) if o.startswith("q") else 0.0
                self.descs.append(_Desc(kind, log, 0, 0, float(a[0]), float(a[1]), q))
                self.tables.append(None)
        self.cdf = np.asarray(cdf if cdf else [1.0], dtype=np.float64)

    # ------------------------------------------------------------------ raw draws [n, P] (fp64)
    def draw_host(self, n: int, seed: int, row0: int = 0) -> np.ndarray:
        P = len(self.descs)
        rows = np.arange(row0, row0 + n, dtype=np.uint64)
        r_lo = (rows & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        r_hi = (rows >> np.uint64(32)).astype(np.uint32)
        out = np.empty((n, P), dtype=np.float64)
        for p, d in enumerate(self.descs):
            w0, w1, w2, w3 = philox4x32_10(r_lo, r_hi, np.full(n, p, np.uint32), np.full(n, _TAG, np.uint32),
                                           seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
            u = _u53(w0, w1)
            if d.kind == 0:
                v = d.a + (d.b - d.a) * u
            elif d.kind == 1:
                v = d.a + d.b * np.sqrt(-2.0 * np.log(1.0 - u)) * np.cos(6.283185307179586 * _u53(w2, w3))
            elif d.kind == 2:
                v = np.minimum(np.floor(u * d.count), d.count - 1)
            else:
                c = self.cdf[d.cdf: d.cdf + d.count]
                v = np.minimum(np.searchsorted(c, u, side="right"), d.count - 1).astype(np.float64)
            if d.kind <= 1:
                if d.log:
                    v = np.exp(v)
                if d.q > 0:
                    v = np.round(v / d.q) * d.q
            out[:, p] = v
        return out

    def draw_device(self, n: int, seed: int, row0: int = 0, device=None):
        import torch

        from polyaxon_amd.ops import _native

        lib = _native.lib("plx_polytune")
        assert int(lib.plx_philox_desc_size()) == ctypes.sizeof(_Desc)
        dev = torch.device(device or "cuda")
        raw = bytes((_Desc * len(self.descs))(*self.descs))
        desc = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
        cdf = torch.as_tensor(self.cdf, device=dev)
        out = torch.empty((n, len(self.descs)), dtype=torch.float64, device=dev)
        rc = lib.plx_philox_sample(desc.data_ptr(), cdf.data_ptr(), len(self.descs), int(n), int(row0),
                                   int(seed) & 0xFFFFFFFFFFFFFFFF, out.data_ptr(),
                                   torch.cuda.current_stream(dev).cuda_stream)
        _native.check(rc, "plx_philox_sample")
        return out

    def values(self, raw: np.ndarray) -> List[Dict[str, Any]]:
        cols = []
        for p, k in enumerate(self.keys):
            t = self.tables[p]
            col = raw[:, p]
            if t is None:
                cols.append([float(x) for x in col])
            else:
                idx = col.astype(np.int64)
                cols.append([t[i].item() if hasattr(t[i], "item") else t[i] for i in idx])
        return [{k: cols[p][i] for p, k in enumerate(self.keys)} for i in range(raw.shape[0])]


def philox_random_suggestions(matrix: Dict[str, MatrixConfig], n_suggestions: int,
                              suggestion_params: Optional[Dict] = None, seed: Optional[int] = None,
                              device: Optional[str] = "auto") -> List[Dict[str, Any]]:
    """``get_random_suggestions`` semantics (dedup, cap at the size of an all-discrete space) over the Philox
    stream: drawn on the GPU when one is available (``device='auto'``), else by the bit-exact host twin."""
    if not n_suggestions:
        raise ValueError("This search algorithm requires `n_experiments`.")
    size = space_size(matrix)
    if size is not None:
        n_suggestions = min(n_suggestions, size)
    sampler = PhiloxSampler(matrix)
    seed = int(seed) if seed else 0
    use_dev = False
    if device == "auto":
        try:
            import torch

            use_dev = torch.cuda.is_available()
        except Exception:
            use_dev = False
    elif device:
        use_dev = True
    out: List[Dict[str, Any]] = []
    seen = set()
    row0, want = 0, n_suggestions
    while want > 0:
        n = max(want, 1024) if size is not None else want   # discrete spaces collide: draw ahead
        raw = sampler.draw_device(n, seed, row0).cpu().numpy() if use_dev else sampler.draw_host(n, seed, row0)
        row0 += n
        for vals in sampler.values(raw):
            key = tuple(sorted((k, repr(v)) for k, v in vals.items()))
            if key in seen:
                continue
            seen.add(key)
            params = copy.deepcopy(suggestion_params or {})
            params.update(vals)
            out.append(params)
            want -= 1
            if want == 0:
                break
    return out
