"""Python entry points for the polytune bracket kernels (csrc/polytune_kernels.hip).

``BracketMetrics`` is the device-resident [brackets × configs] metric tensor that trial executors write
into (``plx_commit_metric``); ``topk_order`` sorts every bracket in one launch; ``early_stop_any``
evaluates all early-stopping rules in one launch.  CPU tensors take the numpy path, which is also the
parity reference for the GPU tests.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from polyaxon_amd.ops import _native
from polyaxon_amd.polytune.utils import early_stop_any_host


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def topk_order(metrics: torch.Tensor, counts: torch.Tensor, maximize: bool,
               host_counts: Optional[Sequence[int]] = None) -> torch.Tensor:
    """Per-row stable ordering (best first) of the first ``counts[b]`` entries of ``metrics[b]``.
    NaN entries sort last; slots beyond ``counts[b]`` are -1.  ``host_counts`` (the same counts, known on the
    host) lets the bound check skip a device->host read, so the launch does not synchronise."""
    if metrics.dim() != 2:
        raise ValueError("metrics must be [brackets, configs]")
    B, C = metrics.shape
    if metrics.is_cuda:
        metrics = metrics.contiguous().float()
        counts = counts.to(device=metrics.device, dtype=torch.int32).contiguous()
        top = max(host_counts, default=0) if host_counts is not None else int(counts.max().item() if B else 0)
        if counts.numel() != B or top > C:
            raise ValueError("counts must have one entry <= configs per bracket")
        order = torch.empty((B, C), dtype=torch.int32, device=metrics.device)
        rc = _native.lib("plx_polytune").plx_topk_brackets(
            metrics.data_ptr(), counts.data_ptr(), B, C, C, int(maximize), order.data_ptr(), _stream(metrics))
        _native.check(rc, "plx_topk_brackets")
        return order
    return torch.from_numpy(topk_order_reference(metrics.numpy(), counts.numpy(), maximize))


def topk_order_reference(metrics: np.ndarray, counts: np.ndarray, maximize: bool) -> np.ndarray:
    B, C = metrics.shape
    out = -np.ones((B, C), dtype=np.int32)
    for b in range(B):
        n = int(counts[b])
        row = metrics[b, :n].astype(np.float64)
        key = -row if maximize else row
        nan = np.isnan(key)
        key = np.where(nan, np.inf, key)
        # stable: NaN last, then by key, ties by index
        idx = np.lexsort((np.arange(n), key, nan.astype(np.int8)))
        out[b, :n] = idx
    return out


def select_top(metrics: Sequence[Tuple[int, float]], keep: int, maximize: bool,
               device: str = "cuda") -> List[int]:
    """Hyperband ``get_reduced_configs`` on the device: ids of the best ``keep`` entries."""
    if keep <= 0 or not metrics:
        return []
    vals = torch.tensor([[float(m[1]) for m in metrics]], dtype=torch.float32)
    counts = torch.tensor([len(metrics)], dtype=torch.int32)
    if device != "cpu" and torch.cuda.is_available():
        vals, counts = vals.to(device), counts.to(device)
    order = topk_order(vals, counts, maximize)[0].cpu().tolist()
    return [metrics[i][0] for i in order[:keep]]


def early_stop_any(metrics: torch.Tensor, rules: Sequence[Tuple[int, float, bool]]) -> List[bool]:
    """metrics [E, M] (NaN = unreported); rules (column, threshold, maximize) -> triggered per rule."""
    if not rules:
        return []
    if metrics.is_cuda:
        dev = metrics.device
        metrics = metrics.contiguous().float()
        col = torch.tensor([r[0] for r in rules], dtype=torch.int32, device=dev)
        val = torch.tensor([r[1] for r in rules], dtype=torch.float32, device=dev)
        mx = torch.tensor([int(r[2]) for r in rules], dtype=torch.int32, device=dev)
        flags = torch.zeros(len(rules), dtype=torch.int32, device=dev)
        rc = _native.lib("plx_polytune").plx_early_stop_any(
            metrics.data_ptr(), metrics.shape[0], metrics.shape[1], col.data_ptr(), val.data_ptr(), mx.data_ptr(),
            len(rules), flags.data_ptr(), _stream(metrics))
        _native.check(rc, "plx_early_stop_any")
        return [bool(x) for x in flags.cpu().tolist()]
    return early_stop_any_host(metrics.numpy(), rules)


class BracketMetrics:
    """Device tensor [n_brackets, max_configs] of rung metrics (NaN = not yet reported)."""

    def __init__(self, n_brackets: int, max_configs: int, device):
        self.values = torch.full((n_brackets, max_configs), math.nan, dtype=torch.float32, device=device)
        self.counts = torch.zeros(n_brackets, dtype=torch.int32, device=device)
        self._host_counts = [0] * n_brackets

    def reset_bracket(self, b: int, n: int) -> None:
        self.values[b].fill_(math.nan)
        self._host_counts[b] = n
        self.counts[b] = n

    def slot_ptr(self, b: int) -> int:
        return self.values[b].data_ptr()

    def order(self, maximize: bool, rows: Optional[int] = None) -> torch.Tensor:
        """One launch over the first ``rows`` brackets (all by default)."""
        n = self.values.shape[0] if rows is None else rows
        return topk_order(self.values[:n], self.counts[:n], maximize, host_counts=self._host_counts[:n])
