"""The ResNet classifier head's whole training step -- global average pool, fc, cross entropy AND their backward --
queued in the forward pass, outside autograd (the resident executor's fused-head step, polyflow/executor.py).

Through autograd the head's backward is its first work: the engine thread walks the loss, cross-entropy, linear,
accumulate-grad and pool nodes, each a Python / dispatcher round trip around a kernel of a few microseconds.  When
the forward's host time is close to its GPU time (ResNet-50: ~6 of ~7 ms per step) the GPU drained the forward and
idled through those launches, ~250 us per step at the forward -> backward hand-off (scripts/gap_report.py:
``xent_bwd -> Cijk`` 98 us, ``fill -> xent_bwd`` 77 us, ...).  Here the same kernels are queued right behind the
forward, while the host is still ahead, and the backward starts at the last stage with the head's input gradient
(``features.backward(dfeatures)``).

The arithmetic is the autocast path's, op for op: bf16 pooled features, fc in bf16 (weight and bias cast from the fp32
masters), the fused cross entropy of ops/lm.py (``plx_xent_cls_fwd`` / ``_bwd``) with a unit incoming gradient,
fc weight gradient ``dlogits^T . pooled`` and bias gradient ``dlogits.sum(0)`` in bf16 accumulated into the fp32
gradient slots, ``dpooled = dlogits . W`` and the pool's backward (csrc/pool_kernels.hip ``plx_gap_backward``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn

from polyaxon_amd.ops import _native


def _stream() -> int:
    return _native.current_stream()


def supported(features: torch.Tensor, fc: nn.Module, labels: torch.Tensor, labels_in_range: bool = False) -> bool:
    """``labels_in_range``: the caller guarantees 0 <= label < fc.out_features for every row (the executor's own
    synthetic data); the fused step has no ignore-index handling of its own (its mean divides by every row)."""
    n, c = features.shape[:2]
    return (labels_in_range and features.is_cuda and features.dtype == torch.bfloat16 and features.dim() == 4 and c % 8 == 0
            and features.is_contiguous(memory_format=torch.channels_last) and features.data_ptr() % 16 == 0
            and isinstance(fc, nn.Linear) and fc.bias is not None and fc.in_features == c
            and fc.weight.grad is not None and fc.bias.grad is not None
            and labels.dtype == torch.int64 and labels.is_contiguous() and labels.shape == (n,)
            and _native.available("plx_pool") and _native.available("plx_lm"))


@torch.no_grad()
def classifier_head_step(features: torch.Tensor, fc: nn.Linear, labels: torch.Tensor,
                         ones: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(mean cross-entropy loss, d loss / d features) for logits = fc(mean over H x W of features); the fc gradients
    are accumulated into ``fc.weight.grad`` / ``fc.bias.grad``.  ``features``: the last stage's bf16 channels_last
    output.  ``ones``: a device fp32 [1] tensor holding 1.0 (the incoming gradient of the mean), reused across
    steps."""
    n, c, h, w = features.shape
    dev = features.device
    pool, lm = _native.lib("plx_pool"), _native.lib("plx_lm")
    pooled = torch.empty((n, c), dtype=torch.bfloat16, device=dev)
    _native.check(pool.plx_gap_forward(features.data_ptr(), pooled.data_ptr(), n, h * w, c, _stream()),
                  "plx_gap_forward")
    wb = fc.weight.to(torch.bfloat16)
    logits = torch.addmm(fc.bias.to(torch.bfloat16), pooled, wb.t())
    v = logits.shape[1]
    lse = torch.empty(n, dtype=torch.float32, device=dev)
    rows = torch.empty(n, dtype=torch.float32, device=dev)
    _native.check(lm.plx_xent_cls_fwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), rows.data_ptr(), n, v,
                                      _stream()), "plx_xent_cls_fwd")
    loss = rows.mean()
    if ones is None:
        ones = torch.ones(1, dtype=torch.float32, device=dev)
    dlogits = torch.empty_like(logits)
    _native.check(lm.plx_xent_cls_bwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), ones.data_ptr(),
                                      dlogits.data_ptr(), n, v, 0.0, _stream()), "plx_xent_cls_bwd")
    fc.weight.grad.add_(torch.mm(dlogits.t(), pooled))
    fc.bias.grad.add_(dlogits.sum(0))
    dpooled = torch.mm(dlogits, wb)
    dfeat = torch.empty((n, c, h, w), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    _native.check(pool.plx_gap_backward(dpooled.data_ptr(), dfeat.data_ptr(), n, h * w, c, _stream()),
                  "plx_gap_backward")
    return loss, dfeat
