"""Dispatch for the fused NHWC BatchNorm(+add)(+ReLU) HIP kernels (filled in by csrc/bn_kernels.hip)."""
from __future__ import annotations

import torch


def supported(x: torch.Tensor) -> bool:
    return False


def bn_act(*args, **kwargs):  # pragma: no cover - replaced once the kernels land
    raise NotImplementedError
