"""HBM budget of a trial process (budget the 288 GB of an MI355X between packed trials).

polyflow reserves ``resources.hbm`` GB (and a compute share for ``gpu: 0.25``-style fractions) per replica in
its allocator (polyflow/devices.py); the reservation is bookkeeping until the trial process enforces it.  The
scheduler exports the budget (polyflow/env.py ``trial_env``, pool.py for resident executors):

* ``PLX_HBM_GB``        -- the replica's HBM reservation in GB, and/or
* ``PLX_HBM_FRACTION``  -- its share of the device (fractional ``gpu``), used when no GB figure is given;

and every framework entry point (tracking client, trainers, resident executors) calls :func:`apply_hbm_budget`
before allocating, which caps PyTorch's caching allocator on that device with
``torch.cuda.set_per_process_memory_fraction``: an allocation past the budget then raises an out-of-memory error
in the offending trial instead of starving the trials packed beside it.
"""
from __future__ import annotations

import os
from typing import Optional


def budget_fraction(total_bytes: int, env=None) -> Optional[float]:
    """Fraction of a device with ``total_bytes`` of memory this process may use, or None for no budget."""
    env = os.environ if env is None else env
    gb = float(env.get("PLX_HBM_GB", "0") or 0)
    if gb > 0 and total_bytes > 0:
        return max(1e-6, min(1.0, gb * 2 ** 30 / total_bytes))
    frac = float(env.get("PLX_HBM_FRACTION", "0") or 0)
    if 0 < frac < 1:
        return frac
    return None


_applied = set()


def apply_hbm_budget(device=None) -> Optional[float]:
    """Cap this process's allocations on ``device`` (default: the current CUDA/HIP device) to its budget.
    Idempotent per device; a no-op without a budget or without a GPU.  Returns the fraction applied."""
    if not (os.environ.get("PLX_HBM_GB") or os.environ.get("PLX_HBM_FRACTION")):
        return None
    import torch

    if not torch.cuda.is_available():
        return None
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.type != "cuda":
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    frac = budget_fraction(torch.cuda.get_device_properties(idx).total_memory)
    if frac is None or idx in _applied:
        return frac
    torch.cuda.set_per_process_memory_fraction(frac, idx)
    _applied.add(idx)
    return frac
