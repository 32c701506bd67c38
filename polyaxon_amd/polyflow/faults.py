"""Fault-injection specs (SURVEY.md §5.3 — the reference has none).

``POLYFLOW_FAULT=kill_rank:R@t:SECONDS`` — the scheduler SIGKILLs replica R that long after spawn;
``POLYFLOW_FAULT=kill_rank:R@step:N`` — the tracking client of rank R kills its own process when it logs step N.
Both fire on the first attempt only, so ``environment.max_restarts`` retries can be tested end to end.
"""
from __future__ import annotations

from typing import Any, Dict, Optional


def parse_fault(text: str) -> Optional[Dict[str, Any]]:
    """``kill_rank:1@step:100`` -> {"rank": 1, "at": "step", "value": 100}; None when malformed."""
    try:
        what, when = text.split("@", 1)
        kind, rank = what.split(":", 1)
        at, value = when.split(":", 1)
        if kind != "kill_rank" or at not in ("step", "t"):
            return None
        return {"rank": int(rank), "at": at, "value": float(value) if at == "t" else int(value)}
    except ValueError:
        return None
