"""Health / status checks (reference polyaxon/checks/*.py: Postgres, Redis, RabbitMQ and a round-trip
health task per Celery queue).  Here: the store, the scheduler thread (round-trip through its command
queue), the native libraries, the HIP devices and RCCL availability."""
from __future__ import annotations

import time
from typing import Any, Dict


def _result(ok: bool, message: str = "", **extra) -> Dict[str, Any]:
    return {"status": "ok" if ok else "error", "message": message, **extra}


def check_store(flow) -> Dict[str, Any]:
    try:
        flow.store.execute("SELECT 1").fetchone()
        return _result(True, path=flow.store.path)
    except Exception as e:
        return _result(False, str(e))


def check_scheduler(flow) -> Dict[str, Any]:
    if flow._thread is None or not flow._thread.is_alive():
        return _result(False, "scheduler thread not running")
    t = time.perf_counter()
    try:
        flow.call(lambda: None, timeout=5)
    except Exception as e:
        return _result(False, f"scheduler round trip failed: {e}")
    return _result(True, round_trip_ms=round((time.perf_counter() - t) * 1000, 3),
                   running=len(flow.running_experiments()), pending=len(flow.pending))


def check_native() -> Dict[str, Any]:
    from polyaxon_amd.ops import _native

    missing = [n for n in _native.LIBRARIES if not _native.available(n)]
    return _result(not missing, "missing: " + ", ".join(missing) if missing else "", libraries=list(_native.LIBRARIES))


def check_devices(flow) -> Dict[str, Any]:
    devs = flow.call(flow.alloc.snapshot)
    unhealthy = [d["index"] for d in devs if not d["healthy"]]
    return _result(not unhealthy, f"unhealthy: {unhealthy}" if unhealthy else "", n_devices=len(devs))


def check_rccl() -> Dict[str, Any]:
    try:
        import torch.distributed as dist

        return _result(dist.is_available() and dist.is_nccl_available(), backend="nccl (RCCL)")
    except Exception as e:
        return _result(False, str(e))


def run_checks(flow) -> Dict[str, Any]:
    checks = {"store": check_store(flow), "scheduler": check_scheduler(flow), "native": check_native(),
              "devices": check_devices(flow), "rccl": check_rccl()}
    return {"status": "ok" if all(c["status"] == "ok" for c in checks.values()) else "degraded", "checks": checks}
