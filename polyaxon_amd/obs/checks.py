"""Health / status checks (reference polyaxon/checks/*.py: Postgres, Redis, RabbitMQ and a round-trip
health task per Celery queue).  Here: the store, the scheduler thread (round-trip through its command
queue), the native libraries, the HIP devices and a real RCCL round trip in a child process (this process stays GPU-free)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
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


_RCCL_CACHE: Dict[str, Any] = {}
RCCL_CACHE_S = 60.0


def check_rccl(timeout: float = 90.0, max_age: float = RCCL_CACHE_S) -> Dict[str, Any]:
    """A real RCCL round trip (obs/rccl_probe.py) in a short-lived child process: this process -- the API /
    scheduler -- never imports torch or maps the HIP runtime.  The result is cached for ``max_age`` seconds so a
    polled ``/_status`` does not start a GPU process per request.  "skipped" (no device visible) counts as healthy."""
    now = time.monotonic()
    hit = _RCCL_CACHE.get("result")
    if hit is not None and now - _RCCL_CACHE.get("at", 0.0) < max_age:
        return dict(hit, cached=True)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    pp = os.environ.get("PYTHONPATH")
    env = dict(os.environ, PYTHONPATH=root + (os.pathsep + pp if pp else ""))
    t = time.perf_counter()
    try:
        out = subprocess.run([sys.executable, "-m", "polyaxon_amd.obs.rccl_probe"], capture_output=True, text=True,
                             timeout=timeout, env=env, cwd=root)
        lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
        res = json.loads(lines[-1]) if lines else {"status": "error",
                                                   "message": f"probe exited {out.returncode}: {out.stderr[-300:]}"}
    except subprocess.TimeoutExpired:
        res = {"status": "error", "message": f"RCCL probe did not finish within {timeout:.0f} s"}
    except Exception as e:
        res = {"status": "error", "message": f"{type(e).__name__}: {e}"}
    res["probe_ms"] = round((time.perf_counter() - t) * 1000, 1)
    healthy = res.get("status") in ("ok", "skipped")
    result = _result(healthy, res.get("message", ""), **{k: v for k, v in res.items() if k not in ("status", "message")})
    if res.get("status") == "skipped":
        result["skipped"] = True
    _RCCL_CACHE.update(result=result, at=now)
    return dict(result, cached=False)


def run_checks(flow) -> Dict[str, Any]:
    checks = {"store": check_store(flow), "scheduler": check_scheduler(flow), "native": check_native(),
              "devices": check_devices(flow), "rccl": check_rccl()}
    return {"status": "ok" if all(c["status"] == "ok" for c in checks.values()) else "degraded", "checks": checks}
