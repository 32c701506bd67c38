"""Resource telemetry: per-GPU (amd-smi / rocm-smi) and per-trial process trees (psutil).

Reference: polyaxon/monitor_resources/monitor.py:27-179 — docker stats + NVML (``polyaxon_gpustat``) per
container every second, GPUs mapped to containers by a regex on ``/dev/nvidia(\\d+)``.  Here the mapping
is exact: polyflow's allocator knows which HIP devices each replica owns, and CPU/memory come from the
replica's own process tree.  GPU samples come from ``amd-smi metric --json`` (utilisation, HBM used of
288 GB, power, temperature) with ``rocm-smi --json`` as fallback; on a host without GPUs the GPU list is
empty.  ``ResourceMonitor`` samples on a background thread (1 s, like the reference) and keeps the
latest sample per experiment for the SSE resources stream (reference RedisToStream latest-only).
"""
from __future__ import annotations

import json
import shutil
import subprocess
import threading
import time
from typing import Any, Dict, List, Optional


def _run_json(cmd: List[str], timeout: float = 5.0) -> Optional[Any]:
    if shutil.which(cmd[0]) is None:
        return None
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        if out.returncode != 0:
            return None
        txt = out.stdout.strip()
        start = min([i for i in (txt.find("{"), txt.find("[")) if i >= 0], default=-1)
        return json.loads(txt[start:]) if start >= 0 else None
    except (subprocess.SubprocessError, ValueError, OSError):
        return None


def _num(v) -> Optional[float]:
    if isinstance(v, dict):
        v = v.get("value", v.get("current"))
    if v is None:
        return None
    try:
        return float(str(v).split()[0].rstrip("%"))
    except (ValueError, IndexError):
        return None


def gpu_stats() -> List[Dict[str, Any]]:
    """One dict per GPU: index, util_pct, mem_used_mb, mem_total_mb, power_w, temp_c."""
    data = _run_json(["amd-smi", "metric", "--json"])
    out: List[Dict[str, Any]] = []
    if isinstance(data, list):
        for i, g in enumerate(data):
            usage = g.get("usage", {}) or {}
            mem = g.get("mem_usage", {}) or {}
            power = g.get("power", {}) or {}
            temp = g.get("temperature", {}) or {}
            out.append({"index": g.get("gpu", i), "util_pct": _num(usage.get("gfx_activity")),
                        "mem_used_mb": _num(mem.get("used_vram")), "mem_total_mb": _num(mem.get("total_vram")),
                        "power_w": _num(power.get("socket_power")),
                        "temp_c": _num(temp.get("hotspot", temp.get("edge")))})
        return out
    data = _run_json(["rocm-smi", "--showuse", "--showmemuse", "--showpower", "--showtemp", "--json"])
    if isinstance(data, dict):
        for key, g in sorted(data.items()):
            if not key.startswith("card"):
                continue
            out.append({"index": int(key[4:]), "util_pct": _num(g.get("GPU use (%)")),
                        "mem_used_pct": _num(g.get("GPU Memory Allocated (VRAM%)")),
                        "power_w": _num(g.get("Current Socket Graphics Package Power (W)")),
                        "temp_c": _num(g.get("Temperature (Sensor junction) (C)"))})
    return out


def process_tree_stats(pid: int) -> Dict[str, float]:
    try:
        import psutil
    except ImportError:
        return {}
    try:
        p = psutil.Process(pid)
        procs = [p] + p.children(recursive=True)
        cpu = sum(q.cpu_percent(interval=None) for q in procs)
        rss = sum(q.memory_info().rss for q in procs)
        return {"cpu_percentage": cpu, "memory_used_mb": rss / 2 ** 20, "n_procs": len(procs)}
    except Exception:
        return {}


def experiment_resources(flow, xid: int) -> Dict[str, Any]:
    """Latest resources of an experiment's replicas: process stats + the GPUs polyflow gave them."""
    def collect():
        run = flow.runs.get(f"experiment:{xid}")
        return [] if run is None else [(r.role, r.index, r.pid, list(r.devices), r.done) for r in run.replicas]

    reps = flow.call(collect) if flow._thread is not None else collect()
    gpus = {g["index"]: g for g in gpu_stats()} if any(r[3] for r in reps) else {}
    out = []
    for role, idx, pid, devs, done in reps:
        item = {"job": f"{role}.{idx}", "devices": devs, "done": done}
        if pid and not done:
            item.update(process_tree_stats(pid))
        item["gpus"] = [gpus[d] for d in devs if d in gpus]
        out.append(item)
    return {"experiment": xid, "time": time.time(), "replicas": out}


class ResourceMonitor:
    """Background sampler (reference monitor_resources management command, 1 s period)."""

    def __init__(self, flow, period_s: float = 1.0):
        self.flow = flow
        self.period_s = period_s
        self.latest: Dict[int, Dict[str, Any]] = {}
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def start(self) -> "ResourceMonitor":
        self._thread = threading.Thread(target=self._run, name="plx-resources", daemon=True)
        self._thread.start()
        return self

    def _run(self) -> None:
        while not self._stop.wait(self.period_s):
            try:
                for xid in self.flow.running_experiments():
                    self.latest[xid] = experiment_resources(self.flow, xid)
            except Exception:
                pass

    def stop(self) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
