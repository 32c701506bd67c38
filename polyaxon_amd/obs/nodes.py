"""Node inventory, GPU health probe and cluster events for the one-node MI355X deployment.

Reference counterparts:

* ``update_system_nodes`` (polyaxon/crons/tasks/nodes.py:47-99) lists the k8s nodes and their allocatable GPUs,
  and ``update_cluster_node`` (monitor_resources/monitor.py:134-147) writes one ``NodeGPU`` row per NVML device
  (index, serial, name, memory).  Here the node is this host: CPUs and memory from /proc, the GPUs from the KFD
  topology (``/sys/class/kfd/kfd/topology/nodes/*``: gfx target, compute units, HBM banks, unique id) enriched
  with ``amd-smi static --json`` (market name, serial, VRAM) when the tool is present -- no GPU runtime call, so
  the scheduler can inventory devices before any trial starts.
* The namespace monitor (monitor_namespace/monitor.py:15-103) persists k8s warning/error events as
  ``ClusterEvent`` rows.  The node-local equivalents are produced where they happen: spawn failures, processes
  killed by a signal nobody requested (OOM killer), GPU faults reported by the runtime in a trial's log, devices
  that turn unhealthy, resident executors that die (``record_cluster_event``).
* SURVEY §5.3 asks for a GPU-health watchdog (amd-smi RAS/ECC).  ``GpuHealthProbe`` reads the RAS error counters
  the amdgpu driver exposes per device (``/sys/class/drm/card*/device/ras/*_err_count``, "ue: N / ce: M") and
  ``amd-smi metric --ecc``; a device whose UNCORRECTABLE count grows, or that drops out of the KFD topology, is
  reported unhealthy and the allocator stops placing work on it.
"""
from __future__ import annotations

import glob
import logging
import os
import re
import time
import threading
from typing import Any, Callable, Dict, List, Optional

from polyaxon_amd.obs.telemetry import _run_json

log = logging.getLogger("polyaxon_amd.obs.nodes")

GPU_FAULT_PATTERNS = ("Memory access fault", "HSA_STATUS_ERROR", "hipErrorLaunchFailure", "GPU Hang",
                      "amdgpu: page fault", "hipErrorIllegalAddress", "HIP error: an illegal memory access")


def _props(path: str) -> Dict[str, str]:
    try:
        with open(path) as f:
            return dict(line.split(None, 1) for line in f.read().splitlines() if " " in line)
    except OSError:
        return {}


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def kfd_gpus(sysfs: str = "/sys") -> List[Dict[str, Any]]:
    """GPU nodes of the KFD topology in HIP enumeration order."""
    root = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    nodes = sorted(glob.glob(os.path.join(root, "*")), key=lambda p: int(os.path.basename(p))
                   if os.path.basename(p).isdigit() else 1 << 30)
    out = []
    for n in nodes:
        p = _props(os.path.join(n, "properties"))
        simd = int((p.get("simd_count") or "0").strip() or 0)
        if simd <= 0:
            continue
        mem = 0
        for bank in glob.glob(os.path.join(n, "mem_banks", "*", "properties")):
            bp = _props(bank)
            try:
                mem += int(bp.get("size_in_bytes", "0"))
            except ValueError:
                pass
        gfx = int((p.get("gfx_target_version") or "0").strip() or 0)
        out.append({
            "index": len(out), "kfd_node": int(os.path.basename(n)),
            "name": _read(os.path.join(n, "name")) or "amdgpu",
            "gfx": f"gfx{gfx // 10000}{(gfx // 100) % 100:x}{gfx % 100:x}" if gfx else None,
            "simd_count": simd, "cu_count": simd // max(1, int(p.get("simd_per_cu", "4") or 4)),
            "memory_gb": round(mem / 2 ** 30, 2), "serial": (p.get("unique_id") or "").strip(),
            "drm_render_minor": (p.get("drm_render_minor") or "").strip(),
            "location_id": (p.get("location_id") or "").strip(),
        })
    return out


def amdsmi_static() -> List[Dict[str, Any]]:
    data = _run_json(["amd-smi", "static", "--json"], timeout=15.0)
    out = []
    if isinstance(data, dict):
        data = data.get("gpu_data") or data.get("gpus") or []
    if isinstance(data, list):
        for i, g in enumerate(data):
            asic = g.get("asic", {}) or {}
            vram = g.get("vram", {}) or {}
            size = vram.get("size", {})
            size = size.get("value") if isinstance(size, dict) else size
            try:
                mem_gb = float(str(size).split()[0]) / 1024.0 if size is not None else None
            except (ValueError, IndexError):
                mem_gb = None
            out.append({"index": g.get("gpu", i), "name": asic.get("market_name"),
                        "serial": asic.get("asic_serial") or (g.get("board", {}) or {}).get("product_serial"),
                        "memory_gb": mem_gb})
    return out


def host_memory_gb(proc: str = "/proc") -> float:
    txt = _read(os.path.join(proc, "meminfo")) or ""
    m = re.search(r"MemTotal:\s+(\d+)\s+kB", txt)
    return round(int(m.group(1)) / 2 ** 20, 2) if m else 0.0


def inventory(sysfs: str = "/sys", proc: str = "/proc", use_smi: bool = True) -> Dict[str, Any]:
    gpus = kfd_gpus(sysfs)
    if use_smi and gpus:
        smi = {g["index"]: g for g in amdsmi_static()}
        for g in gpus:
            s = smi.get(g["index"]) or {}
            if s.get("name"):
                g["name"] = s["name"]
            if s.get("serial"):
                g["serial"] = str(s["serial"])
            if s.get("memory_gb"):
                g["memory_gb"] = round(float(s["memory_gb"]), 2)
    return {"hostname": os.uname().nodename, "cpu": float(os.cpu_count() or 1), "memory_gb": host_memory_gb(proc),
            "gpus": gpus}


def sync_node_inventory(store, n_devices: int, sysfs: str = "/sys", proc: str = "/proc",
                        use_smi: bool = True) -> Dict[str, Any]:
    """Write the node row and its NodeGPU rows (reference crons/tasks/nodes.py:47-99 + monitor.py:134-147)."""
    inv = inventory(sysfs, proc, use_smi)
    nid = store.upsert_node("local", inv["hostname"], inv["cpu"], inv["memory_gb"], max(n_devices, len(inv["gpus"])))
    for g in inv["gpus"]:
        store.upsert_node_gpu(nid, g["index"], g["name"], g["memory_gb"], serial=g["serial"] or "",
                              arch=g["gfx"] or "")
    inv["node_id"] = nid
    return inv


class GpuHealthProbe:
    """Callable returning the indices of unhealthy devices (Polyflow ``health_check``).

    A device is unhealthy when its uncorrectable RAS error count rose since the first probe, or when it vanished
    from the KFD topology.  ``events`` receives (kind, level, message, data) the first time a device turns bad.

    Devices are identified by a stable key (KFD ``unique_id``, else the DRM render minor, else the KFD node id)
    mapped to the HIP index they had at the first probe, so a device that drops out is reported under its own
    index, not under the highest ones.  The sysfs RAS counters are the source; ``amd-smi metric --ecc`` is used
    only when the driver exposes no RAS files at all (decided once, at the first probe), never merely because
    every count is zero.  With ``background=True`` (the scheduler's default) a call never blocks: it returns the
    devices known bad so far, starts a probe on a worker thread when the last one is older than ``interval_s``,
    and delivers the events that probe produced on the calling (scheduler) thread."""

    def __init__(self, sysfs: str = "/sys", use_smi: bool = True,
                 events: Optional[Callable[[str, str, str, Dict[str, Any]], None]] = None,
                 background: bool = False, interval_s: float = 5.0):
        self.sysfs = sysfs
        self.use_smi = use_smi
        self.events = events
        self.background = background
        self.interval_s = interval_s
        self.baseline: Dict[int, int] = {}
        self.keys: Optional[Dict[str, int]] = None  # stable device key -> HIP index at the first probe
        self.known: Optional[int] = None
        self.bad: set = set()
        self._smi_source: Optional[bool] = None     # True: no RAS files anywhere, counts come from amd-smi
        self._lock = threading.Lock()
        self._pending: List[tuple] = []
        self._thread: Optional[threading.Thread] = None
        self._last = 0.0

    @staticmethod
    def _key(g: Dict[str, Any]) -> str:
        for k in ("serial", "drm_render_minor"):
            v = str(g.get(k) or "").strip()
            if v and v != "0":
                return f"{k}:{v}"
        return f"kfd:{g.get('kfd_node')}"

    def _devices(self) -> List[Dict[str, Any]]:
        return kfd_gpus(self.sysfs)

    def uncorrectable(self, devices: Optional[List[Dict[str, Any]]] = None) -> Dict[int, int]:
        """Per current device index: total uncorrectable errors over every RAS block the driver reports."""
        devices = self._devices() if devices is None else devices
        out: Dict[int, int] = {}
        have_ras = False
        for idx, g in enumerate(devices):
            dev = os.path.join(self.sysfs, "class", "drm", f"renderD{g['drm_render_minor']}", "device", "ras")
            total = 0
            for f in glob.glob(os.path.join(dev, "*_err_count")):
                have_ras = True
                m = re.search(r"ue:\s*(\d+)", _read(f) or "")
                if m:
                    total += int(m.group(1))
            out[idx] = total
        if self._smi_source is None:
            self._smi_source = bool(self.use_smi and devices and not have_ras)
        if self._smi_source:
            data = _run_json(["amd-smi", "metric", "--ecc", "--json"], timeout=10.0)
            if isinstance(data, list):
                for i, g in enumerate(data):
                    ecc = (g.get("ecc") or {}) if isinstance(g, dict) else {}
                    v = ecc.get("total_uncorrectable_count", ecc.get("uncorrectable_count"))
                    try:
                        if v is not None:
                            out[int(g.get("gpu", i))] = out.get(int(g.get("gpu", i)), 0) + int(v)
                    except (TypeError, ValueError):
                        pass
        return out

    def probe(self) -> List[int]:
        """One synchronous probe: updates the bad set and queues an event per newly bad device."""
        devices = self._devices()
        counts = self.uncorrectable(devices)
        keys = {self._key(g): i for i, g in enumerate(devices)}
        with self._lock:
            if self.keys is None:
                self.keys = dict(keys)
                self.known = len(devices)
                self.baseline = {i: counts.get(i, 0) for i in range(len(devices))}
            bad = set()
            # counts are per CURRENT index; map them back to the index each device had at the first probe
            for key, cur in keys.items():
                orig = self.keys.get(key)
                if orig is None:
                    continue  # a device that was not there at the start is not ours to place
                if counts.get(cur, 0) > self.baseline.get(orig, counts.get(cur, 0)):
                    bad.add(orig)
            vanished = {orig for key, orig in self.keys.items() if key not in keys}
            bad |= vanished
            new = bad - self.bad
            self.bad |= bad
            by_orig = {self.keys[k]: counts.get(c) for k, c in keys.items() if k in self.keys}
            for idx in sorted(new):
                msg = (f"device {idx} left the KFD topology" if idx in vanished else
                       f"device {idx} unhealthy: uncorrectable RAS errors {by_orig.get(idx, 'n/a')} "
                       f"(baseline {self.baseline.get(idx, 'n/a')})")
                log.error(msg)
                self._pending.append(("gpu_unhealthy", "error", msg, {"device": idx}))
            return sorted(self.bad)

    def _flush(self) -> None:
        with self._lock:
            pending, self._pending = self._pending, []
        if self.events is not None:
            for ev in pending:
                self.events(*ev)

    def _worker(self) -> None:
        try:
            self.probe()
        except Exception:
            log.exception("GPU health probe failed")

    def __call__(self) -> List[int]:
        if not self.background:
            out = self.probe()
            self._flush()
            return out
        now = time.monotonic()
        if (self._thread is None or not self._thread.is_alive()) and now - self._last >= self.interval_s:
            self._last = now
            self._thread = threading.Thread(target=self._worker, name="plx-gpu-health", daemon=True)
            self._thread.start()
        self._flush()
        with self._lock:
            return sorted(self.bad)


def gpu_fault_in_log(path: str, tail_bytes: int = 65536) -> Optional[str]:
    """The first GPU-fault line in the last ``tail_bytes`` of a replica log, if any."""
    try:
        with open(path, "rb") as f:
            f.seek(0, os.SEEK_END)
            size = f.tell()
            f.seek(max(0, size - tail_bytes))
            txt = f.read().decode("utf-8", "replace")
    except OSError:
        return None
    for line in txt.splitlines():
        if any(p in line for p in GPU_FAULT_PATTERNS):
            return line.strip()[:500]
    return None
