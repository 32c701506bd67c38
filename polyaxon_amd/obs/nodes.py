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
    from the KFD topology.  ``events`` receives (kind, level, message, data) the first time a device turns bad."""

    def __init__(self, sysfs: str = "/sys", use_smi: bool = True,
                 events: Optional[Callable[[str, str, str, Dict[str, Any]], None]] = None):
        self.sysfs = sysfs
        self.use_smi = use_smi
        self.events = events
        self.baseline: Dict[int, int] = {}
        self.known: Optional[int] = None
        self.bad: set = set()

    def _render_minors(self) -> List[str]:
        return [g["drm_render_minor"] for g in kfd_gpus(self.sysfs)]

    def uncorrectable(self) -> Dict[int, int]:
        """Per device index: total uncorrectable errors over every RAS block the driver reports."""
        out: Dict[int, int] = {}
        for idx, minor in enumerate(self._render_minors()):
            dev = os.path.join(self.sysfs, "class", "drm", f"renderD{minor}", "device", "ras")
            total = 0
            for f in glob.glob(os.path.join(dev, "*_err_count")):
                m = re.search(r"ue:\s*(\d+)", _read(f) or "")
                if m:
                    total += int(m.group(1))
            out[idx] = total
        if self.use_smi and not any(out.values()):
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

    def __call__(self) -> List[int]:
        counts = self.uncorrectable()
        n = len(counts)
        if self.known is None:
            self.known = n
            self.baseline = dict(counts)
        bad = set()
        for idx, v in counts.items():
            if v > self.baseline.get(idx, v):
                bad.add(idx)
        if n < (self.known or 0):  # a device dropped out of the topology (reset / fallen off the bus)
            bad.update(range(n, self.known))
        new = bad - self.bad
        self.bad |= bad
        for idx in sorted(new):
            msg = f"device {idx} unhealthy: uncorrectable RAS errors {counts.get(idx, 'n/a')} " \
                  f"(baseline {self.baseline.get(idx, 'n/a')})" if idx in counts else f"device {idx} left the KFD topology"
            log.error(msg)
            if self.events is not None:
                self.events("gpu_unhealthy", "error", msg, {"device": idx})
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
