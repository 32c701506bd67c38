"""HIP-device allocator for one 8×MI355X node.

The reference has no GPU accounting of its own: it sets a Kubernetes GPU limit per pod
(scheduler/spawners/templates/resources.py:31-35) and concurrency is per group only
(db/models/experiment_groups.py:192-197 — SURVEY.md §8.6 "no cluster-wide GPU accounting").  polyflow
owns the devices directly:

* every device has 1.0 compute share and its HBM budget (288 GB on MI355X);
* a replica asks for ``gpu`` devices — an integer (gang of whole devices, e.g. DP=2/4/8) or a fraction
  (``0.25`` = four small trials packed on one device, the MLP grid config);
* whole-device gangs take the devices with no fractional tenants first, lowest index first; on MI355X
  every pair of GPUs has its own xGMI link (fully connected), so any k devices are equivalent for RCCL
  and contiguity is kept only so logs/rocm-smi read naturally;
* fractional requests best-fit onto the most-loaded device that still fits (keeps whole devices free
  for gangs, i.e. limits fragmentation);
* allocation is all-or-nothing per gang and the allocator is only touched from the scheduler thread.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

EPS = 1e-9


@dataclass
class Device:
    index: int
    name: str = "AMD Instinct MI355X"
    memory_gb: float = 288.0
    share_used: float = 0.0
    mem_used_gb: float = 0.0
    healthy: bool = True
    owners: Dict[str, float] = field(default_factory=dict)

    @property
    def share_free(self) -> float:
        return 1.0 - self.share_used


@dataclass
class Allocation:
    owner: str
    devices: List[int]
    share: float
    mem_gb: float


def parse_cpulist(text: str) -> List[int]:
    """``"0-3,8,10-11"`` -> [0, 1, 2, 3, 8, 10, 11] (sysfs cpulist format)."""
    out: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out.extend(range(int(lo), int(hi or lo) + 1))
    return out


def device_cpus(index: int, sysfs: str = "/sys") -> Optional[List[int]]:
    """CPUs local to HIP device ``index`` (the NUMA node of its PCIe root), read from the KFD topology (GPU nodes
    in enumeration order -> ``drm_render_minor``) and DRM sysfs -- no GPU runtime call, so the scheduler can
    use it before any trial starts.  None when the topology is not readable."""
    import glob

    gpus = []
    paths = glob.glob(os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes", "*", "properties"))
    for p in sorted(paths, key=lambda s: int(os.path.basename(os.path.dirname(s)))):
        try:
            with open(p) as f:
                props = dict(line.split(None, 1) for line in f.read().splitlines() if " " in line)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            gpus.append(props.get("drm_render_minor", "").strip())
    if index >= len(gpus) or not gpus[index]:
        return None
    try:
        with open(os.path.join(sysfs, "class", "drm", f"renderD{gpus[index]}", "device", "local_cpulist")) as f:
            cpus = parse_cpulist(f.read())
    except (OSError, ValueError):
        return None
    return cpus or None


def detect_devices(sysfs: str = "/sys") -> List[Device]:
    """Visible HIP devices from the KFD topology (sysfs) -- no HIP runtime, no torch: the scheduler process that
    calls this never loads either.  HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES (comma lists of indices) narrow the
    set as they do for HIP; PLX_NUM_GPUS overrides (tests, CPU rehearsals)."""
    n = os.environ.get("PLX_NUM_GPUS")
    if n is not None:
        return [Device(i) for i in range(int(n))]
    from polyaxon_amd.obs.nodes import kfd_gpus

    gpus = kfd_gpus(sysfs)
    if os.path.isdir("/dev/dri"):  # a container sees the render nodes of the GPUs it was given (ROCr opens them)
        gpus = [g for g in gpus if not g.get("drm_render_minor")
                or os.path.exists(f"/dev/dri/renderD{g['drm_render_minor']}")]
    count = len(gpus)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        vis = os.environ.get(var)
        if vis is None:
            continue
        ids = [v for v in vis.split(",") if v.strip() != ""]
        try:
            count = len([i for i in ids if 0 <= int(i) < count])
        except ValueError:  # UUID lists: trust their length
            count = min(count, len(ids))
    return [Device(i) for i in range(count)]


class DeviceAllocator:
    def __init__(self, devices: Optional[List[Device]] = None):
        self.devices: List[Device] = devices if devices is not None else detect_devices()
        self.allocations: Dict[str, Allocation] = {}

    @property
    def n_devices(self) -> int:
        return len(self.devices)

    def free_whole(self) -> List[int]:
        return [d.index for d in self.devices if d.healthy and d.share_used < EPS]

    def can_allocate(self, gpus: float, mem_gb: float = 0.0) -> bool:
        return self._plan(gpus, mem_gb) is not None

    def _plan(self, gpus: float, mem_gb: float) -> Optional[List[int]]:
        if gpus <= 0:
            return []
        if gpus >= 1.0 - EPS:
            k = int(round(gpus))
            if abs(k - gpus) > EPS:
                raise ValueError(f"multi-device requests must be whole devices, got {gpus}")
            free = [d for d in self.devices if d.healthy and d.share_used < EPS
                    and d.memory_gb - d.mem_used_gb >= mem_gb - EPS]
            if len(free) < k:
                return None
            # prefer a contiguous run of indices if one exists, else the lowest free ones
            idx = [d.index for d in free]
            for start in range(len(idx) - k + 1):
                run = idx[start:start + k]
                if run[-1] - run[0] == k - 1:
                    return run
            return idx[:k]
        # fractional: best fit on the most-loaded device that fits
        cands = [d for d in self.devices if d.healthy and d.share_free >= gpus - EPS
                 and d.memory_gb - d.mem_used_gb >= mem_gb - EPS]
        if not cands:
            return None
        cands.sort(key=lambda d: (-d.share_used, d.index))
        return [cands[0].index]

    def allocate(self, owner: str, gpus: float, mem_gb: float = 0.0) -> Optional[Allocation]:
        if owner in self.allocations:
            raise ValueError(f"{owner} already holds an allocation")
        plan = self._plan(gpus, mem_gb)
        if plan is None:
            return None
        share = 1.0 if gpus >= 1.0 - EPS else gpus
        per_dev_mem = mem_gb / max(len(plan), 1)
        for i in plan:
            d = self.devices[i]
            d.share_used += share
            d.mem_used_gb += per_dev_mem
            d.owners[owner] = share
        a = Allocation(owner, plan, share, mem_gb)
        self.allocations[owner] = a
        return a

    def allocate_on(self, owner: str, devices: List[int], gpus: float = 1.0,
                    mem_gb: float = 0.0) -> Optional[Allocation]:
        """Reserve specific devices (a process that already owns them registers with the scheduler, e.g. an
        attached resident executor).  None if any of them cannot take the share / HBM."""
        if owner in self.allocations:
            raise ValueError(f"{owner} already holds an allocation")
        share = 1.0 if gpus >= 1.0 - EPS else gpus
        per_dev_mem = mem_gb / max(len(devices), 1)
        for i in devices:
            if i >= len(self.devices):
                return None
            d = self.devices[i]
            if not d.healthy or d.share_free < share - EPS or d.memory_gb - d.mem_used_gb < per_dev_mem - EPS:
                return None
        for i in devices:
            d = self.devices[i]
            d.share_used += share
            d.mem_used_gb += per_dev_mem
            d.owners[owner] = share
        a = Allocation(owner, list(devices), share, mem_gb)
        self.allocations[owner] = a
        return a

    def release(self, owner: str) -> None:
        a = self.allocations.pop(owner, None)
        if a is None:
            return
        per_dev_mem = a.mem_gb / max(len(a.devices), 1)
        for i in a.devices:
            d = self.devices[i]
            d.share_used = max(0.0, d.share_used - a.share)
            d.mem_used_gb = max(0.0, d.mem_used_gb - per_dev_mem)
            d.owners.pop(owner, None)

    def mark_unhealthy(self, index: int) -> None:
        self.devices[index].healthy = False

    def snapshot(self) -> List[Dict]:
        return [{"index": d.index, "name": d.name, "share_used": round(d.share_used, 4), "memory_gb": d.memory_gb,
                 "mem_used_gb": d.mem_used_gb, "healthy": d.healthy, "owners": dict(d.owners)} for d in self.devices]
