"""Placement robustness (advisor round-1 findings) and the allocator extensions: queue safety on placement errors,
device release when a replica cannot be spawned, gang reservation against starvation, HBM budgets for
fractional-GPU trials."""
import os
import sys
import time

import pytest

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow
from polyaxon_amd.spec.specification import PolyaxonfileError

PY = sys.executable


def _flow(tmp_path, n_gpus=2, settings=None, **kw):
    alloc = DeviceAllocator([Device(i) for i in range(n_gpus)])
    return Polyflow(str(tmp_path / "plx"), allocator=alloc, stop_grace_s=1.0, settings=settings, **kw).start()


def _xp(cmd, gpu=None, hbm=None, **extra):
    d = {"version": 1, "kind": "experiment", "run": {"cmd": cmd}}
    res = {}
    if gpu is not None:
        res["gpu"] = gpu
    if hbm is not None:
        res["hbm"] = hbm
    if res:
        d["environment"] = {"resources": res}
    d["environment"] = dict(d.get("environment") or {}, **extra)
    return d


def test_fractional_multi_gpu_request_rejected_at_parse(tmp_path):
    flow = _flow(tmp_path)
    try:
        with pytest.raises(PolyaxonfileError):
            flow.submit(_xp("true", gpu=1.5))
        with pytest.raises(PolyaxonfileError):
            flow.submit(_xp("true", gpu=-1))
    finally:
        flow.shutdown()


def test_placement_error_does_not_lose_the_queue(tmp_path, monkeypatch):
    """A run whose placement raises is failed; the runs queued behind it are still placed and run."""
    flow = _flow(tmp_path, n_gpus=1)
    try:
        blocker = flow.submit(_xp("sleep 0.5", gpu=1))
        doomed = flow.submit(_xp("true", gpu=1), name="doomed")
        after = flow.submit(_xp("true", gpu=1))
        real = flow.alloc.allocate

        def boom(owner, gpus, mem_gb=0.0):
            if owner.startswith(f"experiment:{doomed['id']}:"):
                raise ValueError("synthetic placement failure")
            return real(owner, gpus, mem_gb)

        monkeypatch.setattr(flow.alloc, "allocate", boom)
        assert flow.wait("experiment", blocker["id"], timeout=30) == "succeeded"
        assert flow.wait("experiment", doomed["id"], timeout=30) == "failed"
        assert "placement failed" in flow.store.experiment_statuses(doomed["id"])[-1]["message"]
        assert flow.wait("experiment", after["id"], timeout=30) == "succeeded"
        assert flow.alloc.allocations == {}
    finally:
        flow.shutdown()


def test_spawn_failure_releases_every_replica_allocation(tmp_path, monkeypatch):
    """OSError on the spawn of replica 1 of 2: the failed replica's device and the never-spawned ones go back."""
    flow = _flow(tmp_path, n_gpus=4)
    try:
        real = flow.pm.spawn
        calls = {"n": 0}

        def spawn(argv, env, cwd=None, log_path=None):
            calls["n"] += 1
            if calls["n"] == 2:
                raise OSError(24, "Too many open files (injected)")
            return real(argv, env, cwd=cwd, log_path=log_path)

        monkeypatch.setattr(flow.pm, "spawn", spawn)
        spec = _xp("sleep 30", gpu=1, pytorch={"n_workers": 2, "default_worker": {"resources": {"gpu": 1}}})
        r = flow.submit(spec)
        assert flow.wait("experiment", r["id"], timeout=30) == "failed"
        deadline = time.time() + 10
        while time.time() < deadline and flow.call(lambda: dict(flow.alloc.allocations)):
            time.sleep(0.05)
        assert flow.call(lambda: dict(flow.alloc.allocations)) == {}
        ev = flow.store.cluster_events()
        assert any(e["kind"] == "spawn_failure" for e in ev)
        monkeypatch.setattr(flow.pm, "spawn", real)
        ok = flow.submit(_xp("true", gpu=4))  # the whole node is free again
        assert flow.wait("experiment", ok["id"], timeout=30) == "succeeded"
    finally:
        flow.shutdown()


class _Settings(dict):
    def get(self, k, default=None):
        return super().get(k, default)


def test_gang_reservation_prevents_starvation(tmp_path):
    """A stream of 1-GPU trials would keep a 2-GPU gang waiting forever under FIFO-with-bypass; after the gang
    has waited ``gang_reserve_s`` the small runs may no longer take the devices it needs."""
    settings = _Settings({"scheduler.gang_reserve_s": 0.3, "scheduler.reconcile_interval_s": 5.0,
                          "scheduler.stop_grace_s": 1.0, "scheduler.numa_bind": False,
                          "scheduler.build_reuse_s": 0.0, "build.backend": "native", "build.registry": "r",
                          "build.push": False, "scheduler.max_restarts": 0, "scheduler.heartbeat_timeout_s": 0.0,
                          "scheduler.clean_after_s": 0.0, "scheduler.resident_idle_s": 10.0})
    flow = _flow(tmp_path, n_gpus=2, settings=settings)
    try:
        first = flow.submit(_xp("sleep 0.4", gpu=1))
        gang = flow.submit(_xp("sleep 0.1", gpu=2))
        small = []
        t_end = time.time() + 6
        gang_done = None
        while time.time() < t_end:
            small.append(flow.submit(_xp("sleep 0.4", gpu=1))["id"])
            st = flow.store.get_experiment(gang["id"])["status"]
            if st == "succeeded":
                gang_done = time.time()
                break
            time.sleep(0.15)
        assert gang_done is not None, "gang starved by the 1-GPU stream"
        for x in small + [first["id"]]:
            assert flow.wait("experiment", x, timeout=60) == "succeeded"
    finally:
        flow.shutdown()


def test_hbm_budget_packs_fractional_trials_by_memory():
    alloc = DeviceAllocator([Device(0, memory_gb=288.0)])
    a = alloc.allocate("a", 0.25, 200.0)
    assert a is not None and a.devices == [0]
    assert alloc.allocate("b", 0.25, 100.0) is None  # compute share is free, HBM is not
    assert alloc.allocate("c", 0.25, 80.0) is not None
    alloc.release("a")
    assert alloc.allocate("b", 0.25, 100.0) is not None
    # pinned allocation (attached executors)
    alloc2 = DeviceAllocator([Device(0), Device(1)])
    assert alloc2.allocate_on("w", [1]) is not None
    assert alloc2.allocate_on("w2", [1]) is None and alloc2.free_whole() == [0]


def test_hbm_budget_honoured_by_scheduler(tmp_path):
    flow = _flow(tmp_path, n_gpus=1)
    try:
        big = flow.submit(_xp("sleep 0.5", gpu=0.25, hbm=200))
        small = flow.submit(_xp("true", gpu=0.25, hbm=50))
        second_big = flow.submit(_xp("true", gpu=0.25, hbm=150))
        assert flow.wait("experiment", small["id"], timeout=30) == "succeeded"
        # second_big had to wait for big's HBM: it started after big finished
        assert flow.wait("experiment", second_big["id"], timeout=30) == "succeeded"
        xb = flow.store.get_experiment(big["id"])
        x2 = flow.store.get_experiment(second_big["id"])
        assert x2["started_at"] >= xb["finished_at"] - 0.05
    finally:
        flow.shutdown()
