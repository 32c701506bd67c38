"""Node inventory (reference crons/tasks/nodes.py:47-99, monitor_resources/monitor.py:134-147), the GPU health probe
(RAS/ECC watchdog) and the cluster-event producer (reference monitor_namespace/monitor.py:15-103) on a
synthetic sysfs tree and real subprocess exits."""
import os
import signal
import sys
import time

import pytest

from polyaxon_amd.obs.nodes import GpuHealthProbe, gpu_fault_in_log, inventory, kfd_gpus, sync_node_inventory
from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow
from polyaxon_amd.store import Store


def _fake_sysfs(root, n_gpus=2, mem_gb=288):
    nodes = root / "class" / "kfd" / "kfd" / "topology" / "nodes"
    cpu = nodes / "0"
    cpu.mkdir(parents=True)
    (cpu / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for i in range(n_gpus):
        n = nodes / str(i + 1)
        (n / "mem_banks" / "0").mkdir(parents=True)
        (n / "properties").write_text(f"simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\n"
                                      f"unique_id {1000 + i}\ndrm_render_minor {128 + i}\nlocation_id {i}\n")
        (n / "mem_banks" / "0" / "properties").write_text(f"size_in_bytes {mem_gb * 2 ** 30}\n")
        (n / "name").write_text("gfx950\n")
        ras = root / "class" / "drm" / f"renderD{128 + i}" / "device" / "ras"
        ras.mkdir(parents=True)
        (ras / "umc_err_count").write_text("ue: 0\nce: 3\n")
        (ras / "gfx_err_count").write_text("ue: 0\nce: 0\n")
    return root


def test_kfd_inventory(tmp_path):
    sysfs = _fake_sysfs(tmp_path / "sys", n_gpus=2)
    gpus = kfd_gpus(str(sysfs))
    assert [g["index"] for g in gpus] == [0, 1]
    assert gpus[0]["gfx"] == "gfx950" and gpus[0]["cu_count"] == 256 and gpus[0]["memory_gb"] == 288.0
    assert gpus[1]["serial"] == "1001"
    inv = inventory(str(sysfs), use_smi=False)
    assert inv["cpu"] >= 1 and inv["memory_gb"] > 0 and len(inv["gpus"]) == 2


def test_sync_node_inventory_writes_node_gpus(tmp_path):
    sysfs = _fake_sysfs(tmp_path / "sys", n_gpus=3)
    store = Store(str(tmp_path / "s.sqlite"))
    inv = sync_node_inventory(store, 3, sysfs=str(sysfs), use_smi=False)
    nodes = store.nodes()
    assert len(nodes) == 1 and nodes[0]["n_gpus"] == 3 and nodes[0]["memory"] > 0
    rows = store.node_gpus(inv["node_id"])
    assert [r["idx"] for r in rows] == [0, 1, 2] and rows[0]["memory"] == 288.0 and rows[2]["serial"] == "1002"
    assert rows[0]["arch"] == "gfx950"


def test_health_probe_flags_new_uncorrectable_errors_and_lost_devices(tmp_path):
    sysfs = _fake_sysfs(tmp_path / "sys", n_gpus=3)
    events = []
    probe = GpuHealthProbe(str(sysfs), use_smi=False, events=lambda *a: events.append(a))
    assert probe() == []
    (sysfs / "class" / "drm" / "renderD129" / "device" / "ras" / "umc_err_count").write_text("ue: 2\nce: 3\n")
    assert probe() == [1]
    assert probe() == [1] and len(events) == 1 and events[0][0] == "gpu_unhealthy"
    # device 2 falls off the bus: it disappears from the topology
    import shutil

    shutil.rmtree(sysfs / "class" / "kfd" / "kfd" / "topology" / "nodes" / "3")
    assert probe() == [1, 2] and len(events) == 2


def test_health_probe_names_the_device_that_vanished_not_the_last_index(tmp_path):
    """Device 0 (of 3) falls off the bus: the probe must report index 0, not the highest index (2), although the
    remaining devices now enumerate as 0 and 1; a later RAS rise on the old device 2 (now enumerated 1) is still
    reported as 2."""
    import shutil

    sysfs = _fake_sysfs(tmp_path / "sys", n_gpus=3)
    probe = GpuHealthProbe(str(sysfs), use_smi=False)
    assert probe() == []
    shutil.rmtree(sysfs / "class" / "kfd" / "kfd" / "topology" / "nodes" / "1")
    assert probe() == [0]
    (sysfs / "class" / "drm" / "renderD130" / "device" / "ras" / "umc_err_count").write_text("ue: 1\nce: 3\n")
    assert probe() == [0, 2]


def test_health_probe_uses_amd_smi_only_without_ras_files(tmp_path, monkeypatch):
    """Zero RAS counts on a healthy node must not trigger an amd-smi call per probe (it blocked the scheduler
    thread up to 10 s every reconcile); amd-smi is the source only when the driver exposes no RAS files."""
    import polyaxon_amd.obs.nodes as nodes

    calls = []
    monkeypatch.setattr(nodes, "_run_json", lambda cmd, timeout=0: calls.append(cmd) or [])
    sysfs = _fake_sysfs(tmp_path / "sys", n_gpus=2)
    probe = GpuHealthProbe(str(sysfs), use_smi=True)
    for _ in range(3):
        assert probe() == []
    assert calls == []
    import shutil

    bare = _fake_sysfs(tmp_path / "bare", n_gpus=2)
    shutil.rmtree(bare / "class" / "drm")
    probe2 = GpuHealthProbe(str(bare), use_smi=True)
    probe2()
    probe2()
    assert len(calls) == 2 and calls[0][:3] == ["amd-smi", "metric", "--ecc"]


def test_health_probe_background_mode_never_blocks_the_caller(tmp_path, monkeypatch):
    """Scheduler mode: the call returns at once; the probe runs on a worker thread and its events are delivered
    on the next call (the scheduler thread), not from the worker."""
    import threading

    sysfs = _fake_sysfs(tmp_path / "sys", n_gpus=2)
    events = []
    probe = GpuHealthProbe(str(sysfs), use_smi=False, background=True, interval_s=0.0,
                           events=lambda *a: events.append((threading.current_thread().name, a)))
    gate = threading.Event()
    real = probe.uncorrectable

    def slow(devices=None):
        gate.wait(5)
        return real(devices)

    monkeypatch.setattr(probe, "uncorrectable", slow)
    t0 = time.time()
    assert probe() == []
    assert time.time() - t0 < 0.5
    gate.set()
    probe._thread.join(5)
    (sysfs / "class" / "drm" / "renderD129" / "device" / "ras" / "umc_err_count").write_text("ue: 4\nce: 3\n")
    probe()
    probe._thread.join(5)
    assert probe() == [1]
    assert len(events) == 1 and events[0][0] == threading.current_thread().name


def test_scheduler_marks_unhealthy_devices_and_records_events(tmp_path):
    sysfs = _fake_sysfs(tmp_path / "sys", n_gpus=2)
    store = Store(str(tmp_path / "plx" / "polyaxon.sqlite"))
    flow = Polyflow(str(tmp_path / "plx"), store=store, allocator=DeviceAllocator([Device(0), Device(1)]),
                    reconcile_s=0.1)
    flow.health_check = GpuHealthProbe(str(sysfs), use_smi=False, events=flow.cluster_event)
    flow.start()
    try:
        time.sleep(0.3)
        (sysfs / "class" / "drm" / "renderD128" / "device" / "ras" / "gfx_err_count").write_text("ue: 1\nce: 0\n")
        end = time.time() + 5
        while time.time() < end and flow.call(lambda: flow.alloc.devices[0].healthy):
            time.sleep(0.05)
        assert not flow.call(lambda: flow.alloc.devices[0].healthy)
        assert any(e["kind"] == "gpu_unhealthy" for e in store.cluster_events())
        # placement avoids the bad device
        r = flow.submit({"version": 1, "kind": "experiment", "run": {"cmd": "true"},
                         "environment": {"resources": {"gpu": 1}}})
        assert flow.wait("experiment", r["id"], timeout=20) == "succeeded"
        assert store.experiment_jobs(r["id"])[0]["devices"] == [1]
    finally:
        flow.shutdown()


def test_cluster_events_for_oom_kill_gpu_fault_and_unschedulable(tmp_path):
    flow = Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0)]), reconcile_s=0).start()
    try:
        killed = flow.submit({"version": 1, "kind": "experiment", "run": {"cmd": "kill -9 $$"}})
        assert flow.wait("experiment", killed["id"], timeout=20) == "failed"
        fault = flow.submit({"version": 1, "kind": "experiment",
                             "run": {"cmd": "echo 'Memory access fault by GPU node-2 on address 0x7f00'; exit 134"}})
        assert flow.wait("experiment", fault["id"], timeout=20) == "failed"
        big = flow.submit({"version": 1, "kind": "experiment", "run": {"cmd": "true"},
                           "environment": {"resources": {"gpu": 4}}})
        assert flow.wait("experiment", big["id"], timeout=20) == "failed"
        kinds = [e["kind"] for e in flow.store.cluster_events()]
        assert "process_killed" in kinds and "gpu_fault" in kinds and "failed_scheduling" in kinds
        ev = next(e for e in flow.store.cluster_events() if e["kind"] == "gpu_fault")
        assert "Memory access fault" in ev["message"] and ev["level"] == "error"
    finally:
        flow.shutdown()


def test_gpu_fault_in_log(tmp_path):
    p = tmp_path / "log"
    p.write_text("ok\n" * 1000 + "HIP error: an illegal memory access was encountered\n")
    assert "illegal memory access" in gpu_fault_in_log(str(p))
    p.write_text("all good\n")
    assert gpu_fault_in_log(str(p)) is None
    assert gpu_fault_in_log(str(tmp_path / "missing")) is None
