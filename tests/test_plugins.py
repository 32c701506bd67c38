"""Notebook and tensorboard plugin jobs: start with a free local port, run until stopped, stop on request.

Mirrors the reference's tests/test_plugins (notebook_scheduler.py:17-92, tensorboard_scheduler.py:16-76,
request_tensorboard_port in spawners/tensorboard_spawner.py:28-38).  Jupyter and TensorBoard are not
installed in the image, so the scheduler's interpreter is replaced by a stub that records its argv and
blocks like a server would."""
import os
import time

import pytest

from polyaxon_amd.polyflow.devices import Device, DeviceAllocator
from polyaxon_amd.polyflow.scheduler import Polyflow


@pytest.fixture
def flow(tmp_path):
    stub = tmp_path / "fake_python"
    stub.write_text(f"#!/bin/sh\necho \"$@\" >> {tmp_path}/argv\nexec sleep 60\n")
    stub.chmod(0o755)
    f = Polyflow(str(tmp_path / "plx"), allocator=DeviceAllocator([Device(0)]), stop_grace_s=1.0,
                 python=str(stub)).start()
    yield f
    f.shutdown()


def _wait_status(flow, jid, status, timeout=20.0):
    end = time.time() + timeout
    while time.time() < end:
        if flow.store.get_job(jid)["status"] == status:
            return True
        time.sleep(0.05)
    return False


@pytest.mark.parametrize("kind,module", [("notebook", "jupyter"), ("tensorboard", "tensorboard.main")])
def test_plugin_start_port_and_stop(flow, tmp_path, kind, module):
    r = flow.submit({"version": 1, "kind": kind})
    assert r["kind"] == kind
    jid = r["id"]
    assert _wait_status(flow, jid, "running")
    rec = flow.store.get_job(jid)
    assert rec["kind"] == kind and 1024 <= rec["port"] <= 65535
    end = time.time() + 10
    while not (tmp_path / "argv").exists() and time.time() < end:
        time.sleep(0.05)
    argv = (tmp_path / "argv").read_text()
    assert f"-m {module}" in argv and f"--port={rec['port']}" in argv
    assert "127.0.0.1" in argv  # plugins bind to the node's loopback only
    assert flow.stop_job(jid)
    assert _wait_status(flow, jid, "stopped")


def test_two_plugins_get_distinct_ports(flow):
    a = flow.submit({"version": 1, "kind": "tensorboard"})["id"]
    b = flow.submit({"version": 1, "kind": "notebook"})["id"]
    assert _wait_status(flow, a, "running") and _wait_status(flow, b, "running")
    assert flow.store.get_job(a)["port"] != flow.store.get_job(b)["port"]
    flow.stop_job(a)
    flow.stop_job(b)
    assert _wait_status(flow, a, "stopped") and _wait_status(flow, b, "stopped")
    assert os.path.isdir(flow.store.get_job(a)["logs_path"])
