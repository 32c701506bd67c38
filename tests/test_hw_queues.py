"""The package raises GPU_MAX_HW_QUEUES to PLX_HW_QUEUES (default 8) before any GPU call, never lowers it, and leaves
it alone with PLX_HW_QUEUES=0 (profiles/r4_rccl_slowdown.md: with 4 queues an RCCL communicator's streams pushed the
side stream onto the compute stream's queue)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("env,want", [({"GPU_MAX_HW_QUEUES": "4"}, "8"), ({}, "8"), ({"GPU_MAX_HW_QUEUES": "16"}, "16"),
                                      ({"GPU_MAX_HW_QUEUES": "4", "PLX_HW_QUEUES": "0"}, "4"),
                                      ({"PLX_HW_QUEUES": "64"}, "32")])
def test_hw_queue_floor(env, want):
    e = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "PLX_HW_QUEUES")}
    e.update(env)
    e["PYTHONPATH"] = REPO
    out = subprocess.run([sys.executable, "-c", "import os, polyaxon_amd; print(os.environ.get('GPU_MAX_HW_QUEUES'))"],
                         env=e, capture_output=True, text=True, check=True).stdout.strip()
    assert out == want
