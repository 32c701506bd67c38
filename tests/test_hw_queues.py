"""GPU_MAX_HW_QUEUES is the operator's: importing the package leaves it alone, and PLX_HW_QUEUES=n is an opt-in floor
applied only to the processes polyflow launches (polyflow/env.py hw_queue_env) and by bench.py (profiles/
r5_hw_queues.md: the weight-gradient side stream's own priority level fits the box's default 4 queues)."""
import os
import subprocess
import sys

import pytest

from polyaxon_amd.polyflow.env import hw_queue_env

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("env", [{"GPU_MAX_HW_QUEUES": "4"}, {}, {"GPU_MAX_HW_QUEUES": "4", "PLX_HW_QUEUES": "8"}])
def test_import_leaves_hw_queues_alone(env):
    e = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "PLX_HW_QUEUES")}
    e.update(env)
    e["PYTHONPATH"] = REPO
    out = subprocess.run([sys.executable, "-c", "import os, polyaxon_amd; print(os.environ.get('GPU_MAX_HW_QUEUES'))"],
                         env=e, capture_output=True, text=True, check=True).stdout.strip()
    assert out == env.get("GPU_MAX_HW_QUEUES", "None")


@pytest.mark.parametrize("env,want", [({"GPU_MAX_HW_QUEUES": "4"}, "4"), ({}, None),
                                      ({"GPU_MAX_HW_QUEUES": "4", "PLX_HW_QUEUES": "8"}, "8"),
                                      ({"GPU_MAX_HW_QUEUES": "16", "PLX_HW_QUEUES": "8"}, "16"),
                                      ({"PLX_HW_QUEUES": "64"}, "32"), ({"PLX_HW_QUEUES": "x"}, None)])
def test_launched_process_floor(env, want):
    assert hw_queue_env(dict(env)).get("GPU_MAX_HW_QUEUES") == want
