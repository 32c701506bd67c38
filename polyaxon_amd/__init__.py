"""polyaxon-mi355x: an experiment-orchestration and HPO engine for one 8×MI355X node.

Subpackages: spec (Polyaxonfile), fsm (lifecycles), store (tracking DB + query DSL), polytune (search
algorithms + HIP kernels), polyflow (scheduler, resident trial executor, pipelines), parallel (RCCL /
distributed runner), client (tracking SDK), api (REST + SSE), cli, obs (events, telemetry, checks),
models, ops (HIP kernel bindings).
"""
import os as _os

__version__ = "0.3.0"

# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4).  A process that holds an RCCL communicator
# (RCCL's own streams) next to the compute stream and our side streams (conv weight gradients, the optimizer's
# bucket updates) ran out of queues: the side stream landed on the compute stream's queue and the two serialised --
# the ResNet-50 bench lost 17 % with a live communicator, the Llama-3 8B step 8 % with per-bucket all-reduces
# (profiles/r4_rccl_slowdown.md).  Eight queues give every stream its own.  Read by the HIP runtime at its first
# initialisation, so this must run before any GPU call (importing the package first is enough).  The queue count is
# raised to PLX_HW_QUEUES (default 8; 0 leaves the environment alone), never lowered; child processes (trials,
# executors) inherit it.


def _raise_hw_queues() -> None:
    want = int(_os.environ.get("PLX_HW_QUEUES", "8") or 0)
    try:
        have = int(_os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)
    except ValueError:
        have = 0
    if want > have:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(min(want, 32))


_raise_hw_queues()
