"""polyaxon-mi355x: an experiment-orchestration and HPO engine for one 8×MI355X node.

Subpackages: spec (Polyaxonfile), fsm (lifecycles), store (tracking DB + query DSL), polytune (search
algorithms + HIP kernels), polyflow (scheduler, resident trial executor, pipelines), parallel (RCCL /
distributed runner), client (tracking SDK), api (REST + SSE), cli, obs (events, telemetry, checks),
models, ops (HIP kernel bindings).
"""
__version__ = "0.3.0"

# No process-wide GPU settings are changed at import.  (Round 4 raised GPU_MAX_HW_QUEUES to 8 here; the streams a
# trial process holds now fit the box's default 4 hardware queues instead -- one framework RCCL communicator per DP
# trial (parallel/comm.py) and the weight-gradient side stream on its own priority level (ops/side_stream.py) --
# and PLX_HW_QUEUES=n is an explicit opt-in read by bench.py and by the processes polyflow launches.)
