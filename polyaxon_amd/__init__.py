"""polyaxon-mi355x: an experiment-orchestration and HPO engine for one 8×MI355X node.

Subpackages: spec (Polyaxonfile), fsm (lifecycles), store (tracking DB + query DSL), polytune (search
algorithms + HIP kernels), polyflow (scheduler, resident trial executor, pipelines), parallel (RCCL /
distributed runner), client (tracking SDK), api (REST + SSE), cli, obs (events, telemetry, checks),
models, ops (HIP kernel bindings).
"""
__version__ = "0.3.0"
