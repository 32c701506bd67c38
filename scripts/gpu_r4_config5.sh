#!/bin/bash
# Round 4: BASELINE config 5 on one GPU -- the bare Llama-3 8B trainer vs the same command through polyflow
# (plx run, examples/llama3_8b_dp1.yml), plus the DP path's overheads at world 1 (nccl PG + every bucket's RCCL
# all-reduce + the RCCL metric communicator) and ZeRO-1's sharded in-backward update.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -m polyaxon_amd.trainers lm --model llama3_8b --bs 1 --seq 4096 --steps 20 --lr 3e-4 --log_every 5"
for v in "" "--world1_collectives" "--zero1" ""; do
  timeout -k 10 400 $T $v > gpurun_out/r4c5_bare.log 2>&1 || { tail -20 gpurun_out/r4c5_bare.log; exit 1; }
  echo "bare [$v] $(grep '^{' gpurun_out/r4c5_bare.log | tail -1 | cut -c1-220)"
done
export PLX_ROOT=/tmp/plxroot_c5
timeout -k 10 600 python -m polyaxon_amd.cli -p llama run -f examples/llama3_8b_dp1.yml --gpus 1 > gpurun_out/r4c5_flow.log 2>&1 || { tail -30 gpurun_out/r4c5_flow.log; exit 1; }
tail -5 gpurun_out/r4c5_flow.log
python - <<'PY' > gpurun_out/r4c5_flow.json
import json, os
from polyaxon_amd.polyflow.paths import Paths
from polyaxon_amd.store.db import Store
st = Store(os.path.join(Paths(os.environ["PLX_ROOT"]).root, "polyaxon.sqlite"))
x = st.list_experiments()[-1]
print(json.dumps({"id": x["id"], "status": x["status"], "last_metric": x["last_metric"],
                  "statuses": [s["status"] for s in st.experiment_statuses(x["id"])],
                  "jobs": [(j["role"], j["status"], j["devices"]) for j in st.experiment_jobs(x["id"])],
                  "metrics": [{k: m[k] for k in m if k in ("step", "values", "name", "value")} for m in st.get_metrics(x["id"])][-8:]},
                 default=str))
PY
cat gpurun_out/r4c5_flow.json
