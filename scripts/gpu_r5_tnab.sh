#!/bin/bash
# ResNet-50 bench A/B, alternating weight-gradient variants.  VARIANTS: space-separated "v2[,ring_kb][:bpc]" items
# (PLX_TN_V2 and PLX_TN2_BPC), e.g. "0 1,64:1 0 1,64:1".
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r5tn}.jsonl
: > $OUT
STEPS=${STEPS:-3}
for item in ${VARIANTS:-0 1,64 0 1,64}; do
  v=${item%%:*}; bpc=0; [ "$item" != "$v" ] && bpc=${item#*:}
  tag=${item//[,:]/_}
  PLX_TN_V2="$v" PLX_TN2_BPC="$bpc" timeout -k 10 420 python -u bench.py --steps $STEPS --warmup 1 > gpurun_out/_tn.json 2> gpurun_out/${TAG:-r5tn}_$tag.err || { tail -5 gpurun_out/${TAG:-r5tn}_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/_tn.json').read().strip().splitlines()[-1]); print(json.dumps({'variant': '$item', 'value': d['value'], 'train_images_per_s': d['train_images_per_s'], 'ms_per_step': d['ms_per_step']}))" >> $OUT
  tail -1 $OUT
done
