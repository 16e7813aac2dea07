#!/bin/bash
# round 6 session 2: re-check of the dW_logit schedule knobs at HEAD
# (CSTCAP_DW_LATE 1 default vs 0 / 2; CSTCAP_DW_PAD 64 default vs 128)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2m
for i in 1 2; do
  for cfg in "CSTCAP_DW_LATE=1" "CSTCAP_DW_LATE=2" "CSTCAP_DW_LATE=0" "CSTCAP_DW_PAD=128"; do
    tag=$(echo $cfg | tr '=' '_')
    env $cfg timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > gpurun_out/s2m/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/s2m/${tag}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2m/${tag}_$i.log > gpurun_out/s2m/${tag}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2m/${tag}_$i.json')); print('$cfg scst', d['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'err', d['device_errors'])"
  done
done
