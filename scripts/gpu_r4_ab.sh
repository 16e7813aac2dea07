#!/bin/bash
# round 4: interleaved A/B of environment configurations on one box.
# usage: AB_A="ENV=.. ENV2=.." AB_B="..." [AB_C="..."] [AB_D="..."] bash scripts/gpu_r4_ab.sh  (REPS, default 3;
# AB_EXTRA: extra bench.py arguments, e.g. --sync_each 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
  for c in A B ${AB_C:+C} ${AB_D:+D}; do
    v=AB_$c
    env ${!v} timeout -k 10 300 python bench.py --steps 30 --warmup 5 --att8 ${AB_ATT8:-0} --json_out gpurun_out/ab_${c}_$i.json > gpurun_out/ab_${c}_$i.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/ab_${c}_$i.json'))
print('$c', '${!v}', 'rep $i', d['ms_per_step'], (d.get('att8') or {}).get('ms_per_step'))"
  done
done
