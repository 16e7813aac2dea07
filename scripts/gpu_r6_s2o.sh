#!/bin/bash
# round 6 session 2: hipBLASLt candidates timed per tuned shape, 32 (default) vs 128
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2o
for i in 1 2; do
  for m in 128 32; do
    CSTCAP_BLASLT_NCAND=$m timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > gpurun_out/s2o/n${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2o/n${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2o/n${m}_$i.log > gpurun_out/s2o/n${m}_$i.json
    python -c "
import json; d=json.load(open('gpurun_out/s2o/n${m}_$i.json'))
print('ncand=$m scst', d['ms_per_step'], 'xe', d['xe']['ms_per_step'], [(c['m'],c['n'],c['k'],c['candidate'],c['us']) for c in d['blaslt_x_choice']])"
  done
done
