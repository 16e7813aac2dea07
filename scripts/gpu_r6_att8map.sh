#!/bin/bash
# round 6: att8 reverse step kernel, XCD row mapping on / off (CSTCAP_BWD_MAP), one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 0 1; do
  rm -rf gpurun_out/prof_att8_m$m
  CSTCAP_BWD_MAP=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_att8_m$m -o att8 -- \
    python bench.py --steps 6 --warmup 4 --num_chunks 8 --beam5 0 --cst 0 --xe 0 > gpurun_out/prof_att8_m$m.log 2>&1 || exit $?
  python scripts/prof_steps.py gpurun_out/prof_att8_m$m/att8_kernel_trace.csv 5 40 adam_update_kernel 'e' > gpurun_out/steps_att8_m$m.txt || exit $?
  rm -f gpurun_out/prof_att8_m$m/att8_kernel_trace.csv
  echo "map $m"; head -n 4 gpurun_out/steps_att8_m$m.txt | cut -c1-110
done
for i in 1 2; do for m in 0 1; do
  CSTCAP_BWD_MAP=$m timeout -k 10 300 python bench.py --num_chunks 8 --beam5 0 --cst 0 --xe 0 > gpurun_out/ab_att8_m${m}_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab_att8_m${m}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('map', $m, 'att8', d['ms_per_step'])"
done; done
