#!/bin/bash
# round 6: PMC passes of the headline (SCST) replayed step + 2 driver-style benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=pmc_r6h bash scripts/gpu_pmc.sh > /dev/null || exit $?
head -n 14 gpurun_out/pmc_r6h/summary.txt
for i in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/bench_r6_rep$i.log 2>&1 || { tail -20 gpurun_out/bench_r6_rep$i.log; exit 1; }
  grep '^{' gpurun_out/bench_r6_rep$i.log > gpurun_out/bench_r6_rep$i.json
  python -c "import json; d=json.load(open('gpurun_out/bench_r6_rep$i.json')); print('scst', d['ms_per_step'], 'cst', d['cst']['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'att8', d['att8']['ms_per_step'], 'beam', d['beam5']['videos_per_s'], 'err', d['device_errors'])"
done
