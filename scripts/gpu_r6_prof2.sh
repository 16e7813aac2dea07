#!/bin/bash
# round 6: per-step rocprofv3 tables with fp16 pre on / off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  rm -rf gpurun_out/prof_p$v
  CSTCAP_PRE16=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_p$v -o head -- python bench.py --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/prof_p$v.log 2>&1 || exit $?
  python scripts/prof_steps.py gpurun_out/prof_p$v/head_kernel_trace.csv 10 14 adam_update_kernel > gpurun_out/steps_p$v.txt && head -n 16 gpurun_out/steps_p$v.txt
  rm -f gpurun_out/prof_p$v/head_kernel_trace.csv
done
