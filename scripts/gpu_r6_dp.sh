#!/bin/bash
# round 6: DP stand-in priority study, per-step kernel table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/dp_standin.py 29517 32 400 10 > gpurun_out/dp_standin.json 2> gpurun_out/dp_standin.err || { tail -20 gpurun_out/dp_standin.err; exit 1; }
cat gpurun_out/dp_standin.json
rm -rf gpurun_out/prof_r6_head
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r6_head -o head -- python bench.py --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/prof_r6_head.log 2>&1 || exit $?
python scripts/prof_steps.py gpurun_out/prof_r6_head/head_kernel_trace.csv 10 40 adam_update_kernel > gpurun_out/steps_r6_head.txt && head -n 30 gpurun_out/steps_r6_head.txt
rm -f gpurun_out/prof_r6_head/head_kernel_trace.csv
