#!/bin/bash
# rocprofv3 per-step kernel table of the att8 step (bench --num_chunks 8) and
# the last step's reverse-loop launch sequence (step kernel / attention
# backward), for the fused attention backward (lstm.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-att8}
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o att8 -- \
  python bench.py --steps 6 --warmup 4 --num_chunks ${NUMCH:-8} --att8 0 --beam5 0 --cst 0 ${BENCH_ARGS} \
  > gpurun_out/prof_$TAG.log 2>&1 || exit $?
python scripts/prof_steps.py gpurun_out/prof_$TAG/att8_kernel_trace.csv 5 45 adam_update_kernel \
  "${SEQ-lstm_step_bwd|att_bwd|att_dgv}" > gpurun_out/steps_$TAG.txt && head -n 30 gpurun_out/steps_$TAG.txt
rm -f gpurun_out/prof_$TAG/att8_kernel_trace.csv
