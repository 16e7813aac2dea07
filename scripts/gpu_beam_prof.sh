#!/bin/bash
# rocprofv3 per-step kernel table of the beam-5 decode (bench --mode beam) and
# the last decode step's launch sequence.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-beam}
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o beam -- \
  python bench.py --mode beam --steps 4 --warmup 3 --att8 0 --beam5 0 --cst 0 ${BENCH_ARGS} \
  > gpurun_out/prof_$TAG.log 2>&1 || exit $?
python scripts/prof_steps.py gpurun_out/prof_$TAG/beam_kernel_trace.csv 27 20 beam_fused_step_kernel \
  "_" > gpurun_out/steps_$TAG.txt && head -n 12 gpurun_out/steps_$TAG.txt
rm -f gpurun_out/prof_$TAG/beam_kernel_trace.csv
