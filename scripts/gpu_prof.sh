#!/bin/bash
# rocprofv3 kernel trace of the headline bench + per-kernel summary and one
# step's timeline; extra bench args via BENCH_ARGS, output tag via TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-rc}
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o $TAG -- python bench.py --steps 5 --warmup 3 --att8 0 $BENCH_ARGS > gpurun_out/prof_$TAG.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv 5 45 > gpurun_out/prof_${TAG}_summary.txt
python scripts/step_timeline.py gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv 1 > gpurun_out/step_timeline_$TAG.txt
