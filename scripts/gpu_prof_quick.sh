#!/bin/bash
# kernel trace of a short headline bench -> per-kernel summary + one-step timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${PROF_TAG:-q}
rm -rf gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o $tag -- python bench.py --steps 5 --warmup 2 $PROF_ARGS > gpurun_out/prof_$tag.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_$tag/${tag}_kernel_trace.csv 7 25 > gpurun_out/prof_${tag}_summary.txt
python scripts/step_timeline.py gpurun_out/prof_$tag/${tag}_kernel_trace.csv 1 > gpurun_out/step_timeline_$tag.txt
