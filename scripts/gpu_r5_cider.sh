#!/bin/bash
# CIDEr-D kernel timing at the bench shapes (scripts/microbench_cider.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/microbench_cider.py > gpurun_out/cider_${TAG:-r5}.json 2> gpurun_out/cider_${TAG:-r5}.err || exit $?
cat gpurun_out/cider_${TAG:-r5}.json
