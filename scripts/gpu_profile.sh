#!/bin/bash
# rocprofv3 kernel trace + stats of the fused-engine SCST bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hip -o hip -- \
   python bench.py --steps 5 --warmup 2 > gpurun_out/prof_hip.log 2>&1
echo "rc=$?"
