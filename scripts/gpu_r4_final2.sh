#!/bin/bash
# round 4 final tree (after the clean-up commits)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_r4_final.sh
