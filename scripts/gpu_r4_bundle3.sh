#!/bin/bash
# round 4 bundle 3: full GPU suite on the current defaults, the index-upload
# A/B, and the back-to-back stamps of the default step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu_full.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_gpu_full.log
[ $e -eq 0 ] || exit $e
AB_A="CSTCAP_IDX_ALIAS=1" AB_B="CSTCAP_IDX_ALIAS=0" REPS=2 bash scripts/gpu_r4_ab.sh || exit $?
TAG=b2b_v3 bash scripts/gpu_r4_stamps.sh
