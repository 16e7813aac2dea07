#!/bin/bash
# round 4 bundle 8: one flat device copy into the captured step's index
# buffer -- graph / DP tests, then A/B (CSTCAP_IDX_ALIAS=1 = upload into the
# buffer itself) and stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dist.py tests/test_gpu_headline.py \
  tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_idx.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_idx.log
[ $e -eq 0 ] || exit $e
TAG=b2b_v5 bash scripts/gpu_r4_stamps.sh
