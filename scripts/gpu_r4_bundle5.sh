#!/bin/bash
# round 4 bundle 5: bundle-4 tests (grad-event check in a fresh process),
# recurrent-weight GEMMs on the side stream A/B, hardware-queue count A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_grad_events.py tests/test_gpu_headline.py tests/test_gpu_graph.py \
  tests/test_gpu_dist.py tests/test_gpu_attention_headline.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_whh.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_whh.log
[ $e -eq 0 ] || exit $e
AB_A="CSTCAP_WHH_SIDE=1" AB_B="CSTCAP_WHH_SIDE=0" AB_C="GPU_MAX_HW_QUEUES=8" AB_D="GPU_MAX_HW_QUEUES=16" \
  REPS=3 AB_ATT8=1 bash scripts/gpu_r4_ab.sh || exit $?
TAG=b2b_v4 bash scripts/gpu_r4_stamps.sh
