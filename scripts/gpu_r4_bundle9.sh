#!/bin/bash
# round 4 bundle 9: (1) W_hh gradient split (late steps on the side stream
# during the loop) -- gradient tests with it on; (2) A/B of the split point and
# of the bias column-sum workgroup size under the concurrent schedule
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_WHH_SPLIT=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_attention_headline.py \
  tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_split.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_split.log
[ $e -eq 0 ] || exit $e
AB_A="CSTCAP_WHH_SPLIT=0" AB_B="CSTCAP_WHH_SPLIT=8" AB_C="CSTCAP_WHH_SPLIT=14" AB_D="CSTCAP_COLSUM_ROWS=2048" \
  REPS=3 bash scripts/gpu_r4_ab.sh || exit $?
