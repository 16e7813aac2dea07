#!/bin/bash
# round 4 bundle 7: the post-loop weight-gradient GEMMs through hipBLASLt's
# measured choice -- gradient tests with the switch on, then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_TUNED_TAIL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_attention_headline.py \
  tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tail.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_tail.log
[ $e -eq 0 ] || exit $e
AB_A="CSTCAP_TUNED_TAIL=0" AB_B="CSTCAP_TUNED_TAIL=1" REPS=3 AB_ATT8=1 bash scripts/gpu_r4_ab.sh || exit $?
