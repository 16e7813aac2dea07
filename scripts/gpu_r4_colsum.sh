#!/bin/bash
# round 4: bias column sums with fewer, longer workgroups (CSTCAP_COLSUM_ROWS)
# -- gradient test at the headline shape, then an interleaved A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_COLSUM_ROWS=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_colsum.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_colsum.log
[ $e -eq 0 ] || exit $e
AB_A="CSTCAP_COLSUM_ROWS=128" AB_B="CSTCAP_COLSUM_ROWS=1024" AB_C="CSTCAP_COLSUM_ROWS=4096" REPS=3 bash scripts/gpu_r4_ab.sh
