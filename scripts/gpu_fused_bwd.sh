#!/bin/bash
# fused dS + dHd backward: numerics tests, then headline A/B (fused off / on, split 1 / 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "match_torch or matches_torch" > gpurun_out/pytest_fused.log 2>&1 || exit $?
CSTCAP_BWD_DHD_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "h512" > gpurun_out/pytest_fused_s1.log 2>&1 || exit $?
for r in 1 2; do
  for cfg in "0 2" "1 1" "1 2"; do
    set -- $cfg
    CSTCAP_BWD_FUSED=$1 CSTCAP_BWD_DHD_SPLIT=$2 timeout -k 10 300 python bench.py --steps 40 --warmup 5 --json_out gpurun_out/fb_$1_$2_$r.json > gpurun_out/fb_$1_$2_$r.log 2>&1 || exit $?
  done
done
