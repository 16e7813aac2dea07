#!/bin/bash
# round 6: persistent reverse loop v2 + fused dW_logit/bias sums -- tests, microbench, A/B, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bwd_loop.py tests/test_gpu_wgrad.py > gpurun_out/pytest_r6_loop.log 2>&1 || { tail -40 gpurun_out/pytest_r6_loop.log; exit 1; }
tail -2 gpurun_out/pytest_r6_loop.log
timeout -k 10 120 python scripts/microbench_loop.py 1280 512 29 20 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_kernels.py > gpurun_out/pytest_r6_loop2.log 2>&1 || { tail -40 gpurun_out/pytest_r6_loop2.log; exit 1; }
tail -2 gpurun_out/pytest_r6_loop2.log
ARMS="steps:CSTCAP_BWD_LOOP=0,CSTCAP_DW_WGRAD=0 loop:CSTCAP_BWD_LOOP=1,CSTCAP_DW_WGRAD=0 loopw:CSTCAP_BWD_LOOP=1,CSTCAP_DW_WGRAD=1" REPS=2 TAG=loop2 bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 python bench.py --stamps 4 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/stamps_loop2.json 2> gpurun_out/stamps_loop2.err || exit $?
grep -A40 "stamps (us" gpurun_out/stamps_loop2.err | head -40
