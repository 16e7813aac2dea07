#!/bin/bash
# round 6: K-split persistent loop -- tests, microbench, A/B, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bwd_loop.py > gpurun_out/pytest_r6_ks.log 2>&1 || { tail -40 gpurun_out/pytest_r6_ks.log; exit 1; }
tail -2 gpurun_out/pytest_r6_ks.log
timeout -k 10 120 python scripts/microbench_loop.py 1280 512 29 20 8 || exit $?
timeout -k 10 120 python scripts/microbench_loop.py 1280 512 29 20 0 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_kernels.py > gpurun_out/pytest_r6_ks2.log 2>&1 || { tail -40 gpurun_out/pytest_r6_ks2.log; exit 1; }
tail -2 gpurun_out/pytest_r6_ks2.log
ARMS="rowread:CSTCAP_BWD_LOOP=2 ksplit:CSTCAP_BWD_LOOP=1" REPS=2 TAG=ks bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 python bench.py --stamps 4 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/stamps_ks.json 2> gpurun_out/stamps_ks.err || exit $?
grep -A40 "stamps (us" gpurun_out/stamps_ks.err | head -40
