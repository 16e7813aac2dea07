#!/bin/bash
# round 6: dist GPU tests + driver-style bench at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist.py tests/test_gpu_attention.py > gpurun_out/pytest_r6_dist.log 2>&1 || { tail -40 gpurun_out/pytest_r6_dist.log; exit 1; }
tail -2 gpurun_out/pytest_r6_dist.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r6_check.log 2>&1 || { tail -20 gpurun_out/bench_r6_check.log; exit 1; }
grep '^{' gpurun_out/bench_r6_check.log
