#!/bin/bash
# Big-tile decode launch: numerics tests, vocab microbenchmark (variant 0 =
# 128 x 64 tiles, 9 = 256 x 256), then the driver-style bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-big}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_decode_step.py} -m gpu -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_$TAG.log
[ $e -eq 0 ] || exit $e
VARIANTS="0 9" TGS=0 CS=0 ATT=0 timeout -k 10 300 python scripts/microbench_kernels.py > gpurun_out/mb_$TAG.json 2> gpurun_out/mb_$TAG.err || exit $?
cat gpurun_out/mb_$TAG.json
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
  tail -n 1 gpurun_out/bench_$TAG.json | cut -c1-600
fi
