#!/bin/bash
# round 6: reverse-step tile map A/B (headline + att8) and the affected GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_attention.py tests/test_gpu_attention_headline.py \
  tests/test_gpu_kernels.py > gpurun_out/pytest_r6_ab1.log 2>&1 || { tail -30 gpurun_out/pytest_r6_ab1.log; exit 1; }
tail -2 gpurun_out/pytest_r6_ab1.log
ARMS="col:CSTCAP_BWD_MAP=0 row:CSTCAP_BWD_MAP=1" REPS=3 TAG=map bash scripts/gpu_ab.sh || exit $?
ARMS="col:CSTCAP_BWD_MAP=0 row:CSTCAP_BWD_MAP=1" REPS=2 TAG=map8 BENCH_ARGS="--num_chunks 8" bash scripts/gpu_ab.sh || exit $?
