#!/bin/bash
# split-K A/B of the fused LSTM backward step: numerics tests, then the bench per S
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_attention.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
for S in 1 2 3 4; do
  CSTCAP_BWD_SPLITK=$S timeout -k 10 300 python bench.py --steps 30 --warmup 5 --json_out gpurun_out/bench_s$S.json > gpurun_out/bench_s$S.log 2>&1 || exit $?
done
CSTCAP_BWD_SPLITK=2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --num_chunks 8 --json_out gpurun_out/bench_att8.json > gpurun_out/bench_att8.log 2>&1 || exit $?
