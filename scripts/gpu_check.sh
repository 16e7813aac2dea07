#!/bin/bash
# GPU validation: kernel numerics tests, smoke, short HIP-engine bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1
echo "bench rc=$?"
