#!/bin/bash
# GPU validation: kernel numerics tests, smoke, short HIP-engine bench, microbench, profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1 || exit $?
VARIANTS=0,1,2,3 timeout -k 10 300 python scripts/microbench_decoder.py > gpurun_out/microbench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hip -o hip -- \
   python bench.py --steps 5 --warmup 2 > gpurun_out/prof_hip.log 2>&1
echo "prof rc=$?"
