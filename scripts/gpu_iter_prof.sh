#!/bin/bash
# iteration loop: GPU tests -> bench -> rocprofv3 kernel trace of a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1 || exit $?
rm -rf gpurun_out/prof_hip
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hip -o hip -- \
   python bench.py --steps 5 --warmup 2 > gpurun_out/prof_hip.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_hip/hip_kernel_trace.csv 7 40 > gpurun_out/prof_summary.txt
echo "rc=$?"
