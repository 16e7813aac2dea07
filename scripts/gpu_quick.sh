#!/bin/bash
# quick measurement: GPU tests (attention first), headline + attention benches, attention profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_att.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --num_chunks 8 --json_out gpurun_out/bench_att8.json > gpurun_out/bench_att8.log 2>&1 || exit $?
rm -rf gpurun_out/prof_att
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_att -o att -- \
   python bench.py --steps 5 --warmup 2 --num_chunks 8 > gpurun_out/prof_att.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_att/att_kernel_trace.csv 7 25 > gpurun_out/prof_att_summary.txt
