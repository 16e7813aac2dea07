#!/bin/bash
# temporal-attention engine: GPU numerics tests, full GPU suite, benches (C=1 headline, C=8)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_att.log 2>&1
rc=$?; echo "pytest_att rc=$rc" >> gpurun_out/pytest_att.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --num_chunks 8 --profile_phases 1 --json_out gpurun_out/bench_att8.json > gpurun_out/bench_att8.log 2>&1 || exit $?
rm -rf gpurun_out/prof_att
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_att -o att -- \
   python bench.py --steps 5 --warmup 2 --num_chunks 8 > gpurun_out/prof_att.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_att/att_kernel_trace.csv 7 40 > gpurun_out/prof_att_summary.txt
echo "rc=$?"
