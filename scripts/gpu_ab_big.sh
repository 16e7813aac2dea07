#!/bin/bash
# 256x256 fused decode tiles: numerics tests, then bench A/B (big on/off), attention bench, profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
for B in 0 1; do
  CSTCAP_VOCAB_BIG=$B timeout -k 10 300 python bench.py --steps 30 --warmup 5 --json_out gpurun_out/bench_big$B.json > gpurun_out/bench_big$B.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --num_chunks 8 --json_out gpurun_out/bench_att8.json > gpurun_out/bench_att8.log 2>&1 || exit $?
rm -rf gpurun_out/prof_big
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_big -o big -- \
   python bench.py --steps 5 --warmup 2 > gpurun_out/prof_big.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_big/big_kernel_trace.csv 7 20 > gpurun_out/prof_big_summary.txt
