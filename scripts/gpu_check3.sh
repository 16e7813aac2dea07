#!/bin/bash
# full GPU suite, smoke, headline (+att8) bench x2, stamps, kernel summaries
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --json_out gpurun_out/bench_c3_$rep.json > gpurun_out/bench_c3_$rep.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 > gpurun_out/stamps_c3.log 2>&1 || exit $?
TAG=c3 bash scripts/gpu_prof.sh || exit $?
BENCH_ARGS="--num_chunks 8" TAG=c3att8 bash scripts/gpu_prof.sh || exit $?
