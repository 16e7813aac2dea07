#!/bin/bash
# GPU suite, headline bench (default and row-resident decode launch), device
# timeline stamps of the graph step, kernel trace of both decode launches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --json_out gpurun_out/bench_stamps.json > gpurun_out/bench_stamps.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --json_out gpurun_out/bench_def_$rep.json > gpurun_out/bench_def_$rep.log 2>&1 || exit $?
  CSTCAP_DECODE_RR=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --att8 0 --json_out gpurun_out/bench_rr_$rep.json > gpurun_out/bench_rr_$rep.log 2>&1 || exit $?
done
TAG=def bash scripts/gpu_prof.sh || exit $?
CSTCAP_DECODE_RR=1 TAG=rr bash scripts/gpu_prof.sh || exit $?
