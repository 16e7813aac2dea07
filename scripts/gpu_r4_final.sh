#!/bin/bash
# round 4 final tree: GPU suite, smoke, driver-style default bench, and a
# rocprofv3 kernel summary of the default step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu_final.log 2>&1
e=$?; tail -n 2 gpurun_out/pytest_gpu_final.log
[ $e -eq 0 ] || exit $e
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_final.log
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
tail -n 1 gpurun_out/bench_final.json | cut -c1-300
TAG=final bash scripts/gpu_prof.sh && head -n 25 gpurun_out/prof_final_summary.txt
