#!/bin/bash
# the driver's round-end commands on the final tree: GPU suite, smoke, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_final.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_final.log
