#!/bin/bash
# Round-5 GPU check: selected GPU tests (TESTS, default the whole -m gpu
# suite), the driver-style bench, and a clean per-step rocprofv3 table of the
# shipped headline step (last 10 timed steps, scripts/prof_steps.py).
# TAG names the outputs; SKIP_PROF=1 / SKIP_BENCH=1 / SKIP_TESTS=1 skip parts.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r5}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
  e=$?; tail -n 3 gpurun_out/pytest_$TAG.log
  [ $e -eq 0 ] || exit $e
fi
if [ -z "$SKIP_SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
  tail -n 1 gpurun_out/smoke_$TAG.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
  tail -n 1 gpurun_out/bench_$TAG.json | cut -c1-400
fi
if [ -z "$SKIP_PROF" ]; then
  rm -rf gpurun_out/prof_$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG \
    -o $TAG -- python bench.py --steps 10 --warmup 5 --att8 0 --beam5 0 $PROF_ARGS \
    > gpurun_out/prof_$TAG.log 2>&1 || exit $?
  python scripts/prof_steps.py gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv 10 45 \
    > gpurun_out/steps_$TAG.txt && head -n 30 gpurun_out/steps_$TAG.txt
  rm -f gpurun_out/prof_$TAG/*_kernel_trace.csv.gz
fi
