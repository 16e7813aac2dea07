#!/bin/bash
# Round-5 iteration check: selected GPU tests, a clean rocprofv3 step table (PROF=1), interleaved
# A/B of the headline step (ARMS, see gpu_ab.sh), one full driver-style bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-chk}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_headline.py} -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_$TAG.log
[ $e -eq 0 ] || exit $e
if [ -n "$PROF" ]; then  # clean per-step kernel table of the shipped step (last 10 timed steps)
  rm -rf gpurun_out/prof_$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG \
    -o $TAG -- python bench.py --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 $PROF_ARGS \
    > gpurun_out/prof_$TAG.log 2>&1 || exit $?
  python scripts/prof_steps.py gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv 10 45 \
    > gpurun_out/steps_$TAG.txt && head -n 24 gpurun_out/steps_$TAG.txt
  rm -f gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv
fi
if [ -n "$ARMS" ]; then TAG=$TAG bash scripts/gpu_ab.sh || exit $?; fi
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'], 'att8', d.get('att8',{}).get('ms_per_step'), 'cst', d.get('cst',{}).get('ms_per_step'), 'beam5', d.get('beam5',{}).get('videos_per_s'))" gpurun_out/bench_$TAG.json
