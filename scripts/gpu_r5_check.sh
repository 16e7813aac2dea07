#!/bin/bash
# Round-5 iteration check: selected GPU tests, decode diagnostics, interleaved
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
if [ -n "$DECODE_DIAG" ]; then
  timeout -k 10 200 python scripts/microbench_decode.py > gpurun_out/mbdec_$TAG.json || exit $?
  cat gpurun_out/mbdec_$TAG.json
fi
if [ -n "$ARMS" ]; then TAG=$TAG bash scripts/gpu_ab.sh || exit $?; fi
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'], 'att8', d.get('att8',{}).get('ms_per_step'), 'cst', d.get('cst',{}).get('ms_per_step'), 'beam5', d.get('beam5',{}).get('videos_per_s'))" gpurun_out/bench_$TAG.json
