#!/bin/bash
# round 4: beam-5 decode -- GPU tests (new top-K kernel, graph replay), then
# the bench's beam5 field with and without the graph replay, and the default
# bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_attention.py tests/test_gpu_cells.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_beam.log 2>&1 || exit $?
for g in 0 1; do
  CSTCAP_BEAM_GRAPH=$g timeout -k 10 300 python bench.py --steps 10 --warmup 3 --att8 0 --json_out gpurun_out/beam_g$g.json > gpurun_out/beam_g$g.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/beam_g$g.json')); print('graph=$g', d['ms_per_step'], d.get('beam5'))"
done
timeout -k 10 400 python bench.py --json_out gpurun_out/r4_default.json > gpurun_out/r4_default.log 2>&1 || exit $?
grep '^{' gpurun_out/r4_default.log
