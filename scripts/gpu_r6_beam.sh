#!/bin/bash
# round 6: beam search with 128-row vocab tiles -- numerics + A/B (interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_BEAM_BN=128 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_kernels.py tests/test_gpu_cells.py -k "beam" > gpurun_out/pytest_r6_beam.log 2>&1 || { tail -40 gpurun_out/pytest_r6_beam.log; exit 1; }
tail -2 gpurun_out/pytest_r6_beam.log
for i in 1 2; do
  for v in 64 128; do
    CSTCAP_BEAM_BN=$v timeout -k 10 300 python bench.py --steps 3 --warmup 2 --att8 0 --cst 0 --xe 0 > gpurun_out/ab_beam_${v}_$i.log 2>&1 || { tail -20 gpurun_out/ab_beam_${v}_$i.log; exit 1; }
    grep '^{' gpurun_out/ab_beam_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('beam_bn', $v, d['beam5'])"
  done
done
