#!/bin/bash
# round 6: dW_logit augmented-row padding (CSTCAP_DW_PAD = N - H), interleaved, + headline tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_bwd_loop.py > gpurun_out/pytest_r6_dwpad.log 2>&1 || { tail -30 gpurun_out/pytest_r6_dwpad.log; exit 1; }
tail -1 gpurun_out/pytest_r6_dwpad.log
for i in 1 2; do for v in 16 32 64 128 256; do
  CSTCAP_DW_PAD=$v timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > gpurun_out/ab_dwpad_${v}_$i.log 2>&1 || { tail -20 gpurun_out/ab_dwpad_${v}_$i.log; exit 1; }
  grep '^{' gpurun_out/ab_dwpad_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pad', $v, 'scst', d['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'err', d['device_errors'])"
done; done
