#!/bin/bash
# round 6: dW_logit placement after the persistent loop (CSTCAP_DW_LATE 0/1/2), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_DW_LATE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py > gpurun_out/pytest_r6_dwlate.log 2>&1 || { tail -30 gpurun_out/pytest_r6_dwlate.log; exit 1; }
tail -1 gpurun_out/pytest_r6_dwlate.log
for i in 1 2; do for v in 0 1 2; do
  CSTCAP_DW_LATE=$v timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > gpurun_out/ab_dwlate_${v}_$i.log 2>&1 || { tail -20 gpurun_out/ab_dwlate_${v}_$i.log; exit 1; }
  grep '^{' gpurun_out/ab_dwlate_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dw_late', $v, 'scst', d['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'err', d['device_errors'])"
done; done
