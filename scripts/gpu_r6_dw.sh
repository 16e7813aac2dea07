#!/bin/bash
# round 6: tuned batched dW_logit GEMM -- numerics + A/B (interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "tuned_blaslt or xe_loss" > gpurun_out/pytest_r6_dw.log 2>&1 || { tail -40 gpurun_out/pytest_r6_dw.log; exit 1; }
tail -2 gpurun_out/pytest_r6_dw.log
for i in 1 2; do
  for v in 0 1; do
    CSTCAP_DW_TUNED=$v timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > gpurun_out/ab_dw_${v}_$i.log 2>&1 || { tail -20 gpurun_out/ab_dw_${v}_$i.log; exit 1; }
    grep '^{' gpurun_out/ab_dw_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dw_tuned', $v, 'scst', d['ms_per_step'], 'xe', d['xe']['ms_per_step'], [c for c in d['blaslt_x_choice'] if c.get('batch',1)>1])"
  done
done
