#!/bin/bash
# round 6 session 2: combine rows per workgroup 4 (default) vs 8 vs 1 -- headline,
# att8 and XE; decode / headline / attention tests at the default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2k
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_decode_step.py tests/test_gpu_attention.py tests/test_gpu_attention_headline.py tests/test_gpu_cst.py \
  > gpurun_out/s2k/pytest.log 2>&1 || { tail -40 gpurun_out/s2k/pytest.log; exit 1; }
tail -1 gpurun_out/s2k/pytest.log
for i in 1 2; do
  for m in 4 8 1; do
    CSTCAP_CMB_ROWS=$m timeout -k 10 300 python bench.py --beam5 0 --cst 0 > gpurun_out/s2k/r${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2k/r${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2k/r${m}_$i.log > gpurun_out/s2k/r${m}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2k/r${m}_$i.json')); print('rows=$m scst', d['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'att8', d['att8']['ms_per_step'], 'err', d['device_errors'])"
  done
done
