#!/bin/bash
# round 6 session 2: combine with 4 rows per workgroup (A/B), host enqueue time
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2j
CSTCAP_CMB_ROWS=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_decode_step.py tests/test_gpu_headline.py tests/test_gpu_graph.py \
  > gpurun_out/s2j/pytest_rows4.log 2>&1 || { tail -40 gpurun_out/s2j/pytest_rows4.log; exit 1; }
tail -1 gpurun_out/s2j/pytest_rows4.log
for i in 1 2 3; do
  for m in 4 1; do
    CSTCAP_CMB_ROWS=$m timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2j/r${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2j/r${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2j/r${m}_$i.log > gpurun_out/s2j/r${m}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2j/r${m}_$i.json')); print('rows=$m scst', d['ms_per_step'], 'err', d['device_errors'])"
  done
done
timeout -k 10 300 python bench.py --sync_debug 1 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2j/sd.log 2>&1 || { tail -20 gpurun_out/s2j/sd.log; exit 1; }
grep "sync_debug" gpurun_out/s2j/sd.log
