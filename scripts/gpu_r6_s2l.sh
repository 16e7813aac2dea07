#!/bin/bash
# round 6 session 2: XE combine split (first half on a side stream) A/B + tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2l
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_cells.py \
  > gpurun_out/s2l/pytest.log 2>&1 || { tail -40 gpurun_out/s2l/pytest.log; exit 1; }
tail -1 gpurun_out/s2l/pytest.log
for i in 1 2 3; do
  for m in 1 0; do
    CSTCAP_XE_SPLIT=$m timeout -k 10 300 python bench.py --mode xe --att8 0 --beam5 0 --cst 0 > gpurun_out/s2l/x${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2l/x${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2l/x${m}_$i.log > gpurun_out/s2l/x${m}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2l/x${m}_$i.json')); print('split=$m xe', d['ms_per_step'], 'loss', d['final_loss'], 'err', d['device_errors'])"
  done
done
