#!/bin/bash
# round 6 session 2: beam decode as sub-batches on two streams inside the graph
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2n
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py -k beam > gpurun_out/s2n/pytest.log 2>&1 || { tail -40 gpurun_out/s2n/pytest.log; exit 1; }
tail -1 gpurun_out/s2n/pytest.log
CSTCAP_BEAM_SPLIT=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention.py -k beam tests/test_gpu_cells.py -k beam > gpurun_out/s2n/pytest2.log 2>&1 || { tail -40 gpurun_out/s2n/pytest2.log; exit 1; }
tail -1 gpurun_out/s2n/pytest2.log
for i in 1 2; do
  for m in 2 1 4; do
    CSTCAP_BEAM_SPLIT=$m timeout -k 10 300 python bench.py --mode beam --att8 0 --cst 0 --xe 0 > gpurun_out/s2n/b${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2n/b${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2n/b${m}_$i.log > gpurun_out/s2n/b${m}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2n/b${m}_$i.json')); print('split=$m', d['value'], d['unit'], d['ms_per_step'])"
  done
done
