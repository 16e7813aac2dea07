#!/bin/bash
# round 6 (session 2): full GPU suite + smoke + driver-style bench at HEAD after a rebuild
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/head2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/head2/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/head2/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/head2/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/head2/smoke.log 2>&1 || { tail -20 gpurun_out/head2/smoke.log; exit 1; }
tail -1 gpurun_out/head2/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/head2/bench.log 2>&1 || { tail -20 gpurun_out/head2/bench.log; exit 1; }
grep '^{' gpurun_out/head2/bench.log > gpurun_out/head2/bench.json
python -c "import json; d=json.load(open('gpurun_out/head2/bench.json')); print('scst', d['ms_per_step'], 'cst', d['cst']['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'att8', d['att8']['ms_per_step'], 'beam', d['beam5']['videos_per_s'], 'err', d['device_errors'])"
