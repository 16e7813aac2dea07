#!/bin/bash
# round 6: packed W_iv shadow -- tests touching the video gate, bench, prologue table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_cells.py tests/test_gpu_grad_events.py > gpurun_out/pytest_r6_wiv.log 2>&1 || { tail -40 gpurun_out/pytest_r6_wiv.log; exit 1; }
tail -1 gpurun_out/pytest_r6_wiv.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > gpurun_out/bench_r6_wiv_$i.log 2>&1 || { tail -20 gpurun_out/bench_r6_wiv_$i.log; exit 1; }
  grep '^{' gpurun_out/bench_r6_wiv_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('scst', d['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'err', d['device_errors'], 'loss', d['final_loss'])"
done
