#!/bin/bash
# round 6: X-independent backward prologue under the X GEMM -- tests, bench, SCST table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_bwd_loop.py tests/test_gpu_graph.py tests/test_gpu_dist.py tests/test_gpu_stamps.py > gpurun_out/pytest_r6_pre.log 2>&1 || { tail -40 gpurun_out/pytest_r6_pre.log; exit 1; }
tail -2 gpurun_out/pytest_r6_pre.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r6_pre.log 2>&1 || { tail -20 gpurun_out/bench_r6_pre.log; exit 1; }
grep '^{' gpurun_out/bench_r6_pre.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('scst', d['ms_per_step'], 'cst', d['cst']['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'att8', d['att8']['ms_per_step'], 'beam', d['beam5']['ms_per_batch'], 'err', d['device_errors'])"
bash scripts/gpu_r6_scst_prof.sh
