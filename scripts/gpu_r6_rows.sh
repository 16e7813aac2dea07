#!/bin/bash
# round 6: dW rows before the loop -- headline tests, bench, SCST table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_kernels.py tests/test_gpu_decode_step.py tests/test_gpu_graph.py > gpurun_out/pytest_r6_rows.log 2>&1 || { tail -40 gpurun_out/pytest_r6_rows.log; exit 1; }
tail -1 gpurun_out/pytest_r6_rows.log
timeout -k 10 400 python bench.py --att8 0 --beam5 0 > gpurun_out/bench_r6_rows.log 2>&1 || { tail -20 gpurun_out/bench_r6_rows.log; exit 1; }
grep '^{' gpurun_out/bench_r6_rows.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('scst', d['ms_per_step'], 'cst', d['cst']['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'err', d['device_errors'])"
bash scripts/gpu_r6_scst_prof.sh > /dev/null
head -1 gpurun_out/steps_scst.txt
sed -n 27,400p gpurun_out/steps_scst.txt | awk '$1<260' | cut -c1-110
