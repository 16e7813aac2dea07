#!/bin/bash
# round 6 session 2: XE all rows with the vocabulary head chunked onto a side
# stream under the recurrence -- tests, chunk-size A/B, step table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2f
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_cells.py tests/test_gpu_kernels.py \
  > gpurun_out/s2f/pytest.log 2>&1 || { tail -40 gpurun_out/s2f/pytest.log; exit 1; }
tail -1 gpurun_out/s2f/pytest.log
for i in 1 2; do
  for c in 4 2 8 0 off; do
    if [ $c = off ]; then envs="CSTCAP_XE_ROWS=0"; else envs="CSTCAP_XE_CHUNK=$c"; fi
    env $envs timeout -k 10 300 python bench.py --mode xe --att8 0 --beam5 0 --cst 0 > gpurun_out/s2f/xe_${c}_$i.log 2>&1 || { tail -20 gpurun_out/s2f/xe_${c}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2f/xe_${c}_$i.log > gpurun_out/s2f/xe_${c}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2f/xe_${c}_$i.json')); print('chunk=$c', d['ms_per_step'], 'loss', d['final_loss'], 'err', d['device_errors'])"
  done
done
rm -rf gpurun_out/s2f/prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2f/prof -o xe -- \
    python bench.py --mode xe --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 > gpurun_out/s2f/prof.log 2>&1 || exit $?
python scripts/prof_steps.py gpurun_out/s2f/prof/xe_kernel_trace.csv 10 30 adam_update_kernel 'e' > gpurun_out/s2f/steps_xe.txt || exit $?
rm -f gpurun_out/s2f/prof/xe_kernel_trace.csv
head -16 gpurun_out/s2f/steps_xe.txt | cut -c1-110
