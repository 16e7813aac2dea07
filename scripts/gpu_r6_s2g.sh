#!/bin/bash
# round 6 session 2: XE decode launches (vocab tiles of step t + the whole LSTM
# step t+1, combines on a side stream) -- tests, A/B, step table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2g
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_cells.py tests/test_gpu_kernels.py \
  tests/test_gpu_bwd_loop.py \
  > gpurun_out/s2g/pytest.log 2>&1 || { tail -40 gpurun_out/s2g/pytest.log; exit 1; }
tail -1 gpurun_out/s2g/pytest.log
for i in 1 2; do
  for m in 1 0; do
    CSTCAP_XE_ROWS=$m timeout -k 10 300 python bench.py --mode xe --att8 0 --beam5 0 --cst 0 > gpurun_out/s2g/xe${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2g/xe${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2g/xe${m}_$i.log > gpurun_out/s2g/xe${m}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2g/xe${m}_$i.json')); print('xe_rows=$m', d['ms_per_step'], 'loss', d['final_loss'], 'err', d['device_errors'])"
  done
done
rm -rf gpurun_out/s2g/prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2g/prof -o xe -- \
    python bench.py --mode xe --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 > gpurun_out/s2g/prof.log 2>&1 || exit $?
python scripts/prof_steps.py gpurun_out/s2g/prof/xe_kernel_trace.csv 10 30 adam_update_kernel 'e' > gpurun_out/s2g/steps_xe.txt || exit $?
rm -f gpurun_out/s2g/prof/xe_kernel_trace.csv
head -12 gpurun_out/s2g/steps_xe.txt | cut -c1-110
