#!/bin/bash
# round 6 session 2: whole-video MFMA attention workgroups (one per video
# over every query slice) -- attention tests, att8 A/B, att8 step table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2h
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention_headline.py tests/test_gpu_attention.py tests/test_gpu_bwd_loop.py tests/test_gpu_cells.py \
  > gpurun_out/s2h/pytest.log 2>&1 || { tail -40 gpurun_out/s2h/pytest.log; exit 1; }
tail -1 gpurun_out/s2h/pytest.log
for i in 1 2; do
  for m in 1 0; do
    CSTCAP_ATT_WHOLE=$m timeout -k 10 300 python bench.py --num_chunks 8 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2h/att8_w${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2h/att8_w${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2h/att8_w${m}_$i.log > gpurun_out/s2h/att8_w${m}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2h/att8_w${m}_$i.json')); print('whole=$m att8', d['ms_per_step'], 'err', d['device_errors'])"
  done
done
rm -rf gpurun_out/s2h/prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2h/prof -o att8 -- \
    python bench.py --steps 6 --warmup 4 --num_chunks 8 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2h/prof.log 2>&1 || exit $?
python scripts/prof_steps.py gpurun_out/s2h/prof/att8_kernel_trace.csv 5 40 adam_update_kernel 'e' > gpurun_out/s2h/steps_att8.txt || exit $?
rm -f gpurun_out/s2h/prof/att8_kernel_trace.csv
head -8 gpurun_out/s2h/steps_att8.txt | cut -c1-110
