#!/bin/bash
# round 6 session 2: split-bf16 FeatPool + unrolled epilogue; greedy MFMA
# attention (opt-in) -- featpool / attention / headline / graph tests, att8
# and headline bench, att8 step table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2d
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_attention_headline.py tests/test_gpu_attention.py \
  tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_cells.py \
  > gpurun_out/s2d/pytest.log 2>&1 || { tail -40 gpurun_out/s2d/pytest.log; exit 1; }
tail -1 gpurun_out/s2d/pytest.log
CSTCAP_GREEDY_ATT_MFMA=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention.py -k greedy > gpurun_out/s2d/pytest_greedy_mfma.log 2>&1 || { tail -40 gpurun_out/s2d/pytest_greedy_mfma.log; exit 1; }
tail -1 gpurun_out/s2d/pytest_greedy_mfma.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --num_chunks 8 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2d/att8_$i.log 2>&1 || { tail -20 gpurun_out/s2d/att8_$i.log; exit 1; }
  grep '^{' gpurun_out/s2d/att8_$i.log > gpurun_out/s2d/att8_$i.json
  python -c "import json; d=json.load(open('gpurun_out/s2d/att8_$i.json')); print('att8', d['ms_per_step'], 'err', d['device_errors'])"
  timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > gpurun_out/s2d/head_$i.log 2>&1 || { tail -20 gpurun_out/s2d/head_$i.log; exit 1; }
  grep '^{' gpurun_out/s2d/head_$i.log > gpurun_out/s2d/head_$i.json
  python -c "import json; d=json.load(open('gpurun_out/s2d/head_$i.json')); print('scst', d['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'err', d['device_errors'])"
done
rm -rf gpurun_out/s2d/prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2d/prof -o att8 -- \
    python bench.py --steps 6 --warmup 4 --num_chunks 8 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2d/prof.log 2>&1 || exit $?
python scripts/prof_steps.py gpurun_out/s2d/prof/att8_kernel_trace.csv 5 40 adam_update_kernel 'e' > gpurun_out/s2d/steps_att8.txt || exit $?
rm -f gpurun_out/s2d/prof/att8_kernel_trace.csv
grep -i "featpool\|^window" gpurun_out/s2d/steps_att8.txt | head -8
