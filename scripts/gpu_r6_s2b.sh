#!/bin/bash
# round 6 session 2: att8 A/B of the greedy MFMA attention (one row per video),
# then the att8 step table (split-bf16 FeatPool kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2b
for i in 1 2; do
  for m in 1 0; do
    CSTCAP_GREEDY_ATT_MFMA=$m timeout -k 10 300 python bench.py --num_chunks 8 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2b/ab_g${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2b/ab_g${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2b/ab_g${m}_$i.log > gpurun_out/s2b/ab_g${m}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2b/ab_g${m}_$i.json')); print('greedy_mfma=$m', d['ms_per_step'], 'err', d['device_errors'])"
  done
done
rm -rf gpurun_out/s2b/prof
CSTCAP_GREEDY_ATT_MFMA=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2b/prof -o att8 -- \
    python bench.py --steps 6 --warmup 4 --num_chunks 8 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2b/prof.log 2>&1 || exit $?
python scripts/prof_steps.py gpurun_out/s2b/prof/att8_kernel_trace.csv 5 40 adam_update_kernel 'e' > gpurun_out/s2b/steps_att8_g0.txt || exit $?
rm -f gpurun_out/s2b/prof/att8_kernel_trace.csv
grep -i "featpool\|att_fwd\|^window" gpurun_out/s2b/steps_att8_g0.txt | head -12
