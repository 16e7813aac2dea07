#!/bin/bash
# round 6: XE vs SCST step on one box -- landmark launches of each step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_graph.py tests/test_gpu_headline.py > gpurun_out/pytest_r6_cmp.log 2>&1 || { tail -30 gpurun_out/pytest_r6_cmp.log; exit 1; }
tail -1 gpurun_out/pytest_r6_cmp.log
for m in scst xe; do
  rm -rf gpurun_out/prof_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$m -o $m -- python bench.py --mode $m --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/prof_$m.log 2>&1 || exit $?
  python scripts/prof_steps.py gpurun_out/prof_$m/${m}_kernel_trace.csv 10 30 adam_update_kernel 'e' > gpurun_out/steps_$m.txt || exit $?
  rm -f gpurun_out/prof_$m/${m}_kernel_trace.csv
  head -1 gpurun_out/steps_$m.txt
  sed -n 27,500p gpurun_out/steps_$m.txt | grep -E "Cijk|lstm_bwd_loop|adam_update|token_group_sum|_loss_fwd|vocab_exp_convert|cider_d|lstm_step_fwd" | cut -c1-100
done
