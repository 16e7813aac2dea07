#!/bin/bash
# round 6: att8 step tables, round-5 tree vs HEAD, one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in r5 r6; do
  rm -rf gpurun_out/prof_att8_$t
  if [ $t = r5 ]; then d=r5ref; x=""; else d=.; x="--xe 0"; fi
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_att8_$t -o att8 -- \
    python bench.py --steps 6 --warmup 4 --num_chunks 8 --beam5 0 --cst 0 $x > $GRAFT_REPO_ROOT/gpurun_out/prof_att8_$t.log 2>&1) || exit $?
  python scripts/prof_steps.py gpurun_out/prof_att8_$t/att8_kernel_trace.csv 5 40 adam_update_kernel 'e' > gpurun_out/steps_att8_$t.txt || exit $?
  rm -f gpurun_out/prof_att8_$t/att8_kernel_trace.csv
  head -n 42 gpurun_out/steps_att8_$t.txt | cut -c1-110
done
