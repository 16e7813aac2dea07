#!/bin/bash
# round 4: kernel traces of the headline bench with the two-launch decode
# step and with the fused one (combine folded into the decode launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in 0 1; do
  rm -rf gpurun_out/prof_fz$f
  CSTCAP_FUSED_DECODE=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fz$f -o fz$f -- python bench.py --steps 5 --warmup 3 --att8 0 > gpurun_out/prof_fz$f.log 2>&1 || exit $?
  python scripts/prof_summary.py gpurun_out/prof_fz$f/fz${f}_kernel_trace.csv 5 45 > gpurun_out/prof_fz${f}_summary.txt
  python scripts/step_timeline.py gpurun_out/prof_fz$f/fz${f}_kernel_trace.csv 1 > gpurun_out/step_timeline_fz$f.txt
  rm -rf gpurun_out/prof_fz$f
done
head -25 gpurun_out/prof_fz0_summary.txt gpurun_out/prof_fz1_summary.txt
