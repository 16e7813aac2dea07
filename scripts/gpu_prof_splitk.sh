#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for S in 1 2; do
rm -rf gpurun_out/prof_s$S
CSTCAP_BWD_SPLITK=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s$S -o s$S -- \
   python bench.py --steps 5 --warmup 2 > gpurun_out/prof_s$S.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_s$S/s${S}_kernel_trace.csv 7 14 > gpurun_out/prof_s${S}_summary.txt
python scripts/timeline_gaps.py gpurun_out/prof_s$S/s${S}_kernel_trace.csv 3 > gpurun_out/gaps_s$S.txt
done
