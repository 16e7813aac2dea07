#!/bin/bash
# round 4 bundle 2: the vocab head's dW_logit placement / GEMM choice
# (A/B/C/D), then a kernel + memory-copy trace of back-to-back steps for the
# gap between replays
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_A="CSTCAP_X=0" AB_B="CSTCAP_VH_SCHED=2" AB_C="CSTCAP_TUNED_GEMM=d" AB_D="CSTCAP_SK_GEMM=d" \
  REPS=3 bash scripts/gpu_r4_ab.sh || exit $?
rm -rf gpurun_out/prof_gap
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_gap -o gap -- \
  python bench.py --steps 10 --warmup 3 --att8 0 --beam5 0 > gpurun_out/prof_gap.log 2>&1 || exit $?
f=$(find gpurun_out/prof_gap -name "*kernel_trace.csv" | head -n 1)
python scripts/timeline_gaps.py "$f" 4 > gpurun_out/gaps.txt 2>&1
head -n 40 gpurun_out/gaps.txt
m=$(find gpurun_out/prof_gap -name "*memory_copy_trace.csv" | head -n 1)
[ -n "$m" ] && python - "$m" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print('memory copies:', len(rows))
for r in rows[-12:]:
    print({k: r[k] for k in r if k in ('Direction', 'Size', 'Start_Timestamp', 'End_Timestamp')})
PY
exit 0
