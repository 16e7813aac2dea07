#!/bin/bash
# X after the rollout x greedy branch enqueued before / after the rollout
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/gpu_capture_probe.py 1 > gpurun_out/probe1.log 2>&1 || exit $?
out=gpurun_out/ab_xq2.txt
: > $out
for rep in 1 2; do
  for cfg in "0 0" "0 1" "1 0" "1 1"; do
    set -- $cfg
    r=$(CSTCAP_X_AFTER_ROLLOUT=$1 CSTCAP_GREEDY_FIRST=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "x_after=$1 greedy_first=$2 rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
CSTCAP_X_AFTER_ROLLOUT=1 CSTCAP_GREEDY_FIRST=1 timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_xgf.log 2>&1 || exit $?
CSTCAP_X_AFTER_ROLLOUT=0 CSTCAP_GREEDY_FIRST=1 timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_gf.log 2>&1 || exit $?
cat $out
