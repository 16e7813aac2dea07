#!/bin/bash
# X after the rollout: which stream, and the graph executor's queue count
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_xq.txt
: > $out
for rep in 1 2; do
  for cfg in "0 own 0" "1 ptab 0" "0 own 8" "1 own 8" "1 ptab 8"; do
    set -- $cfg
    if [ "$3" = "0" ]; then unset DEBUG_HIP_FORCE_GRAPH_QUEUES; else export DEBUG_HIP_FORCE_GRAPH_QUEUES=$3; fi
    r=$(CSTCAP_X_AFTER_ROLLOUT=$1 CSTCAP_X_STREAM=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "x_after=$1 stream=$2 graph_queues=$3 rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
unset DEBUG_HIP_FORCE_GRAPH_QUEUES
CSTCAP_X_AFTER_ROLLOUT=1 CSTCAP_X_STREAM=ptab timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_xptab.log 2>&1 || exit $?
DEBUG_HIP_FORCE_GRAPH_QUEUES=8 CSTCAP_X_AFTER_ROLLOUT=1 timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_xq8.log 2>&1 || exit $?
cat $out
