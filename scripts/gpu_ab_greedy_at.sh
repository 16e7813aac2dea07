#!/bin/bash
# greedy insertion point x X after the rollout
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_greedy_at2.txt
: > $out
for rep in 1 2; do
  for cfg in "0 1" "0 0" "6 0" "3 0"; do
    set -- $cfg
    r=$(CSTCAP_GREEDY_AT=$1 CSTCAP_X_AFTER_ROLLOUT=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "greedy_at=$1 x_after=$2 rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
CSTCAP_GREEDY_AT=6 CSTCAP_X_AFTER_ROLLOUT=0 timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_gat6_nox.log 2>&1 || exit $?
cat $out
