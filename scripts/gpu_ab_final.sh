#!/bin/bash
# X launched after the loss instead of after the rollout; dW under the loop
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_final.txt
: > $out
for rep in 1 2; do
  for cfg in "rollout 3" "loss 3" "rollout 2"; do
    set -- $cfg
    r=$(CSTCAP_X_AT=$1 CSTCAP_VH_SCHED=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "x_at=$1 vh_sched=$2 rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
CSTCAP_X_AT=loss timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_xloss.log 2>&1 || exit $?
cat $out
