#!/bin/bash
# where the greedy branch enters the captured step (CSTCAP_GREEDY_AT)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_stamps.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gat.log 2>&1 || exit $?
out=gpurun_out/ab_greedy_at.txt
: > $out
for rep in 1 2; do
  for cfg in 0 4 6 9; do
    r=$(CSTCAP_GREEDY_AT=$cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "greedy_at=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
for cfg in 6; do
  CSTCAP_GREEDY_AT=$cfg timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 > gpurun_out/stamps_gat$cfg.log 2>&1 || exit $?
done
cat $out
