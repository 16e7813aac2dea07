#!/bin/bash
# graph executor knobs: DEBUG_HIP_GRAPH_BATCH_SIZE (node submission batching)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_batch.txt
: > $out
for rep in 1 2; do
  for cfg in 0 4 16 64; do
    if [ "$cfg" = "0" ]; then unset DEBUG_HIP_GRAPH_BATCH_SIZE; else export DEBUG_HIP_GRAPH_BATCH_SIZE=$cfg; fi
    r=$(timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "graph_batch=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
unset DEBUG_HIP_GRAPH_BATCH_SIZE
for cfg in 16 64; do
  DEBUG_HIP_GRAPH_BATCH_SIZE=$cfg timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_batch$cfg.log 2>&1 || exit $?
done
cat $out
