#!/bin/bash
# interleaved A/B of the dHd chunk schedule (CSTCAP_DHD_CHUNKS) and the
# row-resident decode launch, headline bench; one line per run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_chunks.txt
: > $out
for rep in 1 2; do
  for cfg in 28 2,4 4,8 7,7 2,13; do
    r=$(CSTCAP_DHD_CHUNKS=$cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "chunks=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
  r=$(CSTCAP_DECODE_RR=1 CSTCAP_DHD_CHUNKS=28 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
  echo "rr chunks=28 rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
done
cat $out
