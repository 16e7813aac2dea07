#!/bin/bash
# repeated default bench runs on one box (variance check)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/bench_rep.txt
: > $out
for rep in 1 2 3; do
  r=$(timeout -k 10 300 python bench.py --att8 0 2>/dev/null | grep '^{') || exit $?
  echo "default rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
done
timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_rep.log 2>&1 || exit $?
cat $out
