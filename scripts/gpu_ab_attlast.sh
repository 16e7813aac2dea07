#!/bin/bash
# attention workgroups last in the decode launch (CSTCAP_ATT_LAST), 8 frames
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_ATT_LAST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_attention_headline.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_attlast.log 2>&1 || exit $?
out=gpurun_out/ab_attlast.txt
: > $out
for rep in 1 2; do
  for cfg in 0 1; do
    r=$(CSTCAP_ATT_LAST=$cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --num_chunks 8 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "att_last=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
cat $out
