#!/bin/bash
# bf16-operand backward GEMMs of the attention input projections (CSTCAP_ATT_BF16_BWD)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_attention_headline.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_attbwd.log 2>&1 || exit $?
out=gpurun_out/ab_attbwd.txt
: > $out
for rep in 1 2; do
  for cfg in 0 1; do
    r=$(CSTCAP_ATT_BF16_BWD=$cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --num_chunks 8 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "att_bf16_bwd=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
cat $out
