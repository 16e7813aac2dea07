#!/bin/bash
# per-token sums before the side stream's dW GEMM (CSTCAP_TOKSUM_FIRST)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_toksum.log 2>&1 || exit $?
out=gpurun_out/ab_toksum.txt
: > $out
for rep in 1 2 3; do
  for cfg in 0 1; do
    r=$(CSTCAP_TOKSUM_FIRST=$cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "toksum_first=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
CSTCAP_TOKSUM_FIRST=1 timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_toksum.log 2>&1 || exit $?
cat $out
