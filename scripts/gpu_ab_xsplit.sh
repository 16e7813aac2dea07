#!/bin/bash
# split-K of the X = E W GEMM after the rollout (CSTCAP_X_SPLITK)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_X_SPLITK=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k x_after > gpurun_out/pytest_xsplit.log 2>&1 || exit $?
out=gpurun_out/ab_xsplit.txt
: > $out
for rep in 1 2; do
  for cfg in 1 3; do
    r=$(CSTCAP_X_SPLITK=$cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "x_splitk=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
CSTCAP_X_SPLITK=3 timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_xsplit3.log 2>&1 || exit $?
cat $out
