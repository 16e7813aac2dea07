#!/bin/bash
# interleaved A/B: token-table prefetch under the prologue (CSTCAP_PTAB_PREFETCH)
# x vocab-head schedule (CSTCAP_VH_SCHED 0: dW + column sums after the loop,
# 3: column sums under the loop) x split-K of the dW_logit GEMM
# (CSTCAP_DW_SPLITK); device stamps of two of them
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_cells.py tests/test_gpu_headline.py tests/test_gpu_stamps.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sched.log 2>&1 || exit $?
CSTCAP_DW_SPLITK=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_splitk.log 2>&1 || exit $?
out=gpurun_out/ab_sched.txt
: > $out
for rep in 1 2; do
  for cfg in "0 0 1" "1 0 1" "1 3 1" "1 0 4" "1 3 4" "1 3 7"; do
    set -- $cfg
    r=$(CSTCAP_PTAB_PREFETCH=$1 CSTCAP_VH_SCHED=$2 CSTCAP_DW_SPLITK=$3 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "ptab_prefetch=$1 vh_sched=$2 dw_splitk=$3 rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
for cfg in "0 1" "3 4"; do
  set -- $cfg
  CSTCAP_VH_SCHED=$1 CSTCAP_DW_SPLITK=$2 timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 --att8 0 > gpurun_out/stamps_sched$1_$2.log 2>&1 || exit $?
done
cat $out
