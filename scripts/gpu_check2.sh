#!/bin/bash
# full GPU suite, smoke, A/B of the bias gradient inside the dW GEMM,
# headline (+att8) bench, stamps, kernel summaries of both configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
out=gpurun_out/ab_dbdw.txt
: > $out
for rep in 1 2; do
  for cfg in 0 1; do
    r=$(CSTCAP_DB_IN_DW=$cfg timeout -k 10 200 python bench.py --steps 30 --warmup 5 --att8 0 2>/dev/null | grep '^{') || exit $?
    echo "db_in_dw=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --json_out gpurun_out/bench_c2.json > gpurun_out/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 > gpurun_out/stamps_c2.log 2>&1 || exit $?
TAG=c2 bash scripts/gpu_prof.sh || exit $?
BENCH_ARGS="--num_chunks 8" TAG=c2att8 bash scripts/gpu_prof.sh || exit $?
cat $out
