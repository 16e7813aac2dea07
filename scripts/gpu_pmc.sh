#!/bin/bash
# PMC counters of the shipped training step (bench.py, whole step replayed as
# a HIP graph; GRAPH=0 for the eager step): one rocprofv3 pass per counter
# group (the block limits: <= 4 TCC counters, FETCH_SIZE takes 3, WRITE_SIZE
# 2).  Summary over the last 2 steps of each pass: scripts/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-pmc}
GRAPH=${GRAPH:-1}
mkdir -p gpurun_out/$TAG
run() {
  local p=$1; shift
  rm -rf gpurun_out/$TAG/$p
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/$TAG/$p -o $p -- \
    python bench.py --steps 2 --warmup 3 --cuda_graph $GRAPH --att8 0 --beam5 0 --cst 0 --xe 0 ${BENCH_ARGS} \
    > gpurun_out/$TAG/$p.log 2>&1
}
run p1 FETCH_SIZE || exit $?
run p2 WRITE_SIZE || exit $?
run p3 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES || exit $?
run p4 TCC_HIT_sum TCC_MISS_sum || exit $?
python scripts/pmc_summary.py gpurun_out/$TAG 2 > gpurun_out/$TAG/summary.txt
for p in p1 p2 p3 p4; do rm -f gpurun_out/$TAG/$p/${p}_counter_collection.csv.gz; done
head -n 30 gpurun_out/$TAG/summary.txt
