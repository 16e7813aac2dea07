#!/bin/bash
# PMC counters of one eager training step (bench.py, --cuda_graph 0: same
# kernels, dispatched one by one so the counter collection sees each): one
# rocprofv3 pass per counter group (the block limits: <= 4 TCC counters,
# FETCH_SIZE takes 3, WRITE_SIZE 2).  Summary: scripts/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
run() {
  local tag=$1; shift
  rm -rf gpurun_out/pmc/$tag
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$tag -o $tag -- \
    python bench.py --steps 2 --warmup 2 --cuda_graph 0 ${BENCH_ARGS} > gpurun_out/pmc/$tag.log 2>&1
}
run p1 FETCH_SIZE || exit $?
run p2 WRITE_SIZE || exit $?
run p3 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES || exit $?
run p4 TCC_HIT_sum TCC_MISS_sum || exit $?
python scripts/pmc_summary.py gpurun_out/pmc 4 > gpurun_out/pmc/summary.txt
