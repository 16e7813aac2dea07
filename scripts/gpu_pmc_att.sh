#!/bin/bash
# PMC counters of the attention microbenchmarks (scripts/microbench_att.py):
# one rocprofv3 pass per SQ counter group; summary per kernel (mean per dispatch)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_att
run() {
  local tag=$1; shift
  rm -rf gpurun_out/pmc_att/$tag
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_att/$tag -o $tag -- \
    python scripts/microbench_att.py > gpurun_out/pmc_att/$tag.log 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit $?
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC || exit $?
python scripts/pmc_kernel_means.py gpurun_out/pmc_att a b > gpurun_out/pmc_att/summary.txt
