#!/bin/bash
# round 4: issue / wait breakdown of the decode launch and the combine (eager
# step, one rocprofv3 pass per counter group)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc4
run() {
  local tag=$1; shift
  rm -rf gpurun_out/pmc4/$tag
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc4/$tag -o $tag -- \
    python bench.py --steps 2 --warmup 2 --cuda_graph 0 --att8 0 > gpurun_out/pmc4/$tag.log 2>&1
}
run q1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES || exit $?
run q2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES || exit $?
run q3 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE || exit $?
python scripts/pmc_kernel_means.py gpurun_out/pmc4 q1 q2 q3 > gpurun_out/pmc4/means.txt
grep -A30 "vocab_lstm_fwd_kernel\|vocab_combine" gpurun_out/pmc4/means.txt | head -80
