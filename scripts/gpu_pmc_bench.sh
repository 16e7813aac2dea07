#!/bin/bash
# PMC passes over a short headline bench (one counter group per run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcb
rm -rf gpurun_out/pmcb/*
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcb/p1 -o p1 \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -- python bench.py --steps 2 --warmup 1 > gpurun_out/pmcb/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcb/p2 -o p2 \
  --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM \
  -- python bench.py --steps 2 --warmup 1 > gpurun_out/pmcb/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmcb/p3 -o p3 \
  --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
  -- python bench.py --steps 2 --warmup 1 > gpurun_out/pmcb/p3.log 2>&1 || exit $?
