#!/bin/bash
# PMC counters for the decoder kernels (separate runs, kernel-trace only; no sys/runtime trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
export VARIANTS=0
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o p1 \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -- python scripts/microbench_decoder.py > gpurun_out/pmc/p1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/p2 -o p2 \
  --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -- python scripts/microbench_decoder.py > gpurun_out/pmc/p2.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/p3 -o p3 \
  --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum \
  -- python scripts/microbench_decoder.py > gpurun_out/pmc/p3.log 2>&1
echo "rc=$?"
