#!/bin/bash
# vocab kernel microbenchmark (mainloop vs epilogue pieces) + PMC pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
VARIANTS=4,7 DS=1 timeout -k 10 300 python scripts/microbench_kernels.py > gpurun_out/mb_vocab.log 2>&1 || exit $?
VARIANTS=4 DS=0 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/v1 -o v1 \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -- python scripts/microbench_kernels.py > gpurun_out/pmc/v1.log 2>&1 || exit $?
VARIANTS=4 DS=0 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/v2 -o v2 \
  --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM \
  -- python scripts/microbench_kernels.py > gpurun_out/pmc/v2.log 2>&1
echo "rc=$?"
