#!/bin/bash
# row-resident decode launch: microbenchmark breakdown + PMC passes, then the
# headline beam test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_rr
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_rr.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rr.log 2>&1 || exit $?
timeout -k 10 200 python scripts/microbench_rr.py > gpurun_out/mb_rr.json 2> gpurun_out/mb_rr.err || exit $?
run() {
  local tag=$1; shift
  rm -rf gpurun_out/pmc_rr/$tag
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_rr/$tag -o $tag -- \
    python scripts/microbench_rr.py > gpurun_out/pmc_rr/$tag.log 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit $?
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS || exit $?
run c SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL || exit $?
python scripts/pmc_kernel_means.py gpurun_out/pmc_rr a b c > gpurun_out/pmc_rr/summary.txt
CSTCAP_DECODE_RR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -v --timeout 200 --timeout-method thread -p no:cacheprovider -k beam5 > gpurun_out/pytest_beam5.log 2>&1
exit 0
