#!/bin/bash
# iteration loop: tests -> bench -> decoder microbench -> PMC (VALU/MFMA/waits)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
CSTCAP_VOCAB_VARIANT=${TEST_VARIANT:-4} timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
CSTCAP_VOCAB_VARIANT=${TEST_VARIANT:-4} timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1 || exit $?
VARIANTS=${VARIANTS:-0,3} timeout -k 10 300 python scripts/microbench_decoder.py > gpurun_out/microbench.log 2>&1 || exit $?
[ -n "$SKIP_PMC" ] && exit 0
VARIANTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o p1 \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -- python scripts/microbench_decoder.py > gpurun_out/pmc/p1.log 2>&1 || exit $?
VARIANTS=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/p2 -o p2 \
  --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -- python scripts/microbench_decoder.py > gpurun_out/pmc/p2.log 2>&1
echo "rc=$?"
