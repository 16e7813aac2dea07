#!/bin/bash
# decode (row-resident launch) + attention + graph + headline GPU tests,
# attention microbenchmarks, benches, kernel-trace profiles of the concat and
# att8 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_rr.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rr.log 2>&1 || exit $?
CSTCAP_DECODE_RR=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_attention_headline.py tests/test_gpu_attention.py tests/test_gpu_graph.py tests/test_gpu_headline.py tests/test_gpu_kernels.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_att.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_hip.log 2>&1 || exit $?
CSTCAP_DECODE_RR=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --att8 0 > gpurun_out/bench_hip_rr.log 2>&1 || exit $?
CSTCAP_DECODE_RR=1 TAG=rc bash scripts/gpu_prof.sh || exit $?
TAG=att8 BENCH_ARGS="--num_chunks 8" bash scripts/gpu_prof.sh || exit $?
timeout -k 10 200 python scripts/microbench_att.py > gpurun_out/mb_att.json 2> gpurun_out/mb_att.err || exit $?
exit $rc
