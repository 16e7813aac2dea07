#!/bin/bash
# round 4: the hand-written X = E W GEMM -- exactness tests, probe vs
# hipBLASLt, then an interleaved full-step A/B (default / tuned hipBLASLt /
# hand-written GEMM)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_sk.py tests/test_gpu_attention.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sk.log 2>&1
e=$?; tail -n 4 gpurun_out/pytest_sk.log
[ $e -eq 0 ] || exit $e
timeout -k 10 200 python scripts/sk_probe.py > gpurun_out/sk_probe.json 2> gpurun_out/sk_probe.err || exit $?
cat gpurun_out/sk_probe.json
AB_A="CSTCAP_X=0" AB_B="CSTCAP_TUNED_GEMM=1" AB_C="CSTCAP_SK_GEMM=1" REPS=3 bash scripts/gpu_r4_ab.sh
