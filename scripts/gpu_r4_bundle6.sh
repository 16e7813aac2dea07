#!/bin/bash
# round 4 bundle 6: GEMM choices under the concurrent schedule -- X through
# the measured hipBLASLt choice; dW_logit through the hand-written GEMM with
# fewer persistent workgroups (CUs left to the reverse loop)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_A="CSTCAP_X=0" AB_B="CSTCAP_TUNED_GEMM=x" AB_C="CSTCAP_SK_GEMM=d CSTCAP_SK_GRID=192" \
  AB_D="CSTCAP_SK_GEMM=d CSTCAP_SK_GRID=128" REPS=3 bash scripts/gpu_r4_ab.sh || exit $?
