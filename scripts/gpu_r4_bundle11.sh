#!/bin/bash
# round 4 bundle 11: dW_logit GEMM choice now that it runs under the reverse
# loop (vh_sched 2): PyTorch split-K (shipped) vs measured hipBLASLt choice vs
# the hand-written TN GEMM (full / half grid)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_A="CSTCAP_X=0" AB_B="CSTCAP_TUNED_GEMM=1" AB_C="CSTCAP_SK_GEMM=d" AB_D="CSTCAP_SK_GEMM=d CSTCAP_SK_GRID=128" \
  REPS=3 bash scripts/gpu_r4_ab.sh || exit $?
