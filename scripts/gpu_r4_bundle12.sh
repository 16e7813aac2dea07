#!/bin/bash
# round 4 bundle 12: how many hipBLASLt candidates the X plan times; column
# sums at 768 rows per workgroup
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_A="CSTCAP_TUNED_NCAND=32" AB_B="CSTCAP_TUNED_NCAND=96" AB_C="CSTCAP_TUNED_NCAND=8" AB_D="CSTCAP_COLSUM_ROWS=768" \
  REPS=3 bash scripts/gpu_r4_ab.sh || exit $?
