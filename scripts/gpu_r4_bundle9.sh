#!/bin/bash
# round 4 bundle 9: bias column-sum workgroup size under the concurrent
# vocab-head schedule (512 / 1024 / 2048 rows per workgroup)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_A="CSTCAP_COLSUM_ROWS=1024" AB_B="CSTCAP_COLSUM_ROWS=512" AB_C="CSTCAP_COLSUM_ROWS=2048" \
  REPS=3 AB_ATT8=1 bash scripts/gpu_r4_ab.sh || exit $?
