#!/bin/bash
# X split-K A/B, then PMC counters of the eager step (headline)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu_ab_xsplit.sh || exit $?
bash scripts/gpu_pmc.sh || exit $?
