#!/bin/bash
# decoder-forward microbench, A/B of an env knob (AB_VAR / AB_VALUES)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in $AB_VALUES; do
  echo "$AB_VAR=$v $(env $AB_VAR=$v VARIANTS=4 timeout -k 10 300 python scripts/microbench_decoder.py 2>/dev/null | tail -1)" || exit 1
done
