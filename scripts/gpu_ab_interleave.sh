#!/bin/bash
# interleaved env-knob A/B (AB_VAR, AB_VALUES, AB_REPS): value order alternates each rep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 ${AB_REPS:-3}); do
  for v in $AB_VALUES; do
    env $AB_VAR=$v timeout -k 10 300 python bench.py --steps ${AB_STEPS:-60} --warmup 5 $AB_ARGS --json_out gpurun_out/abi_${v}_$r.json > gpurun_out/abi_${v}_$r.log 2>&1 || exit $?
  done
done
