#!/bin/bash
# generic env-knob A/B: AB_VAR=name AB_VALUES="0 1" -> bench per value (headline config)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $AB_VALUES; do
  env $AB_VAR=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 $AB_ARGS --json_out gpurun_out/ab_$v.json > gpurun_out/ab_$v.log 2>&1 || exit $?
done
for v in $AB_VALUES; do
  env $AB_VAR=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 $AB_ARGS --json_out gpurun_out/ab2_$v.json > gpurun_out/ab2_$v.log 2>&1 || exit $?
done
