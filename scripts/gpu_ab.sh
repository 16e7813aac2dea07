#!/bin/bash
# A/B of an env knob on the bench, alternating runs in one process slot:
#   AB_VAR=NAME AB_VALUES="a b" bash scripts/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in $AB_VALUES; do
    env $AB_VAR=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 \
      --json_out gpurun_out/ab/${AB_VAR}_${v}_$rep.json > gpurun_out/ab/${AB_VAR}_${v}_$rep.log 2>&1 || exit $?
    echo "$AB_VAR=$v rep=$rep $(python -c "import json;d=json.load(open('gpurun_out/ab/${AB_VAR}_${v}_$rep.json'));print(d['ms_per_step'])")"
  done
done
