#!/bin/bash
# A/B of experiment settings (CSTCAP_EXP_* env), interleaved repetitions of
# the headline bench; usage: AB="NAME=ENV ... " REPS=n [BENCH_ARGS=...] bash scripts/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in $(seq 1 ${REPS:-2}); do
  for spec in $AB; do
    name=${spec%%=*}; envs=${spec#*=}
    env ${envs//,/ } timeout -k 10 300 python bench.py --steps ${STEPS:-40} --warmup 5 $BENCH_ARGS --json_out gpurun_out/ab/${name}_$r.json > gpurun_out/ab/${name}_$r.log 2>&1 || exit $?
    echo "$name rep $r: $(python -c "import json;d=json.load(open('gpurun_out/ab/${name}_$r.json'));print(d['value'],d['ms_per_step'])")"
  done
done
