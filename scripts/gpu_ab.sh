#!/bin/bash
# Interleaved A/B of the headline step: ARMS = "name:ENV=V,ENV2=V2 name2:..."
# (an arm with no variables: "name:"), REPS rounds, each arm one driver-style
# bench run (att8 / beam5 / cst off); prints ms per step per arm and round.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-ab}
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for arm in $ARMS; do
    name=${arm%%:*}; vars=${arm#*:}
    env $(echo "$vars" | tr ',' ' ') timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 --xe 0 $BENCH_ARGS \
      > gpurun_out/ab_${TAG}_${name}_$rep.json 2> gpurun_out/ab_${TAG}_${name}_$rep.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'])" gpurun_out/ab_${TAG}_${name}_$rep.json $name $rep
  done
done
