#!/bin/bash
# round 4: device stamps of the headline step (optional env: STAMP_ENV, e.g.
# CSTCAP_INTERLEAVE_GREEDY=0), printed per phase
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-st}
env $STAMP_ENV timeout -k 10 300 python bench.py --stamps 10 --att8 0 --json_out gpurun_out/r4_$TAG.json > gpurun_out/r4_$TAG.log 2>&1 || exit $?
python -c "
import json; d=json.load(open('gpurun_out/r4_$TAG.json'))
print(d['ms_per_step']); [print('%-16s %8.1f' % kv) for kv in d['stamps_us'].items()]"
