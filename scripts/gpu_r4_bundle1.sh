#!/bin/bash
# round 4 bundle: (1) bias column sums with fewer workgroups (test + A/B),
# (2) host enqueue / cProfile of the timed loop, (3) att8 stamps with and
# without the duplicated-row greedy baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_r4_colsum.sh || exit $?
bash scripts/gpu_r4_host.sh || exit $?
for dup in 1 0; do
  CSTCAP_GREEDY_DUP=$dup timeout -k 10 300 python bench.py --stamps 10 --beam5 0 \
    --json_out gpurun_out/r4_att8_dup$dup.json > gpurun_out/r4_att8_dup$dup.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/r4_att8_dup$dup.json'))['att8']
print('dup $dup', d['ms_per_step']); [print('%-16s %8.1f' % kv) for kv in d.get('stamps_us', {}).items()]"
done
