#!/bin/bash
# round 6 session 2: att8 with the augmented-row dW GEMM (bias in the GEMM) vs
# the column sums under the per-step loop (default), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2p
for i in 1 2 3; do
  for m in 1 d; do
    if [ $m = d ]; then envs="CSTCAP_DW_AUG="; else envs="CSTCAP_DW_AUG=1"; fi
    env $envs timeout -k 10 300 python bench.py --num_chunks 8 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2p/a${m}_$i.log 2>&1 || { tail -20 gpurun_out/s2p/a${m}_$i.log; exit 1; }
    grep '^{' gpurun_out/s2p/a${m}_$i.log > gpurun_out/s2p/a${m}_$i.json
    python -c "import json; d=json.load(open('gpurun_out/s2p/a${m}_$i.json')); print('aug=$m att8', d['ms_per_step'], 'err', d['device_errors'])"
  done
done
