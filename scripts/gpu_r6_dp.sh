#!/bin/bash
# round 6: DP stand-in priority study (1-rank RCCL)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/dp_standin.py 29517 32 400 10 > gpurun_out/dp_standin.json 2> gpurun_out/dp_standin.err || { tail -20 gpurun_out/dp_standin.err; exit 1; }
cat gpurun_out/dp_standin.json
