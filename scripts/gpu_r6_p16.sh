#!/bin/bash
# round 6: fp16 pre / ptab -- full GPU suite, A/B, att8 + beam bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r6_p16.log 2>&1 || { tail -40 gpurun_out/pytest_r6_p16.log; exit 1; }
tail -2 gpurun_out/pytest_r6_p16.log
ARMS="p32:CSTCAP_PRE16=0 p16:CSTCAP_PRE16=1" REPS=2 TAG=p16 bash scripts/gpu_ab.sh || exit $?
