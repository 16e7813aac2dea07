#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_LAUNCH_CHECK=2 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bwd_loop.py -k "matches or timeout" > gpurun_out/pytest_r6_dbg.log 2>&1
grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_r6_dbg.log | head -30
