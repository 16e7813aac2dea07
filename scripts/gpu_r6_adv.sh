#!/bin/bash
# round 6: advisor items (attention tests), DP stand-in study
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention.py tests/test_gpu_attention_headline.py tests/test_gpu_bwd_loop.py tests/test_gpu_kernels.py > gpurun_out/pytest_r6_adv.log 2>&1
grep -E "PASS|FAIL|Error" gpurun_out/pytest_r6_adv.log | tail -40
tail -2 gpurun_out/pytest_r6_adv.log
timeout -k 10 400 python scripts/dp_standin.py 29517 32 400 10 > gpurun_out/dp_standin.json 2> gpurun_out/dp_standin.err || { tail -20 gpurun_out/dp_standin.err; exit 1; }
cat gpurun_out/dp_standin.json
