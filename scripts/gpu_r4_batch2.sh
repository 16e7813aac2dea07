#!/bin/bash
# round 4: attention greedy-row test, hipBLASLt algorithm probe of the vocab
# head's backward GEMMs, learning parity on the template task
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_attention_headline.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_att_dup.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_att_dup.log
timeout -k 10 300 python -u scripts/blaslt_probe.py > gpurun_out/blaslt_probe.json 2> gpurun_out/blaslt_probe.err || exit $?
cat gpurun_out/blaslt_probe.json
bash scripts/gpu_r4_learn.sh
