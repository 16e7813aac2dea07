#!/bin/bash
# round-4 baseline on the box: default bench (headline + att8) with device stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --stamps 10 --json_out gpurun_out/r4_base.json > gpurun_out/r4_base.log 2>&1 || exit $?
grep '^{' gpurun_out/r4_base.log
