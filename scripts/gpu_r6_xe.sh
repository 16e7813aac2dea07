#!/bin/bash
# round 6: XE step stamps + att8 regression A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode xe --stamps 4 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/stamps_xe.json 2> gpurun_out/stamps_xe.err || exit $?
grep -A40 "stamps (us" gpurun_out/stamps_xe.err | head -40
CSTCAP_XE_XAFTER=0 timeout -k 10 300 python bench.py --mode xe --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/xe_noxafter.json 2>&1 || exit $?
grep '^{' gpurun_out/xe_noxafter.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('xe no-x-after', d['ms_per_step'])"
ARMS="base: p32:CSTCAP_PRE16=0 aug0:CSTCAP_DW_AUG=0 demb0:CSTCAP_DEMB_TUNED=0" REPS=1 TAG=a8 BENCH_ARGS="--num_chunks 8" bash scripts/gpu_ab.sh || exit $?
