#!/bin/bash
# round 6: loop microbench variants + dW augmented-rows A/B + tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 0 1 2 4 5; do timeout -k 10 120 python scripts/microbench_loop.py 1280 512 29 20 $d || exit $?; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bwd_loop.py tests/test_gpu_wgrad.py tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_kernels.py > gpurun_out/pytest_r6_mb.log 2>&1 || { tail -40 gpurun_out/pytest_r6_mb.log; exit 1; }
tail -2 gpurun_out/pytest_r6_mb.log
ARMS="col:CSTCAP_DW_AUG=0,CSTCAP_DEMB_TUNED=0 aug:CSTCAP_DW_AUG=1,CSTCAP_DEMB_TUNED=0 augd:CSTCAP_DW_AUG=1,CSTCAP_DEMB_TUNED=1" REPS=2 TAG=aug bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 python bench.py --stamps 4 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/stamps_aug.json 2> gpurun_out/stamps_aug.err || exit $?
grep -A40 "stamps (us" gpurun_out/stamps_aug.err | head -40
