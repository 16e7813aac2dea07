#!/bin/bash
# round 4 bundle 10: video-gate gradient on the side stream after the loop
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CSTCAP_VG_SIDE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_kernels.py tests/test_gpu_attention_headline.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_vg.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_vg.log
[ $e -eq 0 ] || exit $e
AB_A="CSTCAP_VG_SIDE=0" AB_B="CSTCAP_VG_SIDE=1" AB_C="CSTCAP_FEAT_CAT=0" REPS=3 bash scripts/gpu_r4_ab.sh || exit $?
