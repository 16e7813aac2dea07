#!/bin/bash
# round 4: fused decode step -- its GPU tests, the engine tests that run the
# rollout, then an interleaved A/B of the fused step against the combine launch
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_step.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_decode_step.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_attention_headline.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine.log 2>&1 || exit $?
for i in 1 2; do
  for f in 0 1; do
    CSTCAP_FUSED_DECODE=$f timeout -k 10 300 python bench.py --steps 30 --warmup 5 --att8 0 --json_out gpurun_out/ab_f${f}_$i.json > gpurun_out/ab_f${f}_$i.log 2>&1 || exit $?
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_f${f}_$i.json | sed "s/^/fused=$f rep=$i /"
  done
done
timeout -k 10 300 python bench.py --stamps 10 --json_out gpurun_out/r4_fused_stamps.json > gpurun_out/r4_fused_stamps.log 2>&1 || exit $?
grep '^{' gpurun_out/r4_fused_stamps.log
