#!/bin/bash
# round 6: fused XE loss + bf16 video-gate dW: tests, bench, XE step table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_bwd_loop.py tests/test_gpu_graph.py > gpurun_out/pytest_r6_xe3.log 2>&1 || { tail -40 gpurun_out/pytest_r6_xe3.log; exit 1; }
tail -2 gpurun_out/pytest_r6_xe3.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r6_xe3.log 2>&1 || { tail -20 gpurun_out/bench_r6_xe3.log; exit 1; }
grep '^{' gpurun_out/bench_r6_xe3.log
rm -rf gpurun_out/prof_xe
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_xe -o xe -- python bench.py --mode xe --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/prof_xe.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_xe.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('xe', d['ms_per_step'], 'dev_err', d.get('device_errors'))"
python scripts/prof_steps.py gpurun_out/prof_xe/xe_kernel_trace.csv 10 24 adam_update_kernel 'e' > gpurun_out/steps_xe3.txt && head -n 26 gpurun_out/steps_xe3.txt
rm -f gpurun_out/prof_xe/xe_kernel_trace.csv
