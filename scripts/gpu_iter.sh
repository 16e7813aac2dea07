#!/bin/bash
# iteration check: the whole GPU suite, an interleaved A/B of experiment
# settings (AB="name=ENV,... ..." as in gpu_ab.sh; optional), the headline
# and attention benches, single-kernel microbenchmarks and a kernel profile
# of the attention configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
if [ -n "$AB" ]; then bash scripts/gpu_ab.sh > gpurun_out/ab_summary.txt 2>&1 || exit $?; fi
ATT=1 CS=0 timeout -k 10 200 python scripts/microbench_kernels.py > gpurun_out/microbench.json 2> gpurun_out/microbench.err || exit $?
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --num_chunks 8 --json_out gpurun_out/bench_att8.json > gpurun_out/bench_att8.log 2>&1 || exit $?
rm -rf gpurun_out/prof_att8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_att8 -o att8 -- python bench.py --steps 5 --warmup 2 --num_chunks 8 > gpurun_out/prof_att8.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_att8/att8_kernel_trace.csv 7 40 > gpurun_out/prof_att8_summary.txt
