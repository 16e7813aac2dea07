#!/bin/bash
# iteration check: graph + kernel GPU tests first, then the whole GPU suite,
# an interleaved A/B of experiment settings (AB="name=ENV,... ..." as in
# gpu_ab.sh; optional), the headline and attention benches and a kernel
# profile of the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_graph.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
if [ -n "$AB" ]; then bash scripts/gpu_ab.sh > gpurun_out/ab_summary.txt 2>&1 || exit $?; fi
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --num_chunks 8 --json_out gpurun_out/bench_att8.json > gpurun_out/bench_att8.log 2>&1 || exit $?
rm -rf gpurun_out/prof_rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rc -o rc -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_rc.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_rc/rc_kernel_trace.csv 5 45 > gpurun_out/prof_rc_summary.txt
python scripts/step_timeline.py gpurun_out/prof_rc/rc_kernel_trace.csv 1 > gpurun_out/step_timeline_rc.txt
