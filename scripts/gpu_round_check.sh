#!/bin/bash
# round-end style check: GPU tests, smoke(), headline + attention benches,
# rocprofv3 kernel trace + --stats of the headline (per-kernel summary, step timeline)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --json_out gpurun_out/bench_hip.json > gpurun_out/bench_hip.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --num_chunks 8 --json_out gpurun_out/bench_att8.json > gpurun_out/bench_att8.log 2>&1 || exit $?
rm -rf gpurun_out/prof_rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rc -o rc -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof_rc.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_rc/rc_kernel_trace.csv 7 40 > gpurun_out/prof_rc_summary.txt
python scripts/step_timeline.py gpurun_out/prof_rc/rc_kernel_trace.csv 1 > gpurun_out/step_timeline_rc.txt
rm -rf gpurun_out/prof_att8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_att8 -o att8 -- python bench.py --steps 5 --warmup 2 --num_chunks 8 > gpurun_out/prof_att8.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_att8/att8_kernel_trace.csv 7 40 > gpurun_out/prof_att8_summary.txt
