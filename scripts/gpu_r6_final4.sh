#!/bin/bash
# round 6 session 2, last call: the host-UBSan engine test + smoke on the final
# .so files, a PMC pass set of the replayed att8 step, and the beam-5 step table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/final_s2c
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_debug.py tests/test_gpu_dist.py > $D/pytest_debug_dist.log 2>&1 || { tail -40 $D/pytest_debug_dist.log; exit 1; }
tail -1 $D/pytest_debug_dist.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
TAG=final_s2c/pmc_att8 BENCH_ARGS="--num_chunks 8" bash scripts/gpu_pmc.sh > /dev/null || exit $?
head -n 14 $D/pmc_att8/summary.txt
rm -rf $D/prof_beam
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_beam -o beam -- python bench.py --mode beam --steps 5 --warmup 3 --att8 0 --cst 0 --xe 0 > $D/prof_beam.log 2>&1 || exit $?
python scripts/prof_steps.py $D/prof_beam/beam_kernel_trace.csv 5 12 beam_fused_step_kernel '_' > $D/steps_beam.txt || exit $?
rm -f $D/prof_beam/beam_kernel_trace.csv
head -8 $D/steps_beam.txt | cut -c1-120
