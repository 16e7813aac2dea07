#!/bin/bash
# round 6 final validation at HEAD: full GPU suite, smoke, driver-style bench,
# per-step rocprofv3 table of the headline step, PMC counter passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
grep '^{' gpurun_out/bench_final.log > gpurun_out/bench_final.json
python -c "import json; d=json.load(open('gpurun_out/bench_final.json')); print('scst', d['ms_per_step'], 'cst', d['cst']['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'att8', d['att8']['ms_per_step'], 'beam', d['beam5']['videos_per_s'], 'err', d['device_errors'])"
bash scripts/gpu_r6_scst_prof.sh > gpurun_out/prof_scst_summary.txt || exit $?
head -3 gpurun_out/prof_scst_summary.txt
TAG=pmc_r6 bash scripts/gpu_pmc.sh > /dev/null || exit $?
head -n 12 gpurun_out/pmc_r6/summary.txt
