#!/bin/bash
# round 6 session 2 final validation at HEAD: full GPU suite, smoke,
# driver-style bench, headline + XE per-step rocprofv3 tables, PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/final_s2b
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
grep '^{' $D/bench.log > $D/bench.json
python -c "import json; d=json.load(open('$D/bench.json')); print('scst', d['ms_per_step'], 'cst', d['cst']['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'att8', d['att8']['ms_per_step'], 'beam', d['beam5']['videos_per_s'], 'err', d['device_errors'])"
rm -rf $D/prof_scst
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_scst -o scst -- python bench.py --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 --xe 0 > $D/prof_scst.log 2>&1 || exit $?
python scripts/prof_steps.py $D/prof_scst/scst_kernel_trace.csv 10 24 adam_update_kernel 'e' > $D/steps_scst.txt || exit $?
rm -f $D/prof_scst/scst_kernel_trace.csv
head -3 $D/steps_scst.txt | cut -c1-150
rm -rf $D/prof_xe
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/prof_xe -o xe -- python bench.py --mode xe --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 > $D/prof_xe.log 2>&1 || exit $?
python scripts/prof_steps.py $D/prof_xe/xe_kernel_trace.csv 10 30 adam_update_kernel 'e' > $D/steps_xe.txt || exit $?
rm -f $D/prof_xe/xe_kernel_trace.csv
head -3 $D/steps_xe.txt | cut -c1-150
TAG=final_s2b/pmc bash scripts/gpu_pmc.sh > /dev/null || exit $?
head -n 8 $D/pmc/summary.txt
