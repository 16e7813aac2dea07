#!/bin/bash
# round 6: SCST (headline) step kernel table + launch sequence at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_scst
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_scst -o scst -- python bench.py --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/prof_scst.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_scst.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('scst', d['ms_per_step'], 'dev_err', d.get('device_errors'))"
python scripts/prof_steps.py gpurun_out/prof_scst/scst_kernel_trace.csv 10 24 adam_update_kernel 'e' > gpurun_out/steps_scst.txt && head -n 26 gpurun_out/steps_scst.txt
rm -f gpurun_out/prof_scst/scst_kernel_trace.csv
