#!/bin/bash
# round 6 session 2: host enqueue time per replayed step vs the synced step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2i
timeout -k 10 300 python bench.py --sync_debug 1 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2i/sd_scst.log 2>&1 || { tail -20 gpurun_out/s2i/sd_scst.log; exit 1; }
grep "sync_debug\|^{" gpurun_out/s2i/sd_scst.log | cut -c1-200
timeout -k 10 300 python bench.py --mode xe --sync_debug 1 --att8 0 --beam5 0 --cst 0 > gpurun_out/s2i/sd_xe.log 2>&1 || { tail -20 gpurun_out/s2i/sd_xe.log; exit 1; }
grep "sync_debug" gpurun_out/s2i/sd_xe.log
timeout -k 10 300 python bench.py --stamps 1 --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/s2i/stamps.log 2>&1 || { tail -20 gpurun_out/s2i/stamps.log; exit 1; }
grep '^{' gpurun_out/s2i/stamps.log > gpurun_out/s2i/stamps.json
python -c "import json; d=json.load(open('gpurun_out/s2i/stamps.json')); print(d.get('stamps_us'))"
