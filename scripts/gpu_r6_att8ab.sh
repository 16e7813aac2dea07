#!/bin/bash
# round 6: att8 and headline, round-5 tree (r5ref/, built in place) vs HEAD, interleaved on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  (cd r5ref && timeout -k 10 300 python bench.py --num_chunks 8 --beam5 0 --cst 0 > ../gpurun_out/ab_r5_att8_$i.log 2>&1) || { tail -20 gpurun_out/ab_r5_att8_$i.log; exit 1; }
  grep '^{' gpurun_out/ab_r5_att8_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r5 att8', d['ms_per_step'])"
  timeout -k 10 300 python bench.py --num_chunks 8 --beam5 0 --cst 0 --xe 0 > gpurun_out/ab_r6_att8_$i.log 2>&1 || { tail -20 gpurun_out/ab_r6_att8_$i.log; exit 1; }
  grep '^{' gpurun_out/ab_r6_att8_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r6 att8', d['ms_per_step'], d.get('device_errors'))"
  CSTCAP_DW_AUG=1 timeout -k 10 300 python bench.py --num_chunks 8 --beam5 0 --cst 0 --xe 0 > gpurun_out/ab_r6aug_att8_$i.log 2>&1 || { tail -20 gpurun_out/ab_r6aug_att8_$i.log; exit 1; }
  grep '^{' gpurun_out/ab_r6aug_att8_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r6 aug att8', d['ms_per_step'], d.get('device_errors'))"
done
for i in 1; do
  (cd r5ref && timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > ../gpurun_out/ab_r5_head_$i.log 2>&1) || { tail -20 gpurun_out/ab_r5_head_$i.log; exit 1; }
  grep '^{' gpurun_out/ab_r5_head_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r5 head', d['ms_per_step'])"
  timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 --xe 0 > gpurun_out/ab_r6_head_$i.log 2>&1 || { tail -20 gpurun_out/ab_r6_head_$i.log; exit 1; }
  grep '^{' gpurun_out/ab_r6_head_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r6 head', d['ms_per_step'])"
done
