#!/bin/bash
# round 4: MFMA attention in beam search -- attention tests (beam vs torch,
# MFMA vs VALU scorer) and the beam decode time with attention
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_attention_headline.py -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_beamatt.log 2>&1
e=$?; tail -n 3 gpurun_out/pytest_beamatt.log
[ $e -eq 0 ] || exit $e
for f in 1 0; do
  CSTCAP_BEAM_ATT_MFMA=$f timeout -k 10 300 python bench.py --mode beam --num_chunks 8 --steps 10 --warmup 2 \
    --json_out gpurun_out/beamatt_$f.json > gpurun_out/beamatt_$f.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/beamatt_$f.json')); print('mfma=$f', d['value'], d['unit'], d['ms_per_step'])"
done
