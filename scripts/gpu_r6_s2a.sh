#!/bin/bash
# round 6 session 2: greedy MFMA attention (one row per video) + split-bf16 FeatPool
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s2a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention_headline.py tests/test_gpu_attention.py tests/test_gpu_kernels.py \
  > gpurun_out/s2a/pytest.log 2>&1 || { tail -40 gpurun_out/s2a/pytest.log; exit 1; }
tail -1 gpurun_out/s2a/pytest.log
timeout -k 10 400 python bench.py --beam5 0 > gpurun_out/s2a/bench.log 2>&1 || { tail -20 gpurun_out/s2a/bench.log; exit 1; }
grep '^{' gpurun_out/s2a/bench.log > gpurun_out/s2a/bench.json
python -c "import json; d=json.load(open('gpurun_out/s2a/bench.json')); print('scst', d['ms_per_step'], 'cst', d['cst']['ms_per_step'], 'xe', d['xe']['ms_per_step'], 'att8', d['att8']['ms_per_step'], 'err', d['device_errors'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_headline.py tests/test_gpu_graph.py tests/test_gpu_cst.py \
  > gpurun_out/s2a/pytest2.log 2>&1 || { tail -40 gpurun_out/s2a/pytest2.log; exit 1; }
tail -1 gpurun_out/s2a/pytest2.log
