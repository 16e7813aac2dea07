#!/bin/bash
# X = E W behind the greedy decode (CSTCAP_X_AFTER_ROLLOUT): capture probes,
# tests, interleaved headline A/B (att8 included), stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/gpu_capture_probe.py 0 > gpurun_out/probe0.log 2>&1 || exit $?
timeout -k 10 120 python -u scripts/gpu_capture_probe.py 1 > gpurun_out/probe1.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_stamps.py tests/test_gpu_attention_headline.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_xafter.log 2>&1 || exit $?
out=gpurun_out/ab_xafter.txt
: > $out
for rep in 1 2; do
  for cfg in 0 1; do
    r=$(CSTCAP_X_AFTER_ROLLOUT=$cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 2>/dev/null | grep '^{') || exit $?
    echo "x_after=$cfg rep=$rep $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["att8"]["value"], d["att8"]["ms_per_step"])')" >> $out
  done
done
CSTCAP_X_AFTER_ROLLOUT=1 timeout -k 10 300 python bench.py --steps 10 --warmup 5 --stamps 5 > gpurun_out/stamps_xafter.log 2>&1 || exit $?
cat $out
