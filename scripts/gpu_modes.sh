#!/bin/bash
# Per-recipe throughput on 1x MI355X (BASELINE.json configs 2 and 3):
#   XE warm-up and CST (SCB* sample baseline) with the fused HIP engine, and
#   the same recipes with PyTorch ops (+ CPU CIDEr-D for CST) as the
#   reference-semantics comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/modes
o=gpurun_out/modes
timeout -k 10 240 python bench.py --mode xe --steps 40 --warmup 5 --json_out $o/xe_hip.json > $o/xe_hip.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --mode cst --steps 40 --warmup 5 --json_out $o/cst_hip.json > $o/cst_hip.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --mode xe --impl torch --precision fp32 --steps 10 --warmup 3 --json_out $o/xe_torch.json > $o/xe_torch.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --mode cst --impl torch --precision fp32 --reward cpu --steps 5 --warmup 2 --json_out $o/cst_torch_cpu.json > $o/cst_torch_cpu.log 2>&1 || exit $?
