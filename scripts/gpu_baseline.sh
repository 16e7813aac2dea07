#!/bin/bash
# First GPU run: reference-semantics baseline (PyTorch ops, fp32, CPU CIDEr-D)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export CSTCAP_ALLOW_TORCH_FALLBACK=1
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python bench.py --impl torch --reward cpu --precision fp32 --dedupe_greedy 0 \
   --steps 5 --warmup 2 --json_out gpurun_out/ref_baseline.json > gpurun_out/ref_baseline.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ref -o ref -- \
   python bench.py --impl torch --reward cpu --precision fp32 --dedupe_greedy 0 --steps 2 --warmup 1 \
   > gpurun_out/prof_ref.log 2>&1
echo "exit $?"
