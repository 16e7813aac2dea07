#!/bin/bash
# round 4: learning parity on the learnable template task at the headline
# shape -- XE then SCST, fused engine vs the PyTorch decoder (bf16 autocast),
# same init and data order; validation greedy CIDEr-D per log point
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
export CSTCAP_PARITY_TASK=template CSTCAP_PARITY_SHAPE=headline
timeout -k 10 500 python -u scripts/scst_parity.py hip bf16 300 300 > gpurun_out/learn_template_hip.jsonl 2> gpurun_out/learn_template_hip.err || exit $?
timeout -k 10 700 python -u scripts/scst_parity.py torch bf16 300 300 > gpurun_out/learn_template_torch_bf16.jsonl 2> gpurun_out/learn_template_torch_bf16.err || exit $?
tail -n 3 gpurun_out/learn_template_hip.jsonl gpurun_out/learn_template_torch_bf16.jsonl
