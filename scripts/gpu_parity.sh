#!/bin/bash
# sampler parity at fixed weights, then the SCST learning curves at the
# headline shape (engine and PyTorch bf16), logs under gpurun_out/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sampler_parity.py 200 20 > gpurun_out/sampler_parity.jsonl 2> gpurun_out/sampler_parity.err || exit $?
CSTCAP_PARITY_SHAPE=headline timeout -k 10 400 python -u scripts/sampler_parity.py 200 10 > gpurun_out/sampler_parity_headline.jsonl 2> gpurun_out/sampler_parity_headline.err || exit $?
CSTCAP_PARITY_SHAPE=headline timeout -k 10 500 python -u scripts/scst_parity.py hip bf16 200 300 > gpurun_out/scst_parity_headline_hip.jsonl 2> gpurun_out/scst_parity_headline_hip.err || exit $?
CSTCAP_PARITY_SHAPE=headline timeout -k 10 600 python -u scripts/scst_parity.py torch bf16 200 300 > gpurun_out/scst_parity_headline_torch_bf16.jsonl 2> gpurun_out/scst_parity_headline_torch_bf16.err || exit $?
