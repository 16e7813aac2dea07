#!/bin/bash
# PMC counters of the eager step: headline config, then the 8-frame attention
# config, each in its own directory
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
BENCH_ARGS="--att8 0" bash scripts/gpu_pmc.sh || exit $?
rm -rf gpurun_out/pmc_headline && mv gpurun_out/pmc gpurun_out/pmc_headline || exit $?
BENCH_ARGS="--num_chunks 8" bash scripts/gpu_pmc.sh || exit $?
rm -rf gpurun_out/pmc_att8 && mv gpurun_out/pmc gpurun_out/pmc_att8 || exit $?
