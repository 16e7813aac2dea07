#!/bin/bash
# rr microbenchmark + PMC, then the chunk A/B
bash scripts/gpu_rr.sh || exit $?
bash scripts/gpu_ab_chunks.sh || exit $?
