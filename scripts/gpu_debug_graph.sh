#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
mkdir -p gpurun_out/dbg
run() { timeout -k 5 120 python scripts/debug_graph_capture.py "$@" > gpurun_out/dbg/$(echo "$@" | tr ' ,' '__').log 2>&1; echo "$* -> $?"; }
run 64 40 3 4 10 1 16,8
run 64 40 3 4 10 0 16,8
run 128 40 3 4 10 0 16,8
run 64 500 3 4 10 0 16,8
run 64 40 5 8 10 0 16,8
run 128 500 5 8 12 0 64,32
run 64 40 3 4 10 0 64,32
exit 0
