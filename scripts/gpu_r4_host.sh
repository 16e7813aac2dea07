#!/bin/bash
# round 4: is the back-to-back headline step host-bound?  host enqueue time of
# one step (sync_debug) and a cProfile of the timed loop
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --att8 0 --beam5 0 --sync_debug 1 \
  --json_out gpurun_out/host_sd.json > gpurun_out/host_sd.log 2>&1 || exit $?
grep -h "host enqueue" gpurun_out/host_sd.log
timeout -k 10 300 python -m cProfile -o gpurun_out/host.prof bench.py --steps 200 --warmup 5 \
  --att8 0 --beam5 0 --json_out gpurun_out/host_prof.json > gpurun_out/host_prof.log 2>&1 || exit $?
python - <<'PY'
import pstats
p = pstats.Stats('gpurun_out/host.prof')
p.sort_stats('tottime').print_stats(25)
PY
