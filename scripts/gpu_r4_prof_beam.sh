#!/bin/bash
# round 4: kernel trace of the beam-5 evaluation decode (bench.py --mode beam)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_beam
CSTCAP_BEAM_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_beam -o beam -- python bench.py --mode beam --steps 5 --warmup 2 --att8 0 > gpurun_out/prof_beam.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/prof_beam/beam_kernel_trace.csv 7 20 > gpurun_out/prof_beam_summary.txt
rm -rf gpurun_out/prof_beam
cat gpurun_out/prof_beam_summary.txt
