#!/bin/bash
# Decode-launch diagnostics + interleaved headline A/B of the decode tiles
# (CSTCAP_DECODE_TILES small / big), then a clean per-step rocprof table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-dec}
mkdir -p gpurun_out
timeout -k 10 300 python scripts/microbench_decode.py > gpurun_out/mbdec_$TAG.json 2> gpurun_out/mbdec_$TAG.err || exit $?
cat gpurun_out/mbdec_$TAG.json
for rep in 1 2; do
  for t in small big; do
    CSTCAP_DECODE_TILES=$t timeout -k 10 300 python bench.py --att8 0 --beam5 0 --cst 0 > gpurun_out/ab_${TAG}_${t}_$rep.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" gpurun_out/ab_${TAG}_${t}_$rep.json $t
  done
done
if [ -z "$SKIP_PROF" ]; then
  rm -rf gpurun_out/prof_$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG \
    -o $TAG -- python bench.py --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 \
    > gpurun_out/prof_$TAG.log 2>&1 || exit $?
  python scripts/prof_steps.py gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv 10 40 \
    > gpurun_out/steps_$TAG.txt && head -n 30 gpurun_out/steps_$TAG.txt
  rm -f gpurun_out/prof_$TAG/*_kernel_trace.csv
fi
