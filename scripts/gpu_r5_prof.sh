#!/bin/bash
# Clean per-step rocprofv3 tables of the shipped headline step, the att8 step
# and the beam-5 decode, plus back-to-back device stamps of the headline step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-prof}
mkdir -p gpurun_out
prof() {  # name, delimiter, steps, bench args...
  local name=$1 delim=$2 n=$3; shift 3
  rm -rf gpurun_out/prof_${TAG}_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$name \
    -o $name -- python bench.py "$@" > gpurun_out/prof_${TAG}_$name.log 2>&1 || return $?
  python scripts/prof_steps.py gpurun_out/prof_${TAG}_$name/${name}_kernel_trace.csv $n 40 $delim \
    > gpurun_out/steps_${TAG}_$name.txt && head -n 16 gpurun_out/steps_${TAG}_$name.txt
  rm -f gpurun_out/prof_${TAG}_$name/${name}_kernel_trace.csv
}
prof head adam_update_kernel 10 --steps 10 --warmup 5 --att8 0 --beam5 0 --cst 0 || exit $?
prof att8 adam_update_kernel 10 --steps 10 --warmup 5 --num_chunks 8 --att8 0 --beam5 0 --cst 0 || exit $?
prof beam beam_fused_step_kernel 27 --mode beam --steps 4 --warmup 3 --att8 0 --beam5 0 --cst 0 || exit $?
timeout -k 10 300 python bench.py --stamps 4 --att8 0 --beam5 0 --cst 0 > gpurun_out/stamps_$TAG.json 2> gpurun_out/stamps_$TAG.err || exit $?
grep -A60 "stamps (us" gpurun_out/stamps_$TAG.err | head -60
