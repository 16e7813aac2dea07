#!/bin/bash
# round 4: several independent GPU checks in one call; a failing part is
# reported and the next part runs, but a timeout / abort / segfault ends it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rc=0
part() {  # name, command...
  local name=$1; shift
  "$@"
  local e=$?
  echo "== $name: exit $e"
  if [ $e -ne 0 ]; then rc=$e; fi
  case $e in 124|134|137|139) echo "== stopping after $name"; exit $e;; esac
  return 0
}
part beam_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_cells.py -x -q -k beam --timeout 120 --timeout-method thread -p no:cacheprovider
part beam_prof bash scripts/gpu_r4_prof_beam.sh
part att_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_attention_headline.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
part blaslt timeout -k 10 300 python -u scripts/blaslt_probe.py
part bench timeout -k 10 400 python bench.py --json_out gpurun_out/r4_combo_default.json
part learn bash scripts/gpu_r4_learn.sh
exit $rc
