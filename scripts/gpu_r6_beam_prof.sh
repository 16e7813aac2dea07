#!/bin/bash
# round 6: beam-5 kernel table (SCST part minimal)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_beam
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_beam -o beam -- python bench.py --steps 2 --warmup 1 --att8 0 --cst 0 --xe 0 > gpurun_out/prof_beam.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_beam.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['beam5'])"
python - <<'PY' > gpurun_out/beam_kernels.txt
import csv
rows = list(csv.DictReader(open('gpurun_out/prof_beam/beam_kernel_trace.csv')))
# the last beam batch: kernels after the last 'beam' kernel-name start minus a window
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'beam' in r['Kernel_Name'].lower()]
last = idx[-1]
# walk back to the previous gap > 200 us
i = last
while i > 0 and int(rows[i]['Start_Timestamp']) - int(rows[i-1]['End_Timestamp']) < 200000:
    i -= 1
t0 = int(rows[i]['Start_Timestamp'])
from collections import defaultdict
agg = defaultdict(lambda: [0, 0.0])
for r in rows[i:last + 1]:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
    k = r['Kernel_Name'][:90]
    agg[k][0] += 1; agg[k][1] += d
print('window %.1f us, %d launches' % ((int(rows[last]['End_Timestamp']) - t0) / 1000, last + 1 - i))
for k, (n, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:20]:
    print('%5d %9.1f %7.2f  %s' % (n, d, d / n, k))
for r in rows[last - 8:last + 1]:
    print('%9.1f %7.1f  %s' % ((int(r['Start_Timestamp']) - t0) / 1000, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000, r['Kernel_Name'][:80]))
PY
cat gpurun_out/beam_kernels.txt
rm -f gpurun_out/prof_beam/beam_kernel_trace.csv
