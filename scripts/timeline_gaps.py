"""Idle-gap analysis of a rocprofv3 kernel trace over the last N optimizer steps.

usage: python scripts/timeline_gaps.py <kernel_trace.csv> [n_steps]
A step ends at an adam_update kernel; reports the wall span per step, the
GPU-busy union, and the largest idle gaps with the kernel that follows them.
"""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = list(csv.DictReader(open(path)))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:70],
             r['Stream_Id']) for r in rows)
adam = [e for e in ev if 'adam_update' in e[2]]
lo, hi = adam[-1 - n][1], adam[-1][1]
ev = [e for e in ev if e[0] >= lo and e[1] <= hi]
busy, gaps = 0, []
cs, ce = ev[0][0], ev[0][1]
prev = ev[0][2]
for s, e, name, st in ev[1:]:
    if s > ce:
        busy += ce - cs
        gaps.append((s - ce, prev, name))
        cs, ce = s, e
    else:
        ce = max(ce, e)
    prev = name
busy += ce - cs
print('steps %d: wall %.3f ms/step, GPU busy %.3f ms/step, idle %.3f ms/step' %
      (n, (hi - lo) / n / 1e6, busy / n / 1e6, (hi - lo - busy) / n / 1e6))
gaps.sort(reverse=True)
for g, a, b in gaps[:25]:
    print('%8.1f us  after %-45s before %s' % (g / 1e3, a[:45], b[:60]))
