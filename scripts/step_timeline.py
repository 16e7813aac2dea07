"""Per-stream timeline of one optimizer step from a rocprofv3 kernel trace.

usage: python scripts/step_timeline.py <kernel_trace.csv> [step_from_end]
Consecutive launches of the same kernel on the same stream are merged into
one line: start offset (us from the step start), span, count, summed busy
time, hardware queue id.  The step spans from the end of one adam_update kernel to
the end of the next.
"""
import csv
import sys

path = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:60],
             r['Queue_Id']) for r in rows)  # (graph replays: streams show as hardware queues)
adam = [e for e in ev if 'adam_update' in e[2]]
lo, hi = adam[-1 - k][1], adam[-k][1]
ev = [e for e in ev if e[0] >= lo and e[1] <= hi]
print('step wall %.1f us, %d kernels' % ((hi - lo) / 1e3, len(ev)))
groups = []
for s, e, name, st in ev:
    g = groups[-1] if groups else None
    if g and g['name'] == name and g['st'] == st:
        g['end'] = e
        g['n'] += 1
        g['busy'] += e - s
    else:
        groups.append(dict(name=name, st=st, start=s, end=e, n=1, busy=e - s))
for g in groups:
    print('%8.1f %8.1f %4d %8.1f  s%-3s %s' % ((g['start'] - lo) / 1e3, (g['end'] - g['start']) / 1e3,
                                            g['n'], g['busy'] / 1e3, g['st'], g['name']))
