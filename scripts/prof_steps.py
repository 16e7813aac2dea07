"""Per-step kernel table of the LAST N training steps of a rocprofv3 kernel
trace (csv), so one-time work (hipBLASLt algorithm search, capture, warm-up
steps, the att8 / beam runs) stays out of the figures.

Steps are delimited by the one kernel every step launches exactly once at its
end (``cst::adam_update_kernel``): the window is (end of the (N+1)-th last
delimiter, end of the last delimiter].  Run the bench with ``--att8 0
--beam5 0`` so nothing follows the timed steps.

usage: prof_steps.py TRACE.csv N [ROWS] [DELIM] [SEQ]

SEQ: '|'-separated kernel-name substrings; the last step's launches of those
kernels are listed in order (start offset from the step start, duration, gap
to the previous listed launch's end).
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2])
    rows_out = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    delim = sys.argv[4] if len(sys.argv) > 4 else 'adam_update_kernel'
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r['s'] = int(r['Start_Timestamp'])
        r['e'] = int(r['End_Timestamp'])
    rows.sort(key=lambda r: r['s'])
    ends = [r['e'] for r in rows if delim in r['Kernel_Name']]
    if len(ends) < n + 1:
        sys.exit('only %d delimiter kernels (%s) in the trace' % (len(ends), delim))
    lo, hi = ends[-n - 1], ends[-1]
    win = [r for r in rows if lo < r['s'] <= hi]
    d = collections.defaultdict(list)
    for r in win:
        d[(r['Kernel_Name'][:60], r['Grid_Size_X'])].append((r['e'] - r['s']) / 1e3)
    busy = sum(sum(v) for v in d.values())
    print('window: last %d steps, %.3f ms per step wall (delimiter %s), %.3f ms of kernel '
          'time per step, %d launches per step' % (n, (hi - lo) / 1e6 / n, delim, busy / n / 1e3,
                                                  len(win) // n))
    print('%-62s %8s %6s %9s %10s' % ('kernel', 'grid_x', 'n/step', 'avg us', 'us/step'))
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:rows_out]:
        print('%-62s %8s %6.1f %9.1f %10.1f' % (k[0], k[1], len(v) / n, sum(v) / len(v),
                                                 sum(v) / n))
    if len(sys.argv) > 5:
        pats = sys.argv[5].split('|')
        step = [r for r in win if ends[-2] < r['s'] <= hi]
        t0, prev = step[0]['s'], None
        print('last step, launches matching %s:' % sys.argv[5])
        print('%10s %9s %9s  %s' % ('start us', 'dur us', 'gap us', 'kernel'))
        for r in step:
            if any(p in r['Kernel_Name'] for p in pats):
                gap = (r['s'] - prev) / 1e3 if prev is not None else 0.0
                print('%10.1f %9.1f %9.1f  %s' % ((r['s'] - t0) / 1e3, (r['e'] - r['s']) / 1e3, gap,
                                                  r['Kernel_Name'][:70]))
                prev = r['e']


if __name__ == '__main__':
    main()
