"""Per-kernel PMC summary of scripts/gpu_pmc.sh: per training step, HBM bytes
read / written (FETCH_SIZE / WRITE_SIZE, KB per dispatch in rocprofv3), MFMA
busy time (SQ_VALU_MFMA_BUSY_CYCLES summed over the 1,024 SIMDs -> per-SIMD
busy microseconds at 2.1 GHz; divide by the kernel's traced duration for the
utilisation), L2 hit rate.

Only the last `steps` steps of each pass are counted: the dispatches after
the (steps+1)-th last `delimiter` dispatch up to the last one (default
delimiter adam_update_kernel, the step's final kernel), so one-time work
(hipBLASLt plan search, capture, warmup) is excluded.

usage: python scripts/pmc_summary.py <pmc dir> <steps> [delimiter]"""
import collections
import csv
import os
import sys

root = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
delim = sys.argv[3] if len(sys.argv) > 3 else 'adam_update_kernel'
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for p in ('p1', 'p2', 'p3', 'p4'):
    path = os.path.join(root, p, p + '_counter_collection.csv')
    if not os.path.exists(path):
        continue
    rows = list(csv.DictReader(open(path)))
    names = {}
    for r in rows:
        names[int(r['Dispatch_Id'])] = r['Kernel_Name']
    ids = sorted(names)
    marks = [i for i in ids if delim in names[i]]
    if len(marks) < steps + 1:
        print('# %s: only %d delimiter dispatches, counting everything' % (p, len(marks)))
        lo, hi = -1, ids[-1]
    else:
        lo, hi = marks[-steps - 1], marks[-1]
    for r in rows:
        d = int(r['Dispatch_Id'])
        if lo < d <= hi:
            short = (r['Kernel_Name'].replace('(anonymous namespace)::', '')
                     .split('(')[0].replace('void ', '')[:48])
            agg[short][r['Counter_Name']] += float(r['Counter_Value'])
tot_r = tot_w = tot_m = 0.0
out = []
for k, v in agg.items():
    rd = v.get('FETCH_SIZE', 0.0) / 1024 / steps  # MB per step
    wr = v.get('WRITE_SIZE', 0.0) / 1024 / steps
    tot_r += rd
    tot_w += wr
    mfma_us = v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) / 1024 / 2100.0 / steps
    tot_m += mfma_us
    hit, miss = v.get('TCC_HIT_sum', 0.0), v.get('TCC_MISS_sum', 0.0)
    out.append((rd + wr, k, rd, wr, mfma_us, hit / (hit + miss) if hit + miss else 0.0))
out.sort(reverse=True)
print('window: last %d steps (delimiter %s)' % (steps, delim))
print('HBM traffic per training step: read %.1f MB, write %.1f MB, total %.1f MB; '
      'MFMA busy %.1f us per SIMD' % (tot_r, tot_w, tot_r + tot_w, tot_m))
print('%-50s %9s %9s %11s %7s' % ('kernel', 'read MB', 'write MB', 'MFMA us/st', 'L2hit%'))
for _, k, rd, wr, mf, hr in out[:40]:
    print('%-50s %9.1f %9.1f %11.1f %7.1f' % (k, rd, wr, mf, 100 * hr))
