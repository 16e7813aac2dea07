"""Per-kernel PMC summary of scripts/gpu_pmc.sh: per training step (the
bench's last `steps` steps), HBM bytes read / written (FETCH_SIZE /
WRITE_SIZE, KB per dispatch in rocprofv3), MFMA busy time
(SQ_VALU_MFMA_BUSY_CYCLES summed over the 1,024 SIMDs -> per-SIMD busy
microseconds at 2.1 GHz; divide by the kernel's traced duration for the
utilisation), L2 hit rate.

usage: python scripts/pmc_summary.py <pmc dir> <steps counted>"""
import collections
import csv
import os
import sys

root = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for p in ('p1', 'p2', 'p3', 'p4'):
    path = os.path.join(root, p, p + '_counter_collection.csv')
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        name = r['Kernel_Name']
        short = name.split('(')[0].replace('void ', '')[:48]
        agg[short][r['Counter_Name']] += float(r['Counter_Value'])
        cnt[short].add((p, r['Dispatch_Id']))
tot_r = tot_w = 0.0
rows = []
for k, v in agg.items():
    rd = v.get('FETCH_SIZE', 0.0) / 1024 / steps  # MB per step
    wr = v.get('WRITE_SIZE', 0.0) / 1024 / steps
    tot_r += rd
    tot_w += wr
    mfma_us = v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) / 1024 / 2100.0 / steps
    hit, miss = v.get('TCC_HIT_sum', 0.0), v.get('TCC_MISS_sum', 0.0)
    rows.append((rd + wr, k, rd, wr, mfma_us, hit / (hit + miss) if hit + miss else 0.0))
rows.sort(reverse=True)
print('HBM traffic per training step: read %.1f MB, write %.1f MB, total %.1f MB'
      % (tot_r, tot_w, tot_r + tot_w))
print('%-50s %9s %9s %11s %7s' % ('kernel', 'read MB', 'write MB', 'MFMA us/st', 'L2hit%'))
for _, k, rd, wr, mf, hr in rows[:40]:
    print('%-50s %9.1f %9.1f %11.1f %7.1f' % (k, rd, wr, mf, 100 * hr))
