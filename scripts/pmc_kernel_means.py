"""Mean PMC counter value per dispatch, per kernel, over rocprofv3 --pmc
passes (usage: python scripts/pmc_kernel_means.py <dir> <pass> ...)."""
import collections
import csv
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sys.argv[2:]:
    path = os.path.join(root, p, p + '_counter_collection.csv')
    if not os.path.exists(path):
        print('missing', path)
        continue
    for r in csv.DictReader(open(path)):
        short = r['Kernel_Name'].split('(')[0].replace('void ', '')[:40]
        agg[short][r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    print(k)
    for c, xs in sorted(v.items()):
        print('   %-28s %14.1f' % (c, sum(xs) / len(xs)))
