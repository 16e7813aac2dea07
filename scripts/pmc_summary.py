import csv, collections, sys
for p in ['p1', 'p2', 'p3']:
    try:
        rows = list(csv.DictReader(open(f'gpurun_out/pmc/{p}/{p}_counter_collection.csv')))
    except FileNotFoundError:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.defaultdict(set)
    for r in rows:
        k = (r['Kernel_Name'][:34], r.get('Grid_Size', ''))
        agg[k][r['Counter_Name']] += float(r['Counter_Value']); cnt[k].add(r['Dispatch_Id'])
    for k, v in agg.items():
        if 'cst::' not in k[0]:
            continue
        n = len(cnt[k])
        w = v.get('SQ_WAVES', 0) / n if 'SQ_WAVES' in v else None
        print(p, k, n, {c: round(x / n) for c, x in v.items()})
