import csv, collections, sys
path = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_hip/hip_kernel_trace.csv'
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
rows = list(csv.DictReader(open(path)))
d = collections.defaultdict(list)
for r in rows:
    d[(r['Kernel_Name'][:50], r['Grid_Size_X'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = sum(sum(v) for v in d.values())
print('kernel time per step: %.3f ms' % (tot / steps / 1e3))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print('%-52s %8s n=%4d avg %8.1f us  per-step %7.3f ms' % (k[0], k[1], len(v), sum(v) / len(v), sum(v) / steps / 1e3))
