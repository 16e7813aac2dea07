"""Node-type census of the captured training-step graph (HIP graph debug
dump): kernels, memcpy / memset nodes, event edges."""
import collections
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

_orig = torch.cuda.CUDAGraph
graphs = []


class DebugGraph(_orig):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.enable_debug_mode()
        graphs.append(self)


torch.cuda.CUDAGraph = DebugGraph
sys.argv = ['bench.py', '--steps', '2', '--warmup', '3']
import bench  # noqa: E402
try:
    bench.main()
except SystemExit:
    pass
os.makedirs('gpurun_out', exist_ok=True)
for i, g in enumerate(graphs):
    path = 'gpurun_out/graph_%d.dot' % i
    g.debug_dump(path)
    txt = open(path).read()
    kinds = collections.Counter(re.findall(r'(KERNEL|MEMCPY|MEMSET|EVENT_RECORD|WAIT_EVENT|EMPTY|HOST|GRAPH)', txt))
    print('graph', i, dict(kinds), 'bytes', len(txt))
    for m in re.findall(r'MEMCPY[^\n]{0,200}', txt)[:20]:
        print('  ', m[:200])
