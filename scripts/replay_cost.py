"""Host submission cost of one captured-step replay vs its GPU time: if
hipGraphLaunch took as long as the GPU work, the step would be host-bound."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench  # noqa: E402

sys.argv = ['bench.py', '--steps', '3', '--warmup', '3']
state = {}
_orig = torch.cuda.CUDAGraph.replay


def timed_replay(self):
    t0 = time.perf_counter()
    _orig(self)
    state.setdefault('host', []).append(time.perf_counter() - t0)


torch.cuda.CUDAGraph.replay = timed_replay
bench.main()
h = state.get('host', [])
print('replays %d, host submit per replay: median %.3f ms, max %.3f ms'
      % (len(h), sorted(h)[len(h) // 2] * 1e3, max(h) * 1e3))
