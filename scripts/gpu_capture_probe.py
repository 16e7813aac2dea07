"""Capture probe: a few SCST trainer steps (eager, capture, replay) of the
small test model with the engine's X-after-rollout on or off (argv[1]);
prints 'ok' or dies (the caller reads the exit status)."""
import faulthandler
import sys
import os

faulthandler.enable()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import torch  # noqa: E402
from test_gpu_graph import _setup  # noqa: E402

tr, loader = _setup(rl=True, drop=0.5, graph=1, H=int(sys.argv[2]) if len(sys.argv) > 2 else 128)
tr.use_x_after_rollout = sys.argv[1] == '1'
for i in range(4):
    out = tr.train_step(loader.get_batch(), 0)
    torch.cuda.synchronize()
    print('step', i, float(out['loss']), 'graph' if tr._graph is not None else 'eager', flush=True)
print('ok')
