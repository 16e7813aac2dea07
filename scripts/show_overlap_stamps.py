"""Run tests/gpu_overlap_worker.py once and print each replayed step's device
stamps in time order (diagnosing the DP slice positions)."""
import os
import socket
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, 'gpurun_out', 'ov.pt')
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=ROOT)
    subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'gpu_overlap_worker.py'), out,
                    str(port)], env=env, cwd=ROOT, check=True)
    r = torch.load(out, weights_only=False)
    print('events_ok', r['events_ok'], 'n_groups', r['n_groups'])
    for st in r['stamps']:
        print(' '.join('%s=%.1f' % kv for kv in sorted(st.items(), key=lambda kv: kv[1])))


if __name__ == '__main__':
    main()
