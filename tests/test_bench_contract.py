"""bench.py output contract (the driver runs it under torch.distributed.run
with N ranks): ONE JSON line from rank 0 with the whole-job value, n_gpus,
steps / warmup, the config and the timing fields.  Exercised on the CPU with
the gloo backend and the PyTorch decoder path at tiny sizes."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('world,launcher', [(1, False), (2, True), (2, False)])
def test_bench_json_line(world, launcher):
    """launcher=False with world 2 is the driver's ``python bench.py --gpus 2``
    shape: bench.py starts the ranks itself."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', OMP_NUM_THREADS='1')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    args = ['bench.py', '--gpus', str(world), '--impl', 'torch', '--steps', '2', '--warmup', '1',
            '--videos', '48', '--vocab', '300', '--batch_size', '4']
    if launcher:
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node',
               str(world), '--master-addr', '127.0.0.1', '--master-port', str(_port())] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step',
              'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'data', 'config'):
        assert k in rec, k
    assert rec['n_gpus'] == world and rec['steps'] == 2 and rec['warmup'] == 1
    assert rec['scaling'] == 'weak' and rec['higher_is_better'] is True
    assert rec['dtype'] == 'fp32'  # the PyTorch path computes in fp32
    assert rec['config']['global_batch'] == 4 * 20 * world
    assert rec['config']['parallelism'] == 'dp%d' % world
    assert rec['world_size_seen'] == world
    assert rec['backend'] == ('gloo' if world > 1 else 'none')
    # whole-job value = global captions / step time
    assert abs(rec['value'] - 4 * 20 * world / (rec['ms_per_step'] / 1e3)) < 0.02 * rec['value']
    # the 8-frame temporal-attention config, timed in the same invocation
    att = rec['att8']
    assert att['temporal_attention_frames'] == 8 and att['value'] > 0
    assert abs(att['value'] - 4 * 20 * world / (att['ms_per_step'] / 1e3)) < 0.02 * att['value']
    # the CST recipe (CST_MS_SCB: GT consensus baseline), same invocation
    cst = rec['cst']
    assert cst['recipe'] == 'CST_MS_SCB' and cst['scb_baseline'] == 1 and cst['value'] > 0
    assert cst['bcmr'].startswith('prepro/evalscores.py')
    assert abs(cst['value'] - 4 * 20 * world / (cst['ms_per_step'] / 1e3)) < 0.02 * cst['value']
    assert 'vs_pytorch_bf16_1gpu' not in rec


def test_bench_world_size_mismatch_fails():
    """A rank whose job size differs from --gpus exits non-zero."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', OMP_NUM_THREADS='1', WORLD_SIZE='1',
               RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, 'bench.py', '--gpus', '2', '--impl', 'torch', '--steps',
                        '1', '--warmup', '0', '--videos', '48', '--vocab', '300',
                        '--batch_size', '4'], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode != 0
    assert 'rank(s)' in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
