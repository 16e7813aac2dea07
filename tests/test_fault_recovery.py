"""Failure detection / recovery: a rank of a 2-process DP
job is killed mid-epoch (``CSTCAP_FAULT_INJECT``, an abrupt ``os._exit``), the
job fails, and relaunching the same command resumes from the ``_last.pth``
sidecar (optimizer, per-rank loader and RNG state) instead of from scratch,
then runs to completion.  CPU ranks, gloo backend.

(torchrun's in-place ``--max-restarts`` is not used: with a static
rendezvous the restarted gloo mesh can read a dead peer's address from the
surviving store; a relaunch is the recovery path this framework documents.)"""
import os
import socket
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_killed_rank_resumes_from_last_sidecar(tmp_path):
    mf = str(tmp_path / 'm' / 'model.pth')
    marker = str(tmp_path / 'fault_fired')
    env = dict(os.environ)
    env.update(PYTHONPATH=ROOT + os.pathsep + env.get('PYTHONPATH', ''), CUDA_VISIBLE_DEVICES='',
               OMP_NUM_THREADS='1', CSTCAP_FAULT_INJECT='1:7:' + marker)
    # 24 videos / (4 per rank x 2 ranks) = 3 iterations per epoch; the sidecar
    # is written at iter 6 (epoch 2), rank 1 dies at iter 7.
    args = ['--synthetic', 'msvd', '--synthetic_videos', '24', '--synthetic_vocab', '40',
            '--seq_length', '10', '--rnn_size', '32', '--input_encoding_size', '32',
            '--feat_dims', '16', '8', '--batch_size', '4', '--train_seq_per_img', '3',
            '--test_batch_size', '4', '--test_seq_per_img', '3', '--beam_size', '2',
            '--impl', 'torch', '--loglevel', 'INFO', '--max_epochs', '4',
            '--save_checkpoint_from', '100', '--model_file', mf, '--print_log_interval', '1']
    def launch():
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node',
               '2', '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
               os.path.join(ROOT, 'train.py')] + args
        r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
        return r.returncode, r.stdout + r.stderr

    rc1, log1 = launch()
    assert rc1 != 0, 'the injected fault should fail the first job'
    assert 'fault injection: rank 1 exits at iter 7' in log1
    rc, log = launch()  # relaunch: resumes from the sidecar
    assert rc == 0, log[-4000:]
    assert os.path.exists(marker), 'the fault never fired'
    assert 'Resumed exactly from' in log and '(iter 6)' in log, log[-4000:]
    last = torch.load(mf.replace('.pth', '_last.pth'), weights_only=False)
    assert last['infos']['iter'] == 12 and last['infos']['epoch'] == 4
    assert len(last['per_rank']) == 2
