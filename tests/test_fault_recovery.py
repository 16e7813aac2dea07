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

from cst_captioning_amd.train.checkpoint import load_checkpoint

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
    last = load_checkpoint(mf.replace('.pth', '_last.pth'))
    assert last['infos']['iter'] == 12 and last['infos']['epoch'] == 4
    assert len(last['per_rank']) == 2


def test_resume_after_validated_epoch_matches_uninterrupted(tmp_path):
    """A single-process RL run (MIXER annealing from the resolved RL start
    epoch) is killed after a validated epoch and relaunched.  The resumed run
    keeps the validated best score / epoch, the history of earlier epochs and
    the schedule origin, and ends bit-identical to an uninterrupted run."""
    args = ['--synthetic', 'msvd', '--synthetic_videos', '24', '--synthetic_vocab', '40',
            '--seq_length', '10', '--rnn_size', '32', '--input_encoding_size', '32',
            '--feat_dims', '16', '8', '--batch_size', '4', '--train_seq_per_img', '3',
            '--test_batch_size', '4', '--test_seq_per_img', '3', '--beam_size', '2',
            '--impl', 'torch', '--loglevel', 'INFO', '--max_epochs', '3',
            '--save_checkpoint_from', '1', '--language_eval', '0', '--eval_metric', 'Loss',
            '--use_rl', '1', '--use_rl_after', '0', '--use_mixer', '1', '--mixer_from', '-1',
            '--mixer_descrease_every', '1', '--use_eos', '1', '--print_log_interval', '1']

    def launch(mf, fault=None):
        env = dict(os.environ)
        env.update(PYTHONPATH=ROOT + os.pathsep + env.get('PYTHONPATH', ''),
                   CUDA_VISIBLE_DEVICES='', OMP_NUM_THREADS='1')
        env.pop('CSTCAP_FAULT_INJECT', None)
        if fault:
            env['CSTCAP_FAULT_INJECT'] = fault
        r = subprocess.run([sys.executable, os.path.join(ROOT, 'train.py')] + args +
                           ['--model_file', mf], env=env, cwd=ROOT, capture_output=True,
                           text=True, timeout=600)
        return r.returncode, r.stdout + r.stderr

    ref_mf = str(tmp_path / 'ref' / 'model.pth')
    rc, log = launch(ref_mf)
    assert rc == 0, log[-4000:]
    mf = str(tmp_path / 'run' / 'model.pth')
    marker = str(tmp_path / 'fired')
    # 24 videos / 4 = 6 iterations per epoch: epoch 1 is validated at iter 6,
    # the process dies at iter 8
    rc1, log1 = launch(mf, '0:8:' + marker)
    assert rc1 != 0 and 'fault injection: rank 0 exits at iter 8' in log1
    rc2, log2 = launch(mf)
    assert rc2 == 0, log2[-4000:]
    assert 'Resumed exactly from' in log2 and '(iter 6)' in log2, log2[-4000:]
    ref = load_checkpoint(ref_mf.replace('.pth', '_last.pth'))
    got = load_checkpoint(mf.replace('.pth', '_last.pth'))
    for k in ('best_score', 'best_epoch', 'best_iter', 'iter', 'epoch', 'mixer_from'):
        assert got['infos'][k] == ref['infos'][k], k
    assert sorted(got['extra']['history']) == sorted(ref['extra']['history'])
    assert got['extra']['use_rl_after'] == ref['extra']['use_rl_after'] == 0
    for k in ref['model']:
        torch.testing.assert_close(got['model'][k], ref['model'][k], rtol=0, atol=0)
    # the history file on disk keeps the epochs validated before the crash
    import json
    with open(mf.replace('.pth', '_history.json')) as f:
        assert len(json.load(f)) == len(ref['extra']['history'])
