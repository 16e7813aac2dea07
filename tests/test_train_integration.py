"""End-to-end training on CPU with tiny synthetic MSVD-shaped data
(SURVEY.md §4.2 "Integration"): XE loss decreases, every README recipe
(XE, WXE, SCST, CST-SCB, CST-SCB*) runs through the trainer, the CLI writes
the reference artefacts (checkpoint, history, test json), and the
``_last.pth`` sidecar resumes bit-exactly (``/root/reference/train.py``
flow, ``:45-274``)."""
import json
import os

import numpy as np
import pytest
import torch

from cst_captioning_amd.cli import build_model, load_splits, train_main
from cst_captioning_amd.cli import test_main as run_test_cli
from cst_captioning_amd.config import parse_opts
from cst_captioning_amd.data import CaptionLoader
from cst_captioning_amd.parallel import DistContext
from cst_captioning_amd.train import checkpoint as ckpt
from cst_captioning_amd.train.trainer import Trainer

BASE = ['--synthetic', 'msvd', '--synthetic_videos', '24', '--synthetic_vocab', '40',
        '--seq_length', '10', '--rnn_size', '32', '--input_encoding_size', '32',
        '--feat_dims', '16', '8', '--batch_size', '6', '--train_seq_per_img', '4',
        '--test_batch_size', '8', '--test_seq_per_img', '4', '--beam_size', '2',
        '--impl', 'torch', '--loglevel', 'WARNING', '--print_log_interval', '1',
        '--learning_rate', '2e-3', '--drop_prob_lm', '0.1']


def _setup(extra, seed=0):
    opt = parse_opts(BASE + list(extra))
    torch.manual_seed(seed)
    np.random.seed(seed)
    tr, va, te = load_splits(opt)
    ctx = DistContext(device=torch.device('cpu'))
    loader = CaptionLoader(tr, opt.batch_size, opt.train_seq_per_img, 'train', 'cpu',
                           seed=opt.seed)
    opt.vocab = loader.get_vocab()
    opt.vocab_size = loader.get_vocab_size()
    opt.seq_length = loader.get_seq_length()
    opt.feat_dims = loader.get_feat_dims()
    model, engine = build_model(opt, torch.device('cpu'))
    val = CaptionLoader(va, opt.test_batch_size, opt.test_seq_per_img, 'test', 'cpu')
    return opt, Trainer(opt, model, loader, val, ctx, engine), te


def test_xe_loss_decreases():
    opt, tr, _ = _setup(['--max_epochs', '100'])
    data = tr.train_loader.get_batch()
    losses = [float(tr.train_step(data, 0)["loss"]) for _ in range(60)]
    assert losses[-1] < 0.75 * losses[0]


@pytest.mark.parametrize('recipe', [
    ['--use_rl', '1', '--use_rl_after', '0', '--use_cst', '0', '--use_mixer', '1',
     '--mixer_from', '1', '--use_eos', '1'],                                   # SCST
    ['--use_rl', '1', '--use_rl_after', '0', '--use_cst', '1', '--use_mixer', '0',
     '--scb_captions', '0'],                                                   # WXE
    ['--use_rl', '1', '--use_rl_after', '0', '--use_cst', '1', '--use_mixer', '1',
     '--mixer_from', '1', '--scb_baseline', '1', '--scb_captions', '4',
     '--use_eos', '1'],                                                        # CST_MS_SCB
    ['--use_rl', '1', '--use_rl_after', '0', '--use_cst', '1', '--use_mixer', '1',
     '--mixer_from', '1', '--scb_baseline', '2', '--scb_captions', '4',
     '--use_eos', '1'],                                                        # SCB(*)
    ['--use_ss', '1', '--use_ss_after', '0', '--ss_max_prob', '0.5'],           # XE + SS
])
def test_recipes_step(recipe):
    opt, tr, _ = _setup(recipe)
    tr.rl_training = False
    for it in range(3):
        out = tr.train_step(tr.train_loader.get_batch(), 0)
        assert np.isfinite(float(out['loss']))
    if opt.use_rl:
        assert tr.rl_training and 'reward' in out
        assert out['reward'].shape == (opt.batch_size * opt.train_seq_per_img,)


def test_cli_train_then_test(tmp_path):
    mf = str(tmp_path / 'model' / 'xe.pth')
    rf = str(tmp_path / 'xe_test.json')
    infos = train_main(BASE + ['--max_epochs', '2', '--save_checkpoint_from', '1',
                               '--model_file', mf, '--result_file', rf,
                               '--eval_metric', 'CIDEr'])
    assert os.path.exists(mf) and os.path.exists(mf.replace('.pth', '_history.json'))
    assert os.path.exists(ckpt.last_path(mf))
    res = json.load(open(rf))
    assert len(res['predictions']) == 8  # synthetic test split: max(8, 24 // 10) videos
    assert {'Bleu_4', 'CIDEr', 'ROUGE_L', 'METEOR', 'Loss'} <= set(res['scores'])
    assert infos['best_epoch'] >= 1
    s = ckpt.load_checkpoint(mf)
    assert set(s) == {'model', 'infos', 'opt'} and s['opt'].vocab_size == 40
    # test CLI reads architecture fields from the checkpoint's opt
    out = run_test_cli(BASE + ['--model_file', mf, '--result_file', str(tmp_path / 't2.json')])
    assert out['scores']['CIDEr'] == pytest.approx(res['scores']['CIDEr'])


def _flat(model):
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


@pytest.mark.parametrize('rl', [False, True])
def test_exact_resume_from_last_sidecar(tmp_path, rl):
    extra = ['--use_rl', '1', '--use_rl_after', '0', '--mixer_from', '1', '--use_eos', '1'] \
        if rl else []
    # uninterrupted: 6 steps
    opt, a, _ = _setup(extra, seed=1)
    a.rl_training = rl
    for _ in range(6):
        a.train_step(a.train_loader.get_batch(), 0)
    ref = _flat(a.model)
    # interrupted after 3 steps: save the sidecar, rebuild everything, resume
    opt, b, _ = _setup(extra, seed=1)
    b.rl_training = rl
    for _ in range(3):
        b.train_step(b.train_loader.get_batch(), 0)
    path = str(tmp_path / 'm_last.pth')
    ckpt.save_last(path, b.model, b.optimizer, b.infos, opt, b.train_loader)
    opt2, c, _ = _setup(extra, seed=99)
    c.rl_training = rl
    s = ckpt.load_checkpoint(path)
    c.model.load_state_dict(s['model'])
    c.optimizer.load_state_dict(s['optimizer'])
    c.train_loader.load_state_dict(s['loader'])
    ckpt.restore_rng(s['rng'])
    for _ in range(3):
        c.train_step(c.train_loader.get_batch(), 0)
    torch.testing.assert_close(_flat(c.model), ref, rtol=0, atol=0)


def test_nan_guard_skips_step():
    opt, tr, _ = _setup([])
    before = _flat(tr.model).clone()
    data = tr.train_loader.get_batch()
    data['masks'] = data['masks'] * float('nan')
    tr.train_step(data, 0)
    torch.testing.assert_close(_flat(tr.model), before, rtol=0, atol=0)
