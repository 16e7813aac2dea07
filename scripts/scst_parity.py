"""SCST learning parity: the same recipe through the fused HIP engine and
through the PyTorch decoder path (bf16 autocast or fp32), same data order,
same init.  XE warm-up, then SCST (MIXER from 1, greedy baseline, CIDEr-D
reward on the GPU).  Prints one JSON line per log point:
{impl, phase, step, loss, reward_mean, sample_cider (m), greedy_cider (b),
 val_greedy_cider}.

usage: python scripts/scst_parity.py IMPL [PRECISION] [XE_STEPS] [RL_STEPS]

CSTCAP_PARITY_TASK=template uses the learnable template captions
(data/synthetic.py).  CSTCAP_PARITY_SHAPE=headline runs the headline model (concat LSTM-512, 4
modalities, V = 10,509, 64 videos x 20 captions per step) instead of the
small default (H = 256, V = 2,000, 32 videos).  Every log line also carries
the optimizer's NaN-guard skip count and the exp-store rows recomputed.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cst_captioning_amd.cli import build_model  # noqa: E402
from cst_captioning_amd.config import default_opts  # noqa: E402
from cst_captioning_amd.data import CaptionLoader, make_splits  # noqa: E402
from cst_captioning_amd.parallel import DistContext  # noqa: E402
from cst_captioning_amd.train.trainer import Trainer  # noqa: E402

impl = sys.argv[1]
precision = sys.argv[2] if len(sys.argv) > 2 else 'bf16'
xe_steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
rl_steps = int(sys.argv[4]) if len(sys.argv) > 4 else 300
if impl == 'torch':
    os.environ['CSTCAP_ALLOW_TORCH_FALLBACK'] = '1'
dev = torch.device('cuda', 0)
torch.manual_seed(0)
HEADLINE = os.environ.get('CSTCAP_PARITY_SHAPE') == 'headline'
if HEADLINE:
    V_, FD_, NV_, B_, H_ = 10509, [2048, 4096, 1024, 300], 6513, 64, 512
else:
    V_, FD_, NV_, B_, H_ = 2000, [256, 128], 1280, 32, 256
# CSTCAP_PARITY_TASK=template: captions nearly a function of the features
# (data/synthetic.py caption_mode), so validation CIDEr-D rises above noise
TASK = os.environ.get('CSTCAP_PARITY_TASK', 'zipf')
tr, va, _ = make_splits('msrvtt', vocab_size=V_, feat_dims=FD_, train_videos=NV_, seed=0,
                        eval_videos=256 if HEADLINE else None, caption_mode=TASK)
opt = default_opts(batch_size=B_, train_seq_per_img=20, rnn_size=H_, input_encoding_size=H_,
                   learning_rate=2e-3, max_epochs=10 ** 9, print_log_interval=0, impl=impl,
                   precision=precision, loglevel='WARNING', use_rl=1, use_rl_after=10 ** 6,
                   use_cst=0, use_mixer=1, mixer_from=1, use_eos=1, drop_prob_lm=0.5)
opt.vocab = {i: w for i, w in enumerate(tr.vocab)}
opt.vocab_size, opt.seq_length, opt.feat_dims = tr.vocab_size, tr.seq_length, tr.feat_dims
loader = CaptionLoader(tr, B_, 20, 'train', dev, seed=0)
val = CaptionLoader(va, 64, 20, 'test', dev)
model, eng = build_model(opt, dev, impl)
t = Trainer(opt, model, loader, None, DistContext(device=dev), eng)


def val_cider():
    """greedy decode of the validation videos, CIDEr-D on the GPU."""
    sc = t._ensure_scorer()
    model.eval()
    tot, n = 0.0, 0
    with torch.no_grad():
        for ii in range((va.num_videos + 63) // 64):
            d = val.get_batch_at(ii)
            seq, _ = model.sample(d['feats'], {'sample_max': 1})
            vs = CiderLike(va, sc)
            tot += float(vs.score(seq, d['video_index']).sum())
            n += seq.size(0)
    model.train()
    return tot / n


class CiderLike:
    """the training scorer's kernel against the validation split's refs"""
    _cache = {}

    def __init__(self, ds, train_scorer):
        from cst_captioning_amd.ops.cider_d import CiderDScorer
        if id(ds) not in self._cache:
            ds.df = train_scorer.ds.df  # train-split document frequencies
            self._cache[id(ds)] = CiderDScorer(ds, use_eos=1, device=dev)
        self.sc = self._cache[id(ds)]

    def score(self, seq, vid):
        return self.sc.score(seq, vid)


def log(phase, step, out):
    rec = {'impl': impl, 'precision': precision if impl == 'torch' else 'bf16',
           'phase': phase, 'step': step, 'loss': round(float(out['loss']), 5)}
    if 'reward' in out:
        rec.update(reward_mean=round(float(out['reward'].float().mean()), 5),
                   sample_cider=round(float(out['m']), 5), greedy_cider=round(float(out['b']), 5))
    rec['val_greedy_cider'] = round(val_cider(), 5)
    rec['skipped'] = int(t.optimizer.skipped()) if hasattr(t.optimizer, 'skipped') else None
    if eng is not None:
        rec['exp_fix_rows'] = int(eng.exp_fix_rows.item())
    print(json.dumps(rec), flush=True)


t.rl_training = False
for it in range(xe_steps):
    out = t.train_step(loader.get_batch(), 0)
    if it % 50 == 0 or it == xe_steps - 1:
        log('xe', it, out)
t.rl_training = True
model.set_mixer_from(1)
for g in t.optimizer.param_groups:
    g['lr'] = 2e-4
for it in range(rl_steps):
    out = t.train_step(loader.get_batch(), 0)
    if it % 25 == 0 or it == rl_steps - 1:
        log('scst', it, out)
