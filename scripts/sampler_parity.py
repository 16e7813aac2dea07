"""Sampler parity at fixed weights: the fused engine's MIXER rollout against
the PyTorch decoder path (torch.multinomial over log_softmax, reference
model.py:326-337) on the SAME weights and batches, after an XE warm-up.

Explains a gap between two SCST learning curves: if both samplers draw from
the same distribution, their sampled-caption CIDEr-D, lengths and log-probs
agree here to within sampling noise, and a gap in the curves comes from the
trajectories (different random draws amplified by training), not from a
biased sampler.  Prints one JSON line per implementation.

usage: python scripts/sampler_parity.py [XE_STEPS] [BATCHES]
(CSTCAP_PARITY_SHAPE=headline: the headline model shape)
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cst_captioning_amd.cli import build_model  # noqa: E402
from cst_captioning_amd.config import default_opts  # noqa: E402
from cst_captioning_amd.data import CaptionLoader, make_splits  # noqa: E402
from cst_captioning_amd.parallel import DistContext  # noqa: E402
from cst_captioning_amd.train.trainer import Trainer  # noqa: E402

xe_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
n_batches = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device('cuda', 0)
torch.manual_seed(0)
if os.environ.get('CSTCAP_PARITY_SHAPE') == 'headline':
    V_, FD_, NV_, B_, H_ = 10509, [2048, 4096, 1024, 300], 6513, 64, 512
else:
    V_, FD_, NV_, B_, H_ = 2000, [256, 128], 1280, 32, 256
tr, va, _ = make_splits('msrvtt', vocab_size=V_, feat_dims=FD_, train_videos=NV_, seed=0)
opt = default_opts(batch_size=B_, train_seq_per_img=20, rnn_size=H_, input_encoding_size=H_,
                   learning_rate=2e-3, max_epochs=10 ** 9, print_log_interval=0, impl='hip',
                   loglevel='WARNING', use_rl=1, use_rl_after=10 ** 6, use_cst=0, use_mixer=1,
                   mixer_from=1, use_eos=1, drop_prob_lm=0.5)
opt.vocab = {i: w for i, w in enumerate(tr.vocab)}
opt.vocab_size, opt.seq_length, opt.feat_dims = tr.vocab_size, tr.seq_length, tr.feat_dims
loader = CaptionLoader(tr, B_, 20, 'train', dev, seed=0)
model, eng = build_model(opt, dev, 'hip')
assert eng is not None, 'the fused engine must be active'
t = Trainer(opt, model, loader, None, DistContext(device=dev), eng)
t.rl_training = False
for _ in range(xe_steps):
    t.train_step(loader.get_batch(), 0)
scorer = t._ensure_scorer()
model.train()
model.set_mixer_from(1)
batches = [loader.get_batch() for _ in range(n_batches)]


def lengths(seq):
    alive = torch.cumprod((seq > 0).long(), 1)
    return alive.sum(1).float()


for impl in ('hip', 'torch'):
    model.impl = impl
    scores, lens, lps = [], [], []
    torch.manual_seed(1)
    with torch.no_grad():
        for data in batches:
            if impl == 'hip':
                seq, lp, _ = eng.rollout(model, data['feats'], data['labels'])
            else:
                _, seq, lp = model(data['feats'], data['labels'])
            S = loader.get_seq_per_img()
            sc = scorer.score(seq, data['video_index'].repeat_interleave(S)).float()
            scores.append(sc)
            lens.append(lengths(seq))
            alive = torch.cumprod((seq > 0).long(), 1)
            # log-prob of the emitted caption up to and including its EOS
            keep = torch.cat([torch.ones_like(alive[:, :1]), alive[:, :-1]], 1).float()
            lps.append((lp.float() * keep).sum(1))
    s, ln, l = torch.cat(scores), torch.cat(lens), torch.cat(lps)
    n = s.numel()
    print(json.dumps({'impl': impl, 'captions': n,
                      'sample_cider_mean': round(float(s.mean()), 5),
                      'sample_cider_stderr': round(float(s.std() / math.sqrt(n)), 5),
                      'length_mean': round(float(ln.mean()), 4),
                      'length_stderr': round(float(ln.std() / math.sqrt(n)), 4),
                      'caption_logprob_mean': round(float(l.mean()), 4),
                      'caption_logprob_stderr': round(float(l.std() / math.sqrt(n)), 4)}),
          flush=True)
model.impl = 'hip'
