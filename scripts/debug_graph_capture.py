"""Bisect a HIP-graph capture crash: one trainer config per process
(argv: H V feat_dims... validate(0/1) drop)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cst_captioning_amd.cli import build_model, load_splits  # noqa: E402
from cst_captioning_amd.config import parse_opts  # noqa: E402
from cst_captioning_amd.data import CaptionLoader  # noqa: E402
from cst_captioning_amd.parallel import DistContext  # noqa: E402
from cst_captioning_amd.train.trainer import Trainer  # noqa: E402

H, V, S, B, L, val = (int(x) for x in sys.argv[1:7])
fd = sys.argv[7].split(',')
args = ['--synthetic', 'msvd', '--synthetic_videos', '24', '--synthetic_vocab', str(V),
        '--seq_length', str(L), '--rnn_size', str(H), '--input_encoding_size', str(H),
        '--feat_dims'] + fd + ['--batch_size', str(B), '--train_seq_per_img', str(S),
        '--test_batch_size', '3', '--test_seq_per_img', str(S), '--beam_size', '2',
        '--impl', 'hip', '--loglevel', 'WARNING', '--drop_prob_lm', '0',
        '--learning_rate', '1e-3', '--language_eval', '0']
opt = parse_opts(args)
dev = torch.device('cuda', 0)
tr_ds, va, _ = load_splits(opt)
loader = CaptionLoader(tr_ds, opt.batch_size, opt.train_seq_per_img, 'train', dev, 0, 1, opt.seed)
opt.vocab, opt.vocab_size = loader.get_vocab(), loader.get_vocab_size()
opt.seq_length, opt.feat_dims = loader.get_seq_length(), loader.get_feat_dims()
model, engine = build_model(opt, dev)
tr = Trainer(opt, model, loader, None, DistContext(device=dev), engine)
if val:
    tr.validate(CaptionLoader(va, 3, S, 'test', dev))
for i in range(4):
    out = tr.train_step(loader.get_batch(), 0)
    torch.cuda.synchronize()
    print('step', i, float(out['loss']), 'graph' if tr._graph is not None else 'eager', flush=True)
print('OK', sys.argv[1:])
