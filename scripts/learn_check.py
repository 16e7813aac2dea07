import sys, json, torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from cst_captioning_amd.config import default_opts
from cst_captioning_amd.data import make_splits, CaptionLoader
from cst_captioning_amd.cli import build_model
from cst_captioning_amd.train.trainer import Trainer
impl = sys.argv[1]; dev = torch.device(sys.argv[2]); zero = int(sys.argv[3])
torch.manual_seed(0)
tr, va, te = make_splits('msrvtt', vocab_size=400, feat_dims=[64, 32], train_videos=640, seed=0)
opt = default_opts(batch_size=32, train_seq_per_img=20, rnn_size=128, input_encoding_size=128,
                   learning_rate=2e-3, max_epochs=10**9, print_log_interval=0, impl=impl, loglevel='WARNING')
opt.vocab = {i: w for i, w in enumerate(tr.vocab)}; opt.vocab_size = tr.vocab_size
opt.seq_length = tr.seq_length; opt.feat_dims = tr.feat_dims
ld = CaptionLoader(tr, 32, 20, 'train', dev); vl = CaptionLoader(va, 32, 20, 'train', dev)
model, eng = build_model(opt, dev, impl)
t = Trainer(opt, model, ld, None, None, eng); t.device = dev; t.ctx.device = dev
def val():
    model.eval(); tot = 0
    with torch.no_grad():
        for _ in range(2):
            d = vl.get_batch()
            if zero: d['feats'] = [f * 0 for f in d['feats']]
            pred = model(d['feats'], d['labels'])[0] if eng is None else None
            if eng is None:
                tot += float(t.xe_criterion(pred, d['labels'][:, 1:], d['masks'][:, 1:]))
            else:
                lp = eng.teacher_forced(model, d['feats'], d['labels'])
                tot += float(t.xe_criterion(lp, d['labels'][:, 1:], d['masks'][:, 1:]))
    model.train(); return tot / 2
for it in range(301):
    d = ld.get_batch()
    if zero: d['feats'] = [f * 0 for f in d['feats']]
    out = t.train_step(d, 0)
    if it % 100 == 0: print(it, 'train', round(float(out['loss']), 3), 'val', round(val(), 3), flush=True)
