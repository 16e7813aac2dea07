"""Device stamps of the trainer's data-parallel step at the HEADLINE shape
(64 videos x 20 captions, V = 10,509, L = 30): the DP code path with a 1-rank
gloo group standing in for RCCL (DistContext world size 2, so the streamed
bucket, the slice events and the two graphs are built as under RCCL; each
collective is a no-op), so the stamps show where each slice's all-reduce can
start inside the replayed backward.  Prints one JSON line: the mean stamps
(us after the step start) of a few back-to-back replays.  Input of
profiles/r5/dp_model_n8.md."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

from cst_captioning_amd.cli import build_model, seed_everything
from cst_captioning_amd.config import default_opts
from cst_captioning_amd.data import CaptionLoader, make_synthetic
from cst_captioning_amd.parallel import DistContext
from cst_captioning_amd.train.trainer import Trainer
from cst_captioning_amd.utils import stamps


def main(port):
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('gloo', rank=0, world_size=1, init_method='tcp://127.0.0.1:%s' % port)
    ctx = DistContext(rank=0, world_size=2, local_rank=0, device=dev, backend='gloo')
    seed_everything(123, 0)
    ds = make_synthetic('msrvtt', num_videos=6513, vocab_size=10509, seed=123)
    S = 20
    opt = default_opts(batch_size=64, train_seq_per_img=S, test_seq_per_img=S, rnn_size=512,
                       input_encoding_size=512, drop_prob_lm=0.5, learning_rate=1e-4,
                       grad_clip=0.25, use_rl=1, use_rl_after=0, use_cst=0, use_mixer=1,
                       mixer_from=1, use_eos=1, impl='hip', loglevel='WARNING', save_last=0)
    opt.vocab = {i: w for i, w in enumerate(ds.vocab)}
    opt.vocab_size, opt.seq_length, opt.feat_dims = ds.vocab_size, ds.seq_length, ds.feat_dims
    loader = CaptionLoader(ds, 64, S, 'train', dev, 0, 2, 123)
    model, engine = build_model(opt, dev, 'hip')
    tr = Trainer(opt, model, loader, None, ctx, engine)
    tr.rl_training = True
    stamps.enable(dev)
    for _ in range(6):
        tr.train_step(loader.get_batch(), 0)
    acc, n = {}, 4
    for _ in range(n):
        tr.train_step(loader.get_batch(), 0)
        tr.train_step(loader.get_batch(), 0)
        for k, v in stamps.read().items():
            acc[k] = acc.get(k, 0.0) + v / n
    stamps.disable()
    out = {k: round(v, 1) for k, v in sorted(acc.items(), key=lambda kv: kv[1])}
    out['_events_ok'] = bool(tr._graph_events_ok)
    out['_grad_slices_mb'] = [round((hi - lo) * 4 / 1e6, 2) for lo, hi in tr.bucket.groups]
    out['_grad_total_mb'] = round(tr.bucket.grad.numel() * 4 / 1e6, 2)
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else '29533')
