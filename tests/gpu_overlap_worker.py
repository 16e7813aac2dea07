"""Worker of tests/test_gpu_dist.py::test_dp_slice_allreduce_starts_inside_the_backward
(one process, fresh: a long-lived test process has created many streams).

The data-parallel code path of the trainer with a 1-rank gloo process group
standing in for the collectives: the trainer is told the job has 2 ranks
(DistContext world_size 2), so it builds the streamed bucket, the slice
events and the two graphs around the all-reduce exactly as under RCCL, while
each "all-reduce" is a 1-rank no-op.  (Two processes sharing the one GPU of
the test box time-slice the device at millisecond granularity, which says
nothing about the order of one process's streams.)

Headline-like width (LSTM 512, 320 caption rows, L = 30, V = 4,000): SCST
steps captured and replayed as HIP graphs around the streamed bucket
all-reduce (parallel/dist.py).  Device stamps (utils/stamps.py) are on: the
comm stream stamps ``comm0`` right after it waited for the vocab-head
slice's event, ``comm1`` after the embedding slice's and ``comm2`` after the
W_ih + FeatPool slice's; the replayed graph
stamps ``bwd_end`` when the whole backward is done.  Saves the stamps of a
few replayed steps and whether every step's backward recorded its slice
events."""
import os
import sys

import torch

from cst_captioning_amd.cli import build_model, load_splits
from cst_captioning_amd.config import parse_opts
from cst_captioning_amd.data import CaptionLoader
from cst_captioning_amd.train.trainer import Trainer
from cst_captioning_amd.utils import stamps

ARGS = ['--synthetic', 'msrvtt', '--synthetic_videos', '64', '--synthetic_vocab', '4000',
        '--seq_length', '30', '--rnn_size', '512', '--input_encoding_size', '512',
        '--feat_dims', '512', '256', '--batch_size', '16', '--train_seq_per_img', '20',
        '--test_batch_size', '4', '--test_seq_per_img', '20', '--impl', 'hip',
        '--loglevel', 'WARNING', '--cuda_graph', '1', '--language_eval', '0',
        '--use_rl', '1', '--use_mixer', '1', '--mixer_from', '1', '--use_eos', '1']


def main(out):
    import torch.distributed as dist
    from cst_captioning_amd.parallel import DistContext
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    backend = sys.argv[3] if len(sys.argv) > 3 else 'gloo'
    kw = {'device_id': dev} if backend == 'nccl' else {}
    # ('nccl' = RCCL: a 1-rank communicator runs the real RCCL collectives of
    # the shipped path on the comm stream)
    dist.init_process_group(backend, rank=0, world_size=1,
                            init_method='tcp://127.0.0.1:%s' % sys.argv[2], **kw)
    ctx = DistContext(rank=0, world_size=2, local_rank=0, device=dev, backend=backend)
    opt = parse_opts(ARGS)
    tr_split, _, _ = load_splits(opt)
    loader = CaptionLoader(tr_split, opt.batch_size, opt.train_seq_per_img, 'train', ctx.device,
                           ctx.rank, ctx.world_size, opt.seed)
    opt.vocab, opt.vocab_size = loader.get_vocab(), loader.get_vocab_size()
    opt.seq_length, opt.feat_dims = loader.get_seq_length(), loader.get_feat_dims()
    model, engine = build_model(opt, ctx.device)
    assert engine is not None
    opt.comm_priority = os.environ.get('CSTCAP_TEST_COMM_PRIO', 'normal')
    tr = Trainer(opt, model, loader, None, ctx, engine)
    tr.rl_training = True
    standin = os.environ.get('CSTCAP_TEST_STANDIN')  # 'blocks,us': a ring-kernel stand-in
    if standin:
        b, us = standin.split(',')
        tr.bucket.standin = (int(b), float(us))
    stamps.enable(ctx.device)  # before the capture: the graph carries the stamp nodes
    runs = []
    oks = []
    for i in range(6):
        tr.train_step(loader.get_batch(), 0)
        oks.append(bool(tr._graph is not None and tr._graph_events_ok))
        if i >= 3:
            runs.append(stamps.read())
    stamps.disable()
    finite = bool(torch.isfinite(tr.bucket.data).all())
    torch.save({'stamps': runs, 'events_ok': oks, 'graphed': tr._graph is not None,
                'finite': finite, 'backend': dist.get_backend(),
                'comm_priority': tr.bucket.comm.priority, 'n_groups': len(tr.bucket.groups)},
               out)
    dist.destroy_process_group()


if __name__ == '__main__':
    main(sys.argv[1])
