"""Comm-stream priority under a collective-shaped load (verdict r5 item 5).

The trainer's data-parallel step at the HEADLINE shape (64 videos x 20
captions, V = 10,509, L = 30; DistContext world size 2 over a 1-rank
group, so the streamed bucket, the slice events and the replayed graphs are
built exactly as under RCCL while each collective is a no-op).  Where the
vocab-head slice's all-reduce starts -- on the comm stream, right after the
backward's event, under the reverse LSTM loop -- a stand-in kernel occupies
``blocks`` workgroups copying HBM for ``us`` microseconds (engine busy_copy;
RCCL's ring kernel on 8 ranks runs one workgroup per channel for about as
long as the slice takes over xGMI: 21 MB x 2 x 7/8 at ~50-100 GB/s).

For each comm-stream priority (high / normal) the script times back-to-back
replayed steps without and with the stand-in, plus device stamps of the
reverse loop (bwd.loop0 -> bwd.loop) and of the stand-in's start (comm0).
Prints one JSON line.  Usage: dp_standin.py PORT [BLOCKS] [US] [STEPS]."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

from cst_captioning_amd.cli import build_model, seed_everything
from cst_captioning_amd.config import default_opts
from cst_captioning_amd.data import CaptionLoader, make_synthetic
from cst_captioning_amd.parallel import DistContext
from cst_captioning_amd.train.trainer import Trainer
from cst_captioning_amd.utils import stamps


def run(dev, ctx, ds, priority, blocks, us, steps):
    S = 20
    seed_everything(123, 0)
    opt = default_opts(batch_size=64, train_seq_per_img=S, test_seq_per_img=S, rnn_size=512,
                       input_encoding_size=512, drop_prob_lm=0.5, learning_rate=1e-4,
                       grad_clip=0.25, use_rl=1, use_rl_after=0, use_cst=0, use_mixer=1,
                       mixer_from=1, use_eos=1, impl='hip', loglevel='WARNING', save_last=0,
                       comm_priority=priority)
    opt.vocab = {i: w for i, w in enumerate(ds.vocab)}
    opt.vocab_size, opt.seq_length, opt.feat_dims = ds.vocab_size, ds.seq_length, ds.feat_dims
    loader = CaptionLoader(ds, 64, S, 'train', dev, 0, 2, 123)
    model, engine = build_model(opt, dev, 'hip')
    tr = Trainer(opt, model, loader, None, ctx, engine)
    tr.rl_training = True
    out = {'priority': tr.bucket.comm.priority}

    def timed(standin):
        tr.bucket.standin = standin
        for _ in range(3):
            tr.train_step(loader.get_batch(), 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            tr.train_step(loader.get_batch(), 0)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    # interleaved: off, on, off, on
    ms_off, ms_on = [], []
    for _ in range(2):
        ms_off.append(round(timed(None), 3))
        ms_on.append(round(timed((blocks, us)), 3))
    out['ms_per_step_no_standin'] = ms_off
    out['ms_per_step_standin'] = ms_on
    # device stamps (a new capture carries the stamp nodes)
    for name, standin in (('stamps_no_standin', None), ('stamps_standin', (blocks, us))):
        tr.bucket.standin = standin
        tr._graph_key = None  # (recaptured with the stamp nodes)
        stamps.enable(dev)
        for _ in range(3):
            tr.train_step(loader.get_batch(), 0)
        acc, n = {}, 4
        for _ in range(n):
            tr.train_step(loader.get_batch(), 0)
            tr.train_step(loader.get_batch(), 0)
            for k, v in stamps.read().items():
                acc[k] = acc.get(k, 0.0) + v / n
        stamps.disable()
        keep = ('bwd.begin', 'bwd.loop0', 'bwd.loop', 'bwd.end', 'comm0', 'bwd_end', 'adam_end')
        out[name] = {k: round(v, 1) for k, v in sorted(acc.items(), key=lambda kv: kv[1])
                     if k in keep}
        st = out[name]
        if 'bwd.loop0' in st and 'bwd.loop' in st:
            out[name]['loop_us'] = round(st['bwd.loop'] - st['bwd.loop0'], 1)
    tr.bucket.standin = None
    del tr, model, engine, loader
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    port = sys.argv[1]
    blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    us = float(sys.argv[3]) if len(sys.argv) > 3 else 400.0
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    # a 1-rank RCCL communicator (backend nccl): the collectives of the
    # shipped path are real RCCL launches on the comm stream, each a no-op
    # copy (a 1-rank gloo group would route every CUDA all-reduce through the
    # host, ~5 ms per step, profiles/r6/dp_standin_gloo_distorted.json)
    dist.init_process_group('nccl', rank=0, world_size=1, init_method='tcp://127.0.0.1:%s' % port,
                            device_id=dev)
    ctx = DistContext(rank=0, world_size=2, local_rank=0, device=dev, backend='nccl')
    ds = make_synthetic('msrvtt', num_videos=6513, vocab_size=10509, seed=123)
    res = {'standin_blocks': blocks, 'standin_us': us, 'steps': steps}
    for pr in ('high', 'normal'):
        res[pr] = run(dev, ctx, ds, pr, blocks, us, steps)
        print(json.dumps({pr: res[pr]}), file=sys.stderr, flush=True)
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
