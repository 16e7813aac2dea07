"""Command-line entry points: ``train`` and ``test``.

Same flags and flow as ``/root/reference/train.py:421-519`` and
``/root/reference/test.py:22-77``; one process per GPU under torchrun for
data parallelism (``torchrun --nproc-per-node N -m cst_captioning_amd.cli train ...``).
"""
import json
import logging
import os
import sys
from datetime import datetime

import numpy as np
import torch

from .config import parse_opts
from .data import CaptionLoader, VideoCaptionDataset, make_splits
from .models import CaptionModel
from .parallel import init_distributed

logger = logging.getLogger('cst_captioning_amd')


def setup_logging(opt, rank=0):
    level = getattr(logging, opt.loglevel.upper()) if rank == 0 else logging.WARNING
    logging.basicConfig(level=level, format='%(asctime)s:%(levelname)s: %(message)s')


def seed_everything(seed, rank=0):
    np.random.seed(seed + rank)
    torch.manual_seed(seed + rank)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed + rank)


def load_splits(opt):
    if opt.synthetic:
        n = opt.synthetic_videos or None
        return make_splits(opt.synthetic, vocab_size=opt.synthetic_vocab,
                           seq_length=opt.seq_length, feat_dims=opt.feat_dims,
                           num_chunks=opt.num_chunks, train_videos=n, seed=opt.seed,
                           with_consensus=bool(opt.use_cst and opt.scb_baseline == 1) or
                           bool(opt.use_cst and not opt.use_mixer),
                           seq_per_img=opt.train_seq_per_img)
    df = opt.train_cached_tokens if isinstance(opt.train_cached_tokens, str) else None
    tr = VideoCaptionDataset.from_files(opt.train_label_h5, opt.train_feat_h5, opt.num_chunks,
                                        opt.train_bcmrscores_pkl, opt.eval_metric,
                                        opt.train_cocofmt_file, df)
    va = VideoCaptionDataset.from_files(opt.val_label_h5, opt.val_feat_h5, opt.num_chunks,
                                        cocofmt_file=opt.val_cocofmt_file) \
        if opt.val_label_h5 else None
    te = VideoCaptionDataset.from_files(opt.test_label_h5, opt.test_feat_h5, opt.num_chunks,
                                        cocofmt_file=opt.test_cocofmt_file) \
        if opt.test_label_h5 else None
    return tr, va, te


def build_model(opt, device, impl=None):
    model = CaptionModel(opt).to(device)
    impl = impl or opt.impl
    engine = None
    if impl == 'auto':
        impl = 'hip' if device.type == 'cuda' else 'torch'
    if impl == 'hip' and getattr(opt, 'precision', 'bf16') == 'fp32':
        # the fused engine computes with bf16 MFMA operands; fp32 means the
        # plain PyTorch path
        logger.warning('--precision fp32: using the PyTorch decoder path (the HIP engine is bf16)')
        return model, None
    if impl == 'hip':
        from .models.decoder_engine import DecoderEngine, engine_unsupported_reason
        why = engine_unsupported_reason(opt)
        if why is not None:
            # (the engine covers lstm / gru / rnn cells, concat / standard /
            # manet models, up to 5 stacked layers and temporal attention)
            logger.warning('fused HIP decoder: %s; using the PyTorch decoder path', why)
            return model, None
        engine = DecoderEngine(model, opt)
        model.impl = 'hip'
        model._engine = engine
    return model, engine


def train_main(argv=None):
    opt = parse_opts(argv)
    ctx = init_distributed()
    setup_logging(opt, ctx.rank)
    logger.info('Input arguments: %s', json.dumps(vars(opt), sort_keys=True, indent=4,
                                                 default=str))
    seed_everything(opt.seed, ctx.rank)
    tr, va, te = load_splits(opt)
    dev = ctx.device
    train_loader = CaptionLoader(tr, opt.batch_size, opt.train_seq_per_img, 'train', dev,
                                 ctx.rank, ctx.world_size, opt.seed)
    val_loader = CaptionLoader(va, opt.test_batch_size, opt.test_seq_per_img, 'test', dev) \
        if va is not None else None
    test_loader = CaptionLoader(te, opt.test_batch_size, opt.test_seq_per_img, 'test', dev) \
        if te is not None else None
    opt.vocab = train_loader.get_vocab()
    opt.vocab_size = train_loader.get_vocab_size()
    opt.seq_length = train_loader.get_seq_length()
    opt.feat_dims = train_loader.get_feat_dims()
    if opt.model_file:
        opt.history_file = opt.model_file.replace('.pth', '_history.json', 1)
        d = os.path.dirname(opt.model_file)
        if d:
            os.makedirs(d, exist_ok=True)
    logger.info('Building model...')
    model, engine = build_model(opt, dev)
    from .train.trainer import Trainer
    trainer = Trainer(opt, model, train_loader, val_loader, ctx, engine)
    start = datetime.now()
    infos = trainer.train()
    logger.info('Best val %s score: %f. Best iter: %d. Best epoch: %d', opt.eval_metric,
                infos['best_score'], infos['best_iter'], infos['best_epoch'])
    logger.info('Training time: %s', datetime.now() - start)
    if opt.result_file and test_loader is not None:
        from .train.checkpoint import load_checkpoint
        if opt.model_file and os.path.exists(opt.model_file):
            model.load_state_dict(load_checkpoint(opt.model_file, dev)['model'])
            if engine is not None:
                engine.refresh_weights()
        trainer.test(test_loader)
    ctx.destroy()
    return infos


def test_main(argv=None):
    opt = parse_opts(argv)
    ctx = init_distributed()
    setup_logging(opt, ctx.rank)
    from .train.checkpoint import load_checkpoint
    ck = load_checkpoint(opt.model_file, 'cpu')
    copt = ck['opt']
    for k in ('model_type', 'vocab', 'vocab_size', 'seq_length', 'feat_dims'):
        setattr(opt, k, getattr(copt, k))
    if opt.synthetic:
        _, _, te = load_splits(opt)
    else:
        te = VideoCaptionDataset.from_files(opt.test_label_h5, opt.test_feat_h5,
                                            opt.num_chunks,
                                            cocofmt_file=opt.test_cocofmt_file)
    loader = CaptionLoader(te, opt.test_batch_size, opt.test_seq_per_img, 'test', ctx.device)
    assert opt.vocab_size == loader.get_vocab_size()
    assert opt.seq_length == loader.get_seq_length()
    assert list(opt.feat_dims) == list(loader.get_feat_dims())
    model, engine = build_model(opt, ctx.device)
    model.load_state_dict(ck['model'])
    if engine is not None:
        engine.refresh_weights()
    from .train.trainer import Trainer
    res = Trainer(opt, model, loader, None, ctx, engine).test(loader)
    ctx.destroy()
    return res


def main():
    if len(sys.argv) < 2 or sys.argv[1] not in ('train', 'test'):
        print('usage: python -m cst_captioning_amd.cli {train,test} [flags]')
        sys.exit(2)
    cmd = sys.argv.pop(1)
    (train_main if cmd == 'train' else test_main)()


if __name__ == '__main__':
    main()
