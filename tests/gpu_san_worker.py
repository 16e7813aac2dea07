"""Worker for tests/test_gpu_debug.py::test_engine_under_host_ubsan: drives the
host runtime of the HOST-SANITIZED extension (``_C_san``: UBSan with abort on
the first error, libstdc++ bounds checks; setup.py ``CSTCAP_HOST_SANITIZE=1``)
through every decoder configuration and the captured training step, in a
fresh process with ``CSTCAP_EXT=san``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = [  # (rnn_type, model_type, num_layers, num_chunks)
    ('lstm', 'concat', 1, 1), ('lstm', 'concat', 1, 4), ('gru', 'concat', 2, 1),
    ('rnn', 'standard', 1, 1), ('lstm', 'manet', 1, 1)]


def decoder_paths(cell, mt, nl, C):
    import torch
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.models import CaptionModel, RewardCriterion
    from cst_captioning_amd.models.decoder_engine import DecoderEngine
    dev = 'cuda'
    H = 64
    ds = make_synthetic('msrvtt', num_videos=24, vocab_size=300, seq_length=12,
                        feat_dims=[48, 32], num_chunks=C, seed=0)
    opt = default_opts(vocab_size=300, seq_length=12, feat_dims=[48, 32], train_seq_per_img=5,
                       rnn_size=H, input_encoding_size=2 * H if mt == 'standard' else H,
                       drop_prob_lm=0.5, num_chunks=C, rnn_type=cell, model_type=mt,
                       num_layers=nl)
    torch.manual_seed(0)
    model = CaptionModel(opt).to(dev)
    eng = DecoderEngine(model, opt)
    model.impl, model._engine = 'hip', eng
    data = CaptionLoader(ds, 4, 5, 'train', dev, seed=0).get_batch()
    model.train()
    model.set_mixer_from(1)
    seq, g_sel, _ = eng.rollout(model, data['feats'], data['labels'])
    RewardCriterion()(seq, g_sel, torch.randn(seq.size(0), device=dev)).backward()
    model.zero_grad()
    full, _, _ = model(data['feats'], data['labels'])  # full log-probs, dense dS
    full.sum().backward()
    with torch.no_grad():
        eng.sample(model, data['feats'], {'sample_max': 0, 'temperature': 0.8})
        model.eval()
        eng.sample_beam(model, data['feats'], {'beam_size': 3})
    torch.cuda.synchronize()


def graph_training():
    import torch
    from cst_captioning_amd.cli import build_model
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.parallel import DistContext
    from cst_captioning_amd.train.trainer import Trainer
    ds = make_synthetic('msrvtt', num_videos=48, vocab_size=500, seq_length=12,
                        feat_dims=[64, 32], seed=0)
    opt = default_opts(vocab_size=500, seq_length=12, feat_dims=[64, 32], train_seq_per_img=5,
                       batch_size=8, rnn_size=128, input_encoding_size=128, drop_prob_lm=0.5,
                       use_rl=1, use_rl_after=0, use_cst=0, use_mixer=1, mixer_from=1,
                       use_eos=1, impl='hip', cuda_graph=1, learning_rate=1e-3)
    opt.vocab = {i: w for i, w in enumerate(ds.vocab)}
    dev = torch.device('cuda')
    model, eng = build_model(opt, dev, 'hip')
    loader = CaptionLoader(ds, 8, 5, 'train', dev, seed=0)
    tr = Trainer(opt, model, loader, None, DistContext(device=dev), eng)
    tr.rl_training = True
    for _ in range(4):
        tr.train_step(loader.get_batch(), 0)
    assert tr._graph is not None
    torch.cuda.synchronize()


def main():
    from cst_captioning_amd import _ext
    assert _ext.ops().__file__.split('/')[-1].startswith('_C_san'), _ext.ops().__file__
    for cfg in CONFIGS:
        decoder_paths(*cfg)
        print('ubsan ok', cfg, flush=True)
    graph_training()
    print('ubsan ok graph training', flush=True)


if __name__ == '__main__':
    main()
