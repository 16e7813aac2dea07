"""Worker for tests/test_gpu_debug.py: one SCST-style step of the fused engine
(rollout + greedy + beam, backward) in a fresh process, so that
CSTCAP_LAUNCH_CHECK (read once per process) takes effect."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(C):
    import torch
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.models import CaptionModel, RewardCriterion
    from cst_captioning_amd.models.decoder_engine import DecoderEngine
    dev = 'cuda'
    ds = make_synthetic('msrvtt', num_videos=24, vocab_size=300, seq_length=12,
                        feat_dims=[48, 32], num_chunks=C, seed=0)
    opt = default_opts(vocab_size=300, seq_length=12, feat_dims=[48, 32], train_seq_per_img=5,
                       rnn_size=64, input_encoding_size=64, drop_prob_lm=0.5, num_chunks=C)
    torch.manual_seed(0)
    model = CaptionModel(opt).to(dev)
    eng = DecoderEngine(model, opt)
    loader = CaptionLoader(ds, 4, 5, 'train', dev, seed=0)
    data = loader.get_batch()
    model.train()
    model.set_mixer_from(1)
    seq, g_sel, _ = eng.rollout(model, data['feats'], data['labels'])
    RewardCriterion()(seq, g_sel, torch.randn(seq.size(0), device=dev)).backward()
    with torch.no_grad():
        eng.sample(model, data['feats'], {'sample_max': 1})
        model.eval()
        eng.sample_beam(model, data['feats'], {'beam_size': 3})
    torch.cuda.synchronize()
    print('launch-check ok C=%d' % C)


if __name__ == '__main__':
    main(int(sys.argv[1]))
