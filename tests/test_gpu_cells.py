"""GRU and tanh-RNN decoders (``--rnn_type gru | rnn``, reference
``opts.py`` / ``model.py:93-116``) and the ``standard`` and ``manet`` model types
(video vector as the input of step -1; modal attention, ``model.py:119-142,
273-278``) through the fused HIP
engine, against the PyTorch ``nn.GRU`` / ``nn.RNN`` / ``nn.LSTM`` path of
:class:`CaptionModel`: teacher-forced log-probs and XE gradients, REINFORCE
gradients of a MIXER rollout, greedy decoding, the GPU beam search, temporal
attention, and the graph-captured training step whose Adam pass writes the
packed bf16 shadows (unused gate slots stay zero)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'
# (rnn_type, model_type): standard feeds the video (F*H = 2H wide) as the
# step -1 input, so its input encoding size is 2H
# (rnn_type, model_type, num_layers)
VARIANTS = [('gru', 'concat', 1), ('rnn', 'concat', 1), ('lstm', 'standard', 1),
            ('gru', 'standard', 1), ('lstm', 'manet', 1), ('gru', 'manet', 1),
            ('lstm', 'concat', 2), ('gru', 'concat', 3)]
VIDS = ['%s-%s-l%d' % v for v in VARIANTS]


def _tiny(cell, V=300, H=64, S=5, B=6, L=12, seed=0, C=1, model_type='concat', layers=1):
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.models import CaptionModel
    from cst_captioning_amd.models.decoder_engine import DecoderEngine
    ds = make_synthetic('msrvtt', num_videos=40, vocab_size=V, seq_length=L,
                        feat_dims=[48, 32], num_chunks=C, seed=seed)
    opt = default_opts(vocab_size=V, seq_length=L, feat_dims=[48, 32], train_seq_per_img=S,
                       rnn_size=H, input_encoding_size=2 * H if model_type == 'standard' else H,
                       drop_prob_lm=0.0, rnn_type=cell, num_chunks=C, model_type=model_type,
                       num_layers=layers)
    torch.manual_seed(seed)
    model = CaptionModel(opt).to(DEV)
    with torch.no_grad():  # make the decoder non-trivial
        model.logit.weight.mul_(3.0)
        model.core.rnn.weight_hh_l0.mul_(2.0)
    eng = DecoderEngine(model, opt)
    loader = CaptionLoader(ds, B, S, 'train', DEV, seed=seed)
    return ds, opt, model, eng, loader


def _tol(name, base=0.06):
    """MANet's scorer biases get the sum over every row and step of
    softmax-backward terms that cancel (a row's score gradients sum to zero
    over the modalities), computed from the bf16 gate gradients: their
    relative error is the cancelled sum's, not the terms'."""
    if name.startswith('manet.') and name.endswith('bias'):
        return 0.2
    return base


def _grad_errs(model, ref, skip=()):
    out = {}
    for (name, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        if q.grad is None or q.grad.norm() == 0 or name.endswith(skip):
            continue
        out[name] = float((p.grad - q.grad).norm() / (q.grad.norm() + 1e-12))
    return out


@pytest.mark.parametrize('H', [64, 256])
@pytest.mark.parametrize('variant', VARIANTS, ids=VIDS)
def test_cell_teacher_forced_logprobs_and_grads_match_torch(variant, H):
    from cst_captioning_amd.models import CrossEntropyCriterion
    cell, mt, nl = variant
    ds, opt, model, eng, loader = _tiny(cell, V=1299 if H > 64 else 300, H=H, model_type=mt,
                                        layers=nl)
    assert eng.cell == {'lstm': 0, 'gru': 1, 'rnn': 2}[cell] and eng.standard == (mt == 'standard')
    model.train()
    data = loader.get_batch()
    labels = data['labels']
    ref = copy.deepcopy(model)
    ref.impl = 'torch'
    model.set_seq_per_img(5)
    ref.set_seq_per_img(5)
    pred = ref(data['feats'], labels)[0]
    n = pred.size(1)
    ref_lp = pred.gather(2, labels[:, 1:1 + n].unsqueeze(2)).squeeze(2)
    g_xe = eng.teacher_forced(model, data['feats'], labels)
    m = data['masks'][:, 1:1 + n] > 0
    d = (g_xe[:, :n] - ref_lp).abs()[m]
    assert d.max() < 0.08, float(d.max())
    crit = CrossEntropyCriterion()
    crit(pred, labels[:, 1:], data['masks'][:, 1:]).backward()
    crit(g_xe, labels[:, 1:], data['masks'][:, 1:]).backward()
    errs = _grad_errs(model, ref)
    assert {'core.rnn.weight_ih_l0', 'core.rnn.weight_hh_l0', 'embed.weight'} <= set(errs)
    assert {'core.rnn.weight_ih_l%d' % (nl - 1), 'core.rnn.weight_hh_l%d' % (nl - 1)} <= set(errs)
    bad = {k: v for k, v in errs.items() if v > _tol(k)}
    assert not bad, errs


@pytest.mark.parametrize('variant', VARIANTS, ids=VIDS)
def test_cell_rollout_reinforce_gradient_matches_torch(variant):
    from cst_captioning_amd.models import RewardCriterion
    ds, opt, model, eng, loader = _tiny(variant[0], seed=2, model_type=variant[1],
                                        layers=variant[2])
    model.train()
    model.set_mixer_from(1)
    model.set_seq_per_img(5)
    data = loader.get_batch()
    seq, g_sel, _ = eng.rollout(model, data['feats'], data['labels'])
    w = torch.randn(seq.size(0), device=DEV)
    RewardCriterion()(seq, g_sel, w).backward()
    ref = copy.deepcopy(model)
    ref.impl = 'torch'
    ref.zero_grad(set_to_none=True)
    ref.set_mixer_from(0)  # teacher-force the sampled tokens
    lab = torch.cat([data['labels'][:, :1], seq, torch.zeros_like(seq[:, :1])], 1)
    pred = ref(data['feats'], lab)[0]
    k = min(pred.size(1), seq.size(1))
    lp_ref = pred[:, :k].gather(2, seq[:, :k].unsqueeze(2)).squeeze(2)
    alive = torch.cumprod((seq[:, :k] > 0).long(), 1) > 0
    assert (g_sel[:, :k] - lp_ref).abs()[alive].max() < 0.08
    RewardCriterion()(seq[:, :k], lp_ref, w).backward()
    errs = _grad_errs(model, ref)
    bad = {k: v for k, v in errs.items() if v > _tol(k, 0.08)}
    assert not bad, errs


@pytest.mark.parametrize('variant', VARIANTS, ids=VIDS)
def test_cell_greedy_and_beam_match_torch(variant):
    # 24 videos: a single bf16 near-tie flip is < 5% of the rows
    ds, opt, model, eng, loader = _tiny(variant[0], seed=1, model_type=variant[1], B=24,
                                        layers=variant[2])
    with torch.no_grad():
        model.logit.weight.mul_(3.0)  # peaked distributions: few near-ties
    eng.refresh_weights()
    model.eval()
    data = loader.get_batch()
    ref = copy.deepcopy(model)
    ref.impl = 'torch'
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.bfloat16().float())
    seq_ref, _ = ref.sample(data['feats'], {'sample_max': 1})
    seq, _ = eng.sample(model, data['feats'], {'sample_max': 1})
    assert (seq[:, :4] == seq_ref[:, :4]).float().mean().item() > 0.9
    for K in (2, 4):
        b_ref, lp_ref = ref.sample(data['feats'], {'beam_size': K})
        b, lp = eng.sample_beam(model, data['feats'], {'beam_size': K})
        same = (b == b_ref).all(1)
        assert ((lp - lp_ref).abs()[same] < 0.05).all()
        # a different beam wins only on a near-tie of the ranking score (mean
        # token log-prob): deep random decoders give flat, repetitive beams
        def score(seq, l):
            n = (seq > 0).sum(1).clamp(min=1)
            return l.sum(1) / n
        tie = (score(b, lp) - score(b_ref, lp_ref)).abs() < 0.05
        assert same.float().mean().item() >= 0.7, (K, b, b_ref)
        assert (same | tie).float().mean().item() >= 0.9, (K, score(b, lp), score(b_ref, lp_ref))


def test_gru_temporal_attention_matches_torch():
    from cst_captioning_amd.models import CrossEntropyCriterion
    ds, opt, model, eng, loader = _tiny('gru', H=128, V=700, seed=3, C=4)
    assert eng.attention
    model.train()
    data = loader.get_batch()
    labels = data['labels']
    ref = copy.deepcopy(model)
    ref.impl = 'torch'
    model.set_seq_per_img(5)
    ref.set_seq_per_img(5)
    pred = ref(data['feats'], labels)[0]
    n = pred.size(1)
    ref_lp = pred.gather(2, labels[:, 1:1 + n].unsqueeze(2)).squeeze(2)
    g_xe = eng.teacher_forced(model, data['feats'], labels)
    m = data['masks'][:, 1:1 + n] > 0
    assert (g_xe[:, :n] - ref_lp).abs()[m].max() < 0.08
    crit = CrossEntropyCriterion()
    crit(pred, labels[:, 1:], data['masks'][:, 1:]).backward()
    crit(g_xe, labels[:, 1:], data['masks'][:, 1:]).backward()
    errs = _grad_errs(model, ref, skip=('align.bias',))
    bad = {k: v for k, v in errs.items() if v > 0.06}
    assert not bad, errs


@pytest.mark.parametrize('variant', VARIANTS, ids=VIDS)
def test_cell_graph_training_keeps_packed_shadows(variant):
    """Graph-captured SCST steps: the weights train, and the shadows the Adam
    pass wrote equal a fresh packing of the fp32 parameters, zero slots
    included."""
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.cli import build_model
    from cst_captioning_amd.parallel import DistContext
    from cst_captioning_amd.train.trainer import Trainer
    cell, mt, nl = variant
    ds = make_synthetic('msrvtt', num_videos=48, vocab_size=500, seq_length=12,
                        feat_dims=[64, 32], seed=0)
    opt = default_opts(vocab_size=500, seq_length=12, feat_dims=[64, 32], train_seq_per_img=5,
                       batch_size=8, rnn_size=128,
                       input_encoding_size=256 if mt == 'standard' else 128, drop_prob_lm=0.5,
                       use_rl=1, use_rl_after=0, use_cst=0, use_mixer=1, mixer_from=1,
                       use_eos=1, impl='hip', cuda_graph=1, learning_rate=1e-3, rnn_type=cell,
                       model_type=mt, num_layers=nl)
    opt.vocab = {i: w for i, w in enumerate(ds.vocab)}
    torch.manual_seed(0)
    dev = torch.device(DEV)
    model, eng = build_model(opt, dev, 'hip')
    assert eng is not None and eng.cell == {'lstm': 0, 'gru': 1, 'rnn': 2}[cell]
    loader = CaptionLoader(ds, 8, 5, 'train', dev, seed=0)
    tr = Trainer(opt, model, loader, None, DistContext(device=dev), eng)
    tr.rl_training = True
    w0 = model.core.rnn.weight_hh_l0.detach().clone()
    for _ in range(4):
        out = tr.train_step(loader.get_batch(), 0)
        assert torch.isfinite(out['loss']).item()
    assert tr._graph is not None
    assert not torch.equal(w0, model.core.rnn.weight_hh_l0.detach())
    got = [t.clone() for t in (eng.wx, eng.whh_q, eng.emb, eng.wlog, eng.current_ptab())]
    got_up = [t.clone() for t in eng.wup + eng.whh_up]
    wiv = None if eng.wiv is None else eng.wiv.clone()
    assert (wiv is None) == (mt == 'standard')
    eng.refresh_weights()
    for g, r in zip(got, (eng.wx, eng.whh_q, eng.emb, eng.wlog)):
        assert torch.equal(g, r)
    if wiv is not None:  # the video columns' packed shadow, zero rows in unused slots
        assert torch.equal(wiv, eng.wiv)
        assert not eng.wiv[(eng.src_ie == eng.gates * eng.H)].any()
    assert len(got_up) == 2 * (nl - 1)
    for g, r in zip(got_up, eng.wup + eng.whh_up):
        assert torch.equal(g, r)
    torch.testing.assert_close(got[4], eng.ptab, rtol=1e-5, atol=1e-5)
    E = eng.E
    unused_ie = eng.src_ie == eng.gates * eng.H
    unused_hh = eng.src_hh == eng.gates * eng.H
    assert unused_ie.any() == unused_hh.any() == (cell != 'lstm')
    assert (eng.wx[unused_ie, :E] == 0).all() and (eng.wx[unused_hh, E:] == 0).all()


def test_standard_with_embedding_wider_than_1024():
    """'standard' feeds the F*H-wide video vector as the step -1 input, so its
    embedding size is F*H: E = 1,152 here (the embedding-gradient row sums
    run in 1,024-column chunks)."""
    from cst_captioning_amd.models import CrossEntropyCriterion
    ds, opt, model, eng, loader = _tiny('lstm', H=576, V=700, model_type='standard')
    assert eng.E == 1152
    model.train()
    data = loader.get_batch()
    labels = data['labels']
    ref = copy.deepcopy(model)
    ref.impl = 'torch'
    model.set_seq_per_img(5)
    ref.set_seq_per_img(5)
    pred = ref(data['feats'], labels)[0]
    n = pred.size(1)
    ref_lp = pred.gather(2, labels[:, 1:1 + n].unsqueeze(2)).squeeze(2)
    g_xe = eng.teacher_forced(model, data['feats'], labels)
    m = data['masks'][:, 1:1 + n] > 0
    assert (g_xe[:, :n] - ref_lp).abs()[m].max() < 0.08
    crit = CrossEntropyCriterion()
    crit(pred, labels[:, 1:], data['masks'][:, 1:]).backward()
    crit(g_xe, labels[:, 1:], data['masks'][:, 1:]).backward()
    errs = _grad_errs(model, ref)
    assert 'embed.weight' in errs
    bad = {k: v for k, v in errs.items() if v > _tol(k)}
    assert not bad, errs
