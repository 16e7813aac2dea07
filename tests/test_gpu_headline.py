"""Kernel numerics at the headline shape (H = E = 512, V = 10,509, 64 videos
x 20 captions = 1,280 rows, L = 30) with logit dropout 0.5, and the exact
two-level sampler over the full vocabulary.

The fp32 PyTorch reference runs the reference's LSTM decoder loop
(``/root/reference/model.py:218-289``) on the engine's bf16-rounded weights and
applies the engine's own dropout keep-masks, regenerated here from the same
counter hash (``csrc/common.h`` ``dropout_keep``), so the comparison isolates
the kernels' arithmetic (bf16 MFMA operands, bf16 activations, fp32
accumulation / cell state / softmax statistics)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'
M32 = 0xFFFFFFFF


def _mul32(h, c):
    """(h * c) mod 2^32 for int64 tensors holding uint32 values."""
    lo, hi = h & 0xFFFF, h >> 16
    return (lo * c + (((hi * c) & 0xFFFF) << 16)) & M32


def _mix32(h):
    h = h ^ (h >> 16)
    h = _mul32(h, 0x85EBCA6B)
    h = h ^ (h >> 13)
    h = _mul32(h, 0xC2B2AE35)
    return h ^ (h >> 16)


def dropout_keep_mask(seed, step, R, H, p, device=DEV):
    """(R, H) bool keep-mask of csrc/common.h dropout_keep(seed, step, r, u, p)."""
    r = torch.arange(R, device=device, dtype=torch.int64)[:, None]
    u = torch.arange(H, device=device, dtype=torch.int64)[None, :]
    h1 = _mix32((seed ^ ((step * 0x9E3779B1) & M32)) ^ _mul32(r, 0x7FEB352D))
    h = _mix32(h1 ^ _mul32(u, 0x846CA68B))
    u01 = ((h >> 8) + 1).float() * (1.0 / 16777216.0)
    return u01 > p


def _headline_model(seed=0, drop=0.5):
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.models import CaptionModel
    from cst_captioning_amd.models.decoder_engine import DecoderEngine
    ds = make_synthetic('msrvtt', num_videos=128, vocab_size=10509, seq_length=30, seed=seed)
    opt = default_opts(vocab_size=10509, seq_length=30, feat_dims=ds.feat_dims,
                       train_seq_per_img=20, rnn_size=512, input_encoding_size=512,
                       drop_prob_lm=drop)
    torch.manual_seed(seed)
    model = CaptionModel(opt).to(DEV)
    for m in model.feat_pool.feat_list:  # isolate the decoder's logit dropout
        m[2].p = 0.0
    eng = DecoderEngine(model, opt)
    loader = CaptionLoader(ds, 64, 20, 'train', DEV, seed=seed)
    return model, eng, loader


def _reference_logprobs(model, feats, tokens_in, targets, seed, drop, S):
    """fp32 teacher-forced decoder on bf16-rounded weights with the engine's
    dropout masks; returns log p(targets[:, t]) at each step t (R, T)."""
    E, H = model.input_encoding_size, model.rnn_size
    w = {n: p.detach().bfloat16().float().requires_grad_(True)
         for n, p in model.named_parameters()}
    fc = feats_encode(model, w, feats).repeat_interleave(S, 0)
    R = tokens_in.size(0)
    h = torch.zeros(R, H, device=DEV)
    c = torch.zeros(R, H, device=DEV)
    w_ih, w_hh = w['core.rnn.weight_ih_l0'], w['core.rnn.weight_hh_l0']
    out = []
    for t in range(tokens_in.size(1)):
        x = w['embed.weight'][tokens_in[:, t]]
        g = torch.cat([x, fc], 1) @ w_ih.t() + h @ w_hh.t()
        i, f, gg, o = g.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        hd = h
        if drop > 0:
            hd = h * dropout_keep_mask(seed, t, R, H, drop) / (1.0 - drop)
        lp = torch.log_softmax(hd @ w['logit.weight'].t() + w['logit.bias'], -1)
        out.append(lp.gather(1, targets[:, t:t + 1]).squeeze(1))
    return torch.stack(out, 1), w


def feats_encode(model, w, feats):
    outs = []
    for i, f in enumerate(feats):
        W = w['feat_pool.feat_list.%d.0.weight' % i]
        b = w['feat_pool.feat_list.%d.0.bias' % i]
        outs.append(torch.relu(f.squeeze(1) @ W.t() + b))
    return torch.cat(outs, -1)


def _grad_errors(model, w):
    errs = {}
    for n, p in model.named_parameters():
        q = w[n].grad
        if q is None or q.norm() == 0:
            continue
        errs[n] = ((p.grad - q).norm() / q.norm()).item()
    return errs


def test_headline_teacher_forced_with_dropout_matches_fp32():
    from cst_captioning_amd.models import CrossEntropyCriterion
    model, eng, loader = _headline_model()
    seed = 987654321
    eng._rng = lambda dev: torch.tensor([seed, 4242], dtype=torch.int32, device=DEV)
    model.train()
    model.set_seq_per_img(20)
    data = loader.get_batch()
    labels, masks = data['labels'], data['masks']
    assert labels.shape == (1280, 30)
    g_xe = eng.teacher_forced(model, data['feats'], labels)  # (R, 29)
    T = g_xe.size(1)
    ref_lp, w = _reference_logprobs(model, data['feats'], labels[:, :T], labels[:, 1:T + 1],
                                    seed, 0.5, 20)
    m = masks[:, 1:T + 1] > 0
    diff = (g_xe - ref_lp).abs()[m]
    assert diff.max().item() < 0.05, diff.max().item()
    assert diff.mean().item() < 5e-3, diff.mean().item()
    crit = CrossEntropyCriterion()
    crit(g_xe, labels[:, 1:], masks[:, 1:]).backward()
    crit(ref_lp, labels[:, 1:], masks[:, 1:]).backward()
    errs = _grad_errors(model, w)
    assert {'embed.weight', 'logit.weight', 'logit.bias', 'core.rnn.weight_ih_l0',
            'core.rnn.weight_hh_l0'} <= set(errs)
    bad = {k: v for k, v in errs.items() if v > 0.02}
    assert not bad, bad


def test_headline_rollout_reinforce_gradient_with_dropout_matches_fp32():
    from cst_captioning_amd.models import RewardCriterion
    model, eng, loader = _headline_model(seed=1)
    seed = 123456789
    eng._rng = lambda dev: torch.tensor([seed, 777], dtype=torch.int32, device=DEV)
    model.train()
    model.set_seq_per_img(20)
    model.set_mixer_from(1)
    data = loader.get_batch()
    labels = data['labels']
    seq, g_sel, _ = eng.rollout(model, data['feats'], labels)  # (R, 28)
    torch.manual_seed(5)
    reward = torch.randn(seq.size(0), device=DEV)
    RewardCriterion()(seq, g_sel, reward).backward()
    # reference: teacher-force the sampled tokens (input of step t+1 = seq[:, t])
    k = seq.size(1)
    tokens_in = torch.cat([labels[:, :1], seq[:, :k - 1]], 1)
    ref_lp, w = _reference_logprobs(model, data['feats'], tokens_in, seq, seed, 0.5, 20)
    alive = torch.cumprod((seq > 0).long(), 1) > 0
    diff = (g_sel - ref_lp).abs()[alive]
    assert diff.max().item() < 0.05, diff.max().item()
    RewardCriterion()(seq, ref_lp, reward).backward()
    # the REINFORCE gradient with random +-1 rewards is a sum of largely
    # cancelling per-row terms; the video encoder's gradient (summed over 20
    # rows x 28 steps of bf16 gate gradients per video) is the most exposed
    errs = _grad_errors(model, w)
    bad = {k: v for k, v in errs.items()
           if v > (0.05 if k.startswith('feat_pool') else 0.02)}
    assert not bad, errs


@pytest.mark.parametrize('temperature', [1.0, 0.7])
def test_two_level_sampler_chi_square_full_vocab(temperature):
    """102,400 draws from softmax(x / temp) over V = 10,509 (all 83 vocab
    tiles): the logits are exact (h = e_0, W[:, 0] = x, b = 0), so the draw
    frequencies are tested against the exact distribution."""
    from scipy.stats import chisquare
    from cst_captioning_amd import _ext
    C = _ext.ops()
    V, H, R = 10509, 64, 102400
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(V, generator=g) * 1.2).bfloat16().float()
    W = torch.zeros(V, H)
    W[:, 0] = x
    hd = torch.zeros(R, H)
    hd[:, 0] = 1.0
    W, hd = W.bfloat16().to(DEV), hd.bfloat16().to(DEV)
    b = torch.zeros(V, device=DEV)
    rng = torch.tensor([31337, 271828], dtype=torch.int32, device=DEV)
    tok, lse = C.vocab_select(hd, W, b, rng, 1, temperature, 3)
    tok = tok.cpu().numpy()
    torch.testing.assert_close(lse.cpu(), torch.full((R,), float(torch.logsumexp(x, 0))),
                               rtol=1e-5, atol=1e-4)
    p = torch.softmax(x.double() / temperature, 0).numpy()
    counts = np.bincount(tok, minlength=V)
    assert counts.sum() == R
    assert len(np.unique(tok // 128)) == (V + 127) // 128  # every vocab tile drawn from
    exp = p * R
    big = exp >= 5
    obs = np.concatenate([counts[big], [counts[~big].sum()]])
    ex = np.concatenate([exp[big], [exp[~big].sum()]])
    stat, pval = chisquare(obs, ex)
    assert pval > 1e-4, (stat, pval, big.sum())
    # other seeds, other draws; greedy = first argmax
    tok2, _ = C.vocab_select(hd, W, b, rng + 1, 1, temperature, 3)
    assert (tok2.cpu().numpy() != tok).mean() > 0.5
    tg, _ = C.vocab_select(hd[:4], W, b, rng, 2, 1.0, 0)
    assert (tg.cpu().numpy() == int(torch.argmax(x))).all()


def test_headline_beam5_matches_torch_batched_beam():
    """Beam search K = 5 over 64 videos at the headline shape (H = E = 512,
    V = 10,509, L = 30): the GPU beam step (csrc/kernels/beam.hip) against the
    PyTorch batched beam search (itself pinned to a per-video spec of the
    reference's sample_beam, /root/reference/model.py:369-512, in
    tests/test_model.py) on the same bf16-rounded weights."""
    model, eng, loader = _headline_model(seed=3, drop=0.0)
    with torch.no_grad():
        model.logit.weight.mul_(3.0)  # peaked distributions: few near-ties
    eng.refresh_weights()
    model.eval()
    data = loader.get_batch()
    import copy
    ref = copy.deepcopy(model)
    ref.impl = 'torch'
    ref._engine = None
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.bfloat16().float())
        seq_ref, lp_ref = ref.sample(data['feats'], {'beam_size': 5})
        seq, lp = eng.sample_beam(model, data['feats'], {'beam_size': 5})
    assert seq.shape == seq_ref.shape == (64, 30)
    same = (seq == seq_ref).all(1)
    # bf16 hidden states against fp32 ones: where two hypotheses score within
    # rounding of each other the searches may keep different beams, so
    # videos whose captions differ must end on a beam of the same score
    assert same.float().mean().item() >= 0.6, same.float().mean().item()
    assert ((lp - lp_ref).abs()[same] < 0.05).all()

    def score(s, l):  # caption log-prob up to and including its EOS
        alive = torch.cumprod((s > 0).long(), 1)
        keep = torch.cat([torch.ones_like(alive[:, :1]), alive[:, :-1]], 1).float()
        return (l.float() * keep).sum(1)

    s_eng, s_ref = score(seq, lp), score(seq_ref, lp_ref)
    gap = (s_eng - s_ref).abs()
    assert (gap[~same] <= 0.02 * s_ref.abs()[~same] + 0.1).all(), (gap[~same], s_ref[~same])


def test_headline_beam5_graph_replay_equals_eager():
    """The beam decode replayed as a captured HIP graph (engine._beam_graphed)
    equals the eager launches bit for bit, on two different batches through
    the same graph, and after a weight update (the graph reads the engine's
    in-place shadows)."""
    import os
    model, eng, loader = _headline_model(seed=4, drop=0.0)
    model.eval()
    batches = [loader.get_batch()['feats'] for _ in range(2)]
    outs = {}
    for mode in ('1', '0'):
        os.environ['CSTCAP_BEAM_GRAPH'] = mode
        try:
            res = []
            for feats in batches:
                with torch.no_grad():
                    res.append(eng.sample_beam(model, feats, {'beam_size': 5}))
            w0 = model.logit.weight.detach().clone()
            with torch.no_grad():
                model.logit.weight.mul_(1.5)
            eng.refresh_weights()
            with torch.no_grad():
                res.append(eng.sample_beam(model, batches[1], {'beam_size': 5}))
                model.logit.weight.copy_(w0)
            eng.refresh_weights()
            outs[mode] = res
        finally:
            os.environ.pop('CSTCAP_BEAM_GRAPH', None)
    assert getattr(eng, '_beam_graphs', None), 'the graphed beam path never ran'
    for (s1, l1), (s0, l0) in zip(outs['1'], outs['0']):
        assert torch.equal(s1, s0)
        assert torch.equal(l1, l0)


@pytest.mark.parametrize('bias_shift', [0.0, 70.0])
def test_headline_teacher_forced_xe_launches_match_per_step(bias_shift):
    """XE all rows (csrc/engine.cpp: one launch per step = the vocabulary tiles
    of step t + the whole LSTM step t+1, E = exp(x) with offset 0, the combines
    on a side stream) against the general per-step launches + combine (E =
    exp(x - previous LSE)): the same target log-probs and parameter
    gradients.  bias_shift = 70 puts every row's LSE above the exp store's
    guard (|lse| > 60), so the zero-offset backward recomputes every row
    exactly (vocab_grad.hip vgrad_fix, VGradRows::zero_off)."""
    from cst_captioning_amd.models import CrossEntropyCriterion
    from cst_captioning_amd.models import decoder_engine as de
    model, eng, loader = _headline_model(seed=2)
    with torch.no_grad():
        model.logit.bias.add_(bias_shift)
    eng.refresh_weights()
    seed = 192837465
    eng._rng = lambda dev: torch.tensor([seed, 31337], dtype=torch.int32, device=DEV)
    model.train()
    model.set_seq_per_img(20)
    data = loader.get_batch()
    labels, masks = data['labels'], data['masks']
    out = {}
    saved = de.XE_ROWS
    try:
        for rows in (True, False):
            de.XE_ROWS = rows
            model.zero_grad(set_to_none=True)
            g_xe = eng.teacher_forced(model, data['feats'], labels)
            CrossEntropyCriterion()(g_xe, labels[:, 1:], masks[:, 1:]).backward()
            out[rows] = (g_xe.detach().clone(),
                         {n: p.grad.detach().clone() for n, p in model.named_parameters()
                          if p.grad is not None})
    finally:
        de.XE_ROWS = saved
    (g1, gr1), (g0, gr0) = out[True], out[False]
    m = masks[:, 1:g1.size(1) + 1] > 0
    assert torch.isfinite(g1).all()
    assert (g1 - g0).abs()[m].max().item() < 2e-3
    assert set(gr1) == set(gr0)
    for n in gr0:
        err = ((gr1[n] - gr0[n]).norm() / (gr0[n].norm() + 1e-12)).item()
        assert err < 1e-2, (n, err)
