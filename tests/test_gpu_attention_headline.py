"""MFMA temporal attention (csrc/kernels/att_mfma.h, the lstm.hip attention
epilogue and attention.hip att_bwd_mfma) against fp32 PyTorch references:

  * the attention workgroups alone, over query widths A = 128..512, frame
    counts 3..16 (8- and 16-frame padding) and 2..32 rows per video;
  * the headline shape with attention (C = 8 frames, H = E = A = 512,
    V = 10,509, 64 videos x 20 captions = 1,280 rows, logit dropout 0.5):
    teacher-forced log-probs and every parameter gradient, and the REINFORCE
    gradient through a MIXER rollout, at the 2 % gradient-norm tolerance of
    the non-attention headline tests.

The reference decoder is the model's own temporal attention
(``cst_captioning_amd/models/modules.py`` TemporalAttention: the reference
only declares ``--num_chunks``, /root/reference/opts.py:241-245, and asserts
C == 1 in FeatPool, /root/reference/model.py:61-66) run in fp32 on the
engine's bf16-rounded weights with the engine's dropout masks."""
import pytest
import torch

from test_gpu_headline import dropout_keep_mask, _grad_errors

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.mark.parametrize('Bv,vdiv,C,A,H', [(64, 20, 8, 512, 512), (7, 32, 16, 256, 128),
                                           (9, 2, 3, 128, 256), (5, 13, 12, 384, 64),
                                           # one row per video: the SCST greedy baseline
                                           (64, 1, 8, 512, 512), (9, 1, 3, 128, 256)])
@pytest.mark.parametrize('whole', [1, 0])
def test_att_mfma_kernel_matches_fp32(Bv, vdiv, C, A, H, whole):
    from cst_captioning_amd import _ext
    ops = _ext.ops()
    g = torch.Generator(device=DEV).manual_seed(Bv * 31 + C)
    R = Bv * vdiv
    h = (torch.rand(R, H, device=DEV, generator=g) * 2 - 1).bfloat16()
    wq = (torch.randn(A, H, device=DEV, generator=g) / H ** 0.5).bfloat16()
    P = torch.randn(Bv, C, A, device=DEV, generator=g)
    wa = torch.randn(A, device=DEV, generator=g) * 0.3
    ba = torch.randn(1, device=DEV, generator=g)
    gv = torch.randn(Bv, C, 4 * H, device=DEV, generator=g)
    # whole = 1: one workgroup per video over every query slice; 0: A / 64
    # workgroups per video with the last-arriver hand-off
    vg, alpha, q = ops.att_mfma_fwd(h, wq, P, wa, ba, gv, whole)
    q_ref = h.float() @ wq.float().t()
    torch.testing.assert_close(q, q_ref, rtol=1e-4, atol=1e-4)
    pb = P.repeat_interleave(vdiv, 0)  # (R, C, A)
    e = torch.tanh(pb + q_ref[:, None, :]) @ wa + ba
    al_ref = torch.softmax(e, 1)
    torch.testing.assert_close(alpha, al_ref, rtol=2e-4, atol=2e-5)
    vg_ref = torch.bmm(al_ref.bfloat16().float().unsqueeze(1),
                       gv.bfloat16().float().repeat_interleave(vdiv, 0)).squeeze(1)
    err = (vg.float() - vg_ref).norm() / vg_ref.norm()
    assert err < 5e-3, float(err)


def _att_model(seed=0, drop=0.5, C=8):
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.models import CaptionModel
    from cst_captioning_amd.models.decoder_engine import DecoderEngine
    ds = make_synthetic('msrvtt', num_videos=128, vocab_size=10509, seq_length=30, seed=seed,
                        num_chunks=C)
    opt = default_opts(vocab_size=10509, seq_length=30, feat_dims=ds.feat_dims,
                       train_seq_per_img=20, rnn_size=512, input_encoding_size=512,
                       drop_prob_lm=drop, num_chunks=C)
    torch.manual_seed(seed)
    model = CaptionModel(opt).to(DEV)
    for m in model.feat_pool.feat_list:  # isolate the decoder's logit dropout
        m[2].p = 0.0
    with torch.no_grad():  # attention weights that actually vary over frames
        model.temporal_att.align.weight.mul_(8.0)
    eng = DecoderEngine(model, opt)
    loader = CaptionLoader(ds, 64, 20, 'train', DEV, seed=seed)
    return model, eng, loader


def _reference_att_logprobs(model, feats, tokens_in, targets, seed, drop, S):
    """fp32 teacher-forced attention decoder on bf16-rounded weights with the
    engine's dropout masks: log p(targets[:, t]) (R, T) and the weights."""
    E, H = model.input_encoding_size, model.rnn_size
    w = {n: p.detach().bfloat16().float().requires_grad_(True)
         for n, p in model.named_parameters()}
    outs = []
    for i, f in enumerate(feats):  # FeatPool per frame (B, C, F*H)
        W = w['feat_pool.feat_list.%d.0.weight' % i]
        b = w['feat_pool.feat_list.%d.0.bias' % i]
        outs.append(torch.relu(f @ W.t() + b))
    frames = torch.cat(outs, -1).repeat_interleave(S, 0)  # (R, C, F*H)
    pre = frames @ w['temporal_att.f_feat.weight'].t() + w['temporal_att.f_feat.bias']
    R = tokens_in.size(0)
    h = torch.zeros(R, H, device=DEV)
    c = torch.zeros(R, H, device=DEV)
    w_ih, w_hh = w['core.rnn.weight_ih_l0'], w['core.rnn.weight_hh_l0']
    out = []
    for t in range(tokens_in.size(1)):
        q = h @ w['temporal_att.f_h.weight'].t()
        e = (torch.tanh(pre + q[:, None, :]) @ w['temporal_att.align.weight'].t()).squeeze(-1) \
            + w['temporal_att.align.bias']
        al = torch.softmax(e, 1)
        ctx = torch.bmm(al.unsqueeze(1), frames).squeeze(1)
        x = w['embed.weight'][tokens_in[:, t]]
        g = torch.cat([x, ctx], 1) @ w_ih.t() + h @ w_hh.t()
        i, f, gg, o = g.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        hd = h
        if drop > 0:
            hd = h * dropout_keep_mask(seed, t, R, H, drop) / (1.0 - drop)
        lp = torch.log_softmax(hd @ w['logit.weight'].t() + w['logit.bias'], -1)
        out.append(lp.gather(1, targets[:, t:t + 1]).squeeze(1))
    return torch.stack(out, 1), w


def _check_grads(model, w, tol, loose=()):
    errs = _grad_errors(model, w)
    errs.pop('temporal_att.align.bias', None)  # softmax shift invariance: exactly 0
    for k in ('temporal_att.f_h.weight', 'temporal_att.f_feat.weight',
              'temporal_att.align.weight', 'core.rnn.weight_ih_l0', 'core.rnn.weight_hh_l0',
              'logit.weight', 'embed.weight'):
        assert k in errs, (k, sorted(errs))
    bad = {k: v for k, v in errs.items()
           if v > (2.5 * tol if any(k.startswith(p) for p in loose) else tol)}
    assert not bad, errs


def test_headline_attention_teacher_forced_matches_fp32():
    from cst_captioning_amd.models import CrossEntropyCriterion
    model, eng, loader = _att_model()
    seed = 24681357
    eng._rng = lambda dev: torch.tensor([seed, 99], dtype=torch.int32, device=DEV)
    model.train()
    model.set_seq_per_img(20)
    data = loader.get_batch()
    labels, masks = data['labels'], data['masks']
    assert labels.shape == (1280, 30) and data['feats'][0].shape[1] == 8
    g_xe = eng.teacher_forced(model, data['feats'], labels)
    T = g_xe.size(1)
    ref_lp, w = _reference_att_logprobs(model, data['feats'], labels[:, :T], labels[:, 1:T + 1],
                                        seed, 0.5, 20)
    m = masks[:, 1:T + 1] > 0
    diff = (g_xe - ref_lp).abs()[m]
    assert diff.max().item() < 0.05, diff.max().item()
    assert diff.mean().item() < 5e-3, diff.mean().item()
    crit = CrossEntropyCriterion()
    crit(g_xe, labels[:, 1:], masks[:, 1:]).backward()
    crit(ref_lp, labels[:, 1:], masks[:, 1:]).backward()
    _check_grads(model, w, 0.02)


def test_headline_attention_rollout_reinforce_matches_fp32():
    from cst_captioning_amd.models import RewardCriterion
    model, eng, loader = _att_model(seed=1)
    seed = 13572468
    eng._rng = lambda dev: torch.tensor([seed, 555], dtype=torch.int32, device=DEV)
    model.train()
    model.set_seq_per_img(20)
    model.set_mixer_from(1)
    data = loader.get_batch()
    labels = data['labels']
    seq, g_sel, _ = eng.rollout(model, data['feats'], labels)
    torch.manual_seed(5)
    reward = torch.randn(seq.size(0), device=DEV)
    RewardCriterion()(seq, g_sel, reward).backward()
    k = seq.size(1)
    tokens_in = torch.cat([labels[:, :1], seq[:, :k - 1]], 1)
    ref_lp, w = _reference_att_logprobs(model, data['feats'], tokens_in, seq, seed, 0.5, 20)
    alive = torch.cumprod((seq > 0).long(), 1) > 0
    diff = (g_sel - ref_lp).abs()[alive]
    assert diff.max().item() < 0.05, diff.max().item()
    RewardCriterion()(seq, ref_lp, reward).backward()
    # (as in the non-attention headline test, the frame encoder's gradient --
    # summed over 20 rows x 28 steps of bf16 terms per video -- is the most
    # exposed to the cancelling +-1 rewards)
    _check_grads(model, w, 0.02, loose=('feat_pool', 'temporal_att.f_feat'))
