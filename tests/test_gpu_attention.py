"""Temporal attention (num_chunks > 1) on the fused HIP engine vs the PyTorch
CaptionModel path (fp32 reference of the same model): teacher-forced
log-probs and every parameter gradient (attention scorer, frame projection,
LSTM, vocab head, FeatPool), REINFORCE gradients through a rollout, greedy
decoding and beam search.  Kernels: csrc/kernels/attention.hip
(att_fwd_kernel / att_bwd_kernel) plus the K = 4H + A recurrent backward GEMM
at H = A = 64; at H = A = 128 the MFMA path (att_mfma.h workgroups inside the
decode launch, the lstm.hip dalpha epilogue and att_bwd_mfma).
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _tiny(C=4, V=300, H=64, feat_dims=(48, 32), S=5, B=6, L=12, seed=0):
    # (feat_dims: FeatPool output F * H; the attention size equals H)
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.models import CaptionModel
    ds = make_synthetic('msrvtt', num_videos=40, vocab_size=V, seq_length=L,
                        feat_dims=list(feat_dims), num_chunks=C, seed=seed)
    opt = default_opts(vocab_size=V, seq_length=L, feat_dims=list(feat_dims),
                       train_seq_per_img=S, rnn_size=H, input_encoding_size=H,
                       drop_prob_lm=0.0, num_chunks=C)
    torch.manual_seed(seed)
    model = CaptionModel(opt).to(DEV)
    with torch.no_grad():  # non-trivial decoder and attention
        model.logit.weight.mul_(3.0)
        model.core.rnn.weight_hh_l0.mul_(2.0)
        model.temporal_att.align.weight.mul_(4.0)
    loader = CaptionLoader(ds, B, S, 'train', DEV, seed=seed)
    return ds, opt, model, loader


def _engine(model, opt):
    from cst_captioning_amd.models.decoder_engine import DecoderEngine, engine_supports
    assert engine_supports(opt)
    return DecoderEngine(model, opt)


def _grad_errors(model, ref):
    out = {}
    for (name, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        if name == 'temporal_att.align.bias':
            # softmax is shift-invariant: the exact gradient is 0 (both sides
            # hold rounding noise only)
            assert p.grad is None or float(p.grad.abs().max()) < 1e-3
            continue
        if q.grad is None or q.grad.norm() == 0:
            continue
        out[name] = float((p.grad - q.grad).norm() / (q.grad.norm() + 1e-12))
    return out


@pytest.mark.parametrize('C,H,S', [(4, 64, 5), (8, 64, 5), (12, 64, 5), (8, 128, 10),
                                   (12, 128, 16), (3, 128, 4)])
def test_attention_teacher_forced_matches_torch(C, H, S):
    ds, opt, model, loader = _tiny(C=C, H=H, S=S)
    eng = _engine(model, opt)
    model.train()
    data = loader.get_batch()
    labels = data['labels']
    assert data['feats'][0].dim() == 3 and data['feats'][0].size(1) == C
    ref = copy.deepcopy(model)
    ref.impl = 'torch'
    pred = ref(data['feats'], labels)[0]
    tgt = labels[:, 1:1 + pred.size(1)]
    ref_lp = pred.gather(2, tgt.unsqueeze(2)).squeeze(2)
    g_xe = eng.teacher_forced(model, data['feats'], labels)
    n = pred.size(1)
    m = data['masks'][:, 1:1 + n] > 0
    assert (g_xe[:, :n][m] - ref_lp[m]).abs().max() < 0.08
    from cst_captioning_amd.models import CrossEntropyCriterion
    crit = CrossEntropyCriterion()
    crit(pred, labels[:, 1:], data['masks'][:, 1:]).backward()
    crit(g_xe, labels[:, 1:], data['masks'][:, 1:]).backward()
    errs = _grad_errors(model, ref)
    for k in ('temporal_att.f_h.weight', 'temporal_att.f_feat.weight',
              'temporal_att.align.weight', 'core.rnn.weight_ih_l0', 'core.rnn.weight_hh_l0'):
        assert k in errs, (k, sorted(errs))
    bad = {k: v for k, v in errs.items() if v > 0.06}
    assert not bad, bad


@pytest.mark.parametrize('H,S', [(64, 5), (128, 10)])
def test_attention_rollout_gradient_matches_torch(H, S):
    ds, opt, model, loader = _tiny(C=6, seed=2, H=H, S=S)
    eng = _engine(model, opt)
    model.train()
    model.set_mixer_from(1)
    data = loader.get_batch()
    seq, g_sel, _ = eng.rollout(model, data['feats'], data['labels'])
    w = torch.randn(seq.size(0), device=DEV)
    from cst_captioning_amd.models import RewardCriterion
    RewardCriterion()(seq, g_sel, w).backward()
    ref = copy.deepcopy(model)
    ref.impl = 'torch'
    ref.zero_grad(set_to_none=True)
    ref.set_mixer_from(0)
    lab = torch.cat([data['labels'][:, :1], seq, torch.zeros_like(seq[:, :1])], 1)
    pred = ref(data['feats'], lab)[0]
    lp_ref = pred[:, :seq.size(1)].gather(2, seq[:, :pred.size(1)].unsqueeze(2)).squeeze(2)
    k = lp_ref.size(1)
    assert (g_sel[:, :k] - lp_ref).abs().max() < 0.08
    RewardCriterion()(seq[:, :k], lp_ref, w).backward()
    bad = {n: v for n, v in _grad_errors(model, ref).items() if v > 0.08}
    assert not bad, bad


@pytest.mark.parametrize('H,S', [(64, 5), (128, 10)])
def test_attention_greedy_and_beam_match_torch(H, S):
    ds, opt, model, loader = _tiny(C=5, seed=3, H=H, S=S)
    with torch.no_grad():
        model.logit.weight.mul_(3.0)  # peaked distributions: few near-ties
    eng = _engine(model, opt)
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
        b_ref, _ = ref.sample(data['feats'], {'beam_size': K})
        b, _ = eng.sample_beam(model, data['feats'], {'beam_size': K})
        assert b.shape == b_ref.shape
        assert (b == b_ref).all(1).float().mean().item() >= 0.8, (K, b, b_ref)




def test_fused_attention_backward_fp16_scorer_values_near_saturation():
    """The fused attention backward reads the forward's scorer values u =
    tanh(P + q) as one fp16 word each (common.h u_enc: 1 - |u| with u's
    sign), the per-step launch recomputes tanh in fp32.  With the scorer
    inputs scaled so most u are saturated (|u| > 0.99), the attention
    parameters' gradients of the two paths agree to 1e-2 relative (the
    plain fp16 u lost up to all of 1 - u^2 there)."""
    from cst_captioning_amd import _ext
    from cst_captioning_amd.models import CrossEntropyCriterion
    ops = _ext.ops()
    ds, opt, model, loader = _tiny(C=8, H=128, S=10)
    with torch.no_grad():
        model.temporal_att.f_feat.weight.mul_(8.0)  # saturate tanh(P + q)
    eng = _engine(model, opt)
    model.train()
    data = loader.get_batch()
    grads = {}
    try:
        for fuse in (False, True):
            ops.set_att_fuse(fuse)
            model.zero_grad(set_to_none=True)
            torch.manual_seed(0)
            g_xe = eng.teacher_forced(model, data['feats'], data['labels'])
            CrossEntropyCriterion()(g_xe, data['labels'][:, 1:], data['masks'][:, 1:]).backward()
            grads[fuse] = {n: p.grad.clone() for n, p in model.named_parameters()
                           if p.grad is not None}
    finally:
        ops.set_att_fuse(True)
    for k in ('temporal_att.f_h.weight', 'temporal_att.f_feat.weight', 'temporal_att.f_feat.bias',
              'temporal_att.align.weight', 'core.rnn.weight_hh_l0'):
        a, b = grads[True][k], grads[False][k]
        err = ((a - b).norm() / (b.norm() + 1e-20)).item()
        assert err < 1e-2, (k, err)


@pytest.mark.parametrize('H', [128, 512])
def test_attention_inputs_node_matches_fp32_module_path(H):
    """ops/featpool.py _AttInputsFn (FeatPool + ONE bf16-operand GEMM for the
    per-frame gate table Gv and the projected frames P, fp32 accumulation and
    fp32 gradients) against the model's fp32 module path (FeatPool module,
    the W_ih video-column Linear and temporal_att.f_feat): outputs and the
    gradients of W_ih's video columns, f_feat and the FeatPool parameters
    under random upstream gradients.  Stated tolerance: 1e-2 relative (only
    the GEMM operands and the upstream gradient are bf16-rounded)."""
    from cst_captioning_amd.ops.featpool import att_inputs
    ds, opt, model, loader = _tiny(C=8, H=H, S=5, feat_dims=(96, 64))
    eng = _engine(model, opt)
    model.eval()  # (no FeatPool dropout: both paths see the same frames)
    data = loader.get_batch()
    feats = data['feats']
    gv, pre = att_inputs(eng, model, feats)
    ref = copy.deepcopy(model)
    frames = ref.feat_pool(feats)  # (B, C, F*H), fp32 module
    w_iv = ref.core.rnn.weight_ih_l0[:, eng.E:]
    gv_ref = eng.pack_rows(torch.nn.functional.linear(frames, w_iv), eng.src_ie, 2)
    pre_ref = ref.temporal_att.f_feat(frames)
    for a, b in ((gv, gv_ref), (pre, pre_ref)):
        assert ((a - b).norm() / b.norm()).item() < 1e-2
    g = torch.Generator(device=DEV).manual_seed(7)
    dgv = torch.randn(gv.shape, device=DEV, generator=g)
    dpre = torch.randn(pre.shape, device=DEV, generator=g)
    torch.autograd.backward([gv, pre], [dgv, dpre])
    torch.autograd.backward([gv_ref, pre_ref], [dgv, dpre])
    names = ['core.rnn.weight_ih_l0', 'temporal_att.f_feat.weight', 'temporal_att.f_feat.bias']
    names += [n for n, _ in model.named_parameters() if n.startswith('feat_pool')]
    got = dict(model.named_parameters())
    want = dict(ref.named_parameters())
    for n in names:
        a, b = got[n].grad, want[n].grad
        assert a is not None and b is not None, n
        if n == 'core.rnn.weight_ih_l0':  # the video columns (the token columns: no gradient here)
            a, b = a[:, eng.E:], b[:, eng.E:]
        err = ((a - b).norm() / (b.norm() + 1e-20)).item()
        assert err < 1e-2, (n, err)
