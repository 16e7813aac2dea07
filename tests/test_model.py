"""CaptionModel (torch path) semantics on CPU: state_dict layout, teacher
forcing, MIXER rollout, greedy/multinomial sampling, beam search vs a
per-video spec implementation of ``/root/reference/model.py:369-512``,
and the loss criteria (``model.py:7-43``).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from cst_captioning_amd.config import default_opts
from cst_captioning_amd.models import CaptionModel
from cst_captioning_amd.models.criteria import (CrossEntropyCriterion, RewardCriterion,
                                                reward_mask)

V, H, L = 23, 16, 9
DIMS = [12, 7]


def _opt(**kw):
    o = dict(vocab_size=V, rnn_size=H, input_encoding_size=H, seq_length=L, feat_dims=DIMS,
             train_seq_per_img=3, drop_prob_lm=0.0, model_type='concat', num_chunks=1)
    o.update(kw)
    return default_opts(**o)


def _feats(b, chunks=1, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(b, chunks, d, generator=g) for d in DIMS]


def _model(seed=0, **kw):
    torch.manual_seed(seed)
    m = CaptionModel(_opt(**kw))
    # larger logit weights: peaked distributions make beam choices non-trivial
    with torch.no_grad():
        m.logit.weight.mul_(20)
    return m


def test_state_dict_layout_matches_reference():
    m = CaptionModel(_opt())
    sd = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    F_ = len(DIMS)
    assert sd == {
        'embed.weight': (V, H),
        'logit.weight': (V, H), 'logit.bias': (V,),
        'feat_pool.feat_list.0.0.weight': (H, 12), 'feat_pool.feat_list.0.0.bias': (H,),
        'feat_pool.feat_list.1.0.weight': (H, 7), 'feat_pool.feat_list.1.0.bias': (H,),
        'core.rnn.weight_ih_l0': (4 * H, H + F_ * H),
        'core.rnn.weight_hh_l0': (4 * H, H),
    }
    assert float(m.logit.bias.detach().abs().max()) == 0
    assert float(m.embed.weight.detach().abs().max()) <= 0.1


def test_manet_and_standard_constraints():
    m = CaptionModel(_opt(model_type='manet'))
    assert any(k.startswith('manet.') for k in m.state_dict())
    with pytest.raises(ValueError):
        CaptionModel(_opt(model_type='standard'))
    CaptionModel(_opt(model_type='standard', feat_dims=[H]))


def _manual_teacher_forcing(m, feats, seq):
    """The reference forward loop written out with nn.LSTM directly."""
    v = m.feat_pool(feats).repeat_interleave(m.feat_expander.n, 0)
    n = seq.size(0)
    h = torch.zeros(1, n, H)
    c = torch.zeros(1, n, H)
    outs = []
    for t in range(seq.size(1) - 1):
        x = torch.cat([m.embed(seq[:, t]), v], 1)[None]
        o, (h, c) = m.core.rnn(x, (h, c))
        outs.append(F.log_softmax(m.logit(o[0]), -1))
        if t + 1 < seq.size(1) - 1 and int(seq[:, t + 1].sum()) == 0:
            break
    return torch.stack(outs, 1)


def test_teacher_forcing_matches_manual_loop():
    m = _model().eval()
    feats = _feats(2)
    seq = torch.randint(3, V, (6, L))
    seq[:, 0] = 1
    seq[:3, 6:] = 0
    lp, sseq, slp = m(feats, seq)
    ref = _manual_teacher_forcing(m, feats, seq)
    assert lp.shape == (6, L - 1, V)
    torch.testing.assert_close(lp, ref, rtol=1e-5, atol=1e-5)
    # sample_seq / sample_logprobs: the input tokens of t >= 1 and their log-probs
    torch.testing.assert_close(sseq, seq[:, 1:L - 1])
    torch.testing.assert_close(slp, lp[:, :-1].gather(2, seq[:, 1:L - 1, None])[..., 0])


def test_forward_breaks_when_all_rows_end():
    m = _model().eval()
    seq = torch.zeros(6, L, dtype=torch.long)
    seq[:, 0] = 1
    seq[:, 1:4] = 5
    lp, _, _ = m(_feats(2), seq)
    assert lp.shape[1] == 4  # steps 0..3, stop before feeding the all-EOS column


def test_mixer_rollout_tokens_and_logprobs():
    m = _model().train()
    m.set_mixer_from(1)
    torch.manual_seed(3)
    seq = torch.randint(3, V, (6, L))
    seq[:, 0] = 1
    lp, sseq, slp = m(_feats(2), seq)
    # sampled tokens' log-probs are read from the previous step's distribution
    T = sseq.size(1)
    torch.testing.assert_close(slp, lp[:, :T].gather(2, sseq[..., None])[..., 0])
    # without mask_after_eos tokens after an EOS are NOT forced to 0 (parity quirk)
    assert sseq.shape[0] == 6


def test_mask_after_eos_flag():
    torch.manual_seed(1)
    m = _model(mask_after_eos=1).train()
    m.set_mixer_from(1)
    with torch.no_grad():
        m.logit.bias[0] = 2.0  # frequent EOS
    seq = torch.randint(3, V, (30, L))
    seq[:, 0] = 1
    _, sseq, _ = m([f.repeat(5, 1, 1) for f in _feats(2)], seq)
    dead = (sseq == 0).cumsum(1) > 0
    assert (sseq[dead] == 0).all()


def test_greedy_sample_is_argmax_chain():
    m = _model().eval()
    feats = _feats(3)
    with torch.no_grad():
        seq, lps = m.sample(feats, {'sample_max': 1})
        v = m.feat_pool(feats)
        h = torch.zeros(1, 3, H)
        c = torch.zeros(1, 3, H)
        it = torch.ones(3, dtype=torch.long)
        alive = torch.ones(3, dtype=torch.bool)
        for t in range(seq.size(1)):
            o, (h, c) = m.core.rnn(torch.cat([m.embed(it), v], 1)[None], (h, c))
            lp = F.log_softmax(m.logit(o[0]), -1)
            best, it = lp.max(1)
            alive &= it > 0
            assert torch.equal(seq[:, t], it * alive)
            torch.testing.assert_close(lps[:, t], best)
    assert seq.shape[1] <= L - 2


def test_multinomial_sample_respects_unfinished_mask():
    m = _model().eval()
    torch.manual_seed(0)
    with torch.no_grad():
        seq, lps = m.sample(_feats(8), {'sample_max': 0, 'temperature': 0.7})
    dead = (seq == 0).cumsum(1) > 0
    assert (seq[dead] == 0).all()
    assert torch.isfinite(lps).all()


def _beam_spec(m, feats, K):
    """One video at a time, candidate lists sorted on the host -- the
    reference algorithm (model.py:369-512) written from its description."""
    T = m.seq_length
    v_all = m.feat_pool(feats)
    seqs, lps = [], []
    for k in range(v_all.size(0)):
        v = v_all[k:k + 1].expand(K, -1)
        h = torch.zeros(1, K, H)
        c = torch.zeros(1, K, H)
        bseq = torch.zeros(T, K, dtype=torch.long)
        blp = torch.zeros(T, K)
        bsum = torch.zeros(K)
        done = []
        logprobs = None
        for t in range(0, T - 1):
            if t == 0:
                it = torch.ones(K, dtype=torch.long)
            else:
                ys, ix = torch.sort(logprobs, 1, True)
                cands = []
                for cc in range(min(K, V)):
                    for q in range(1 if t == 1 else K):
                        cands.append((float(bsum[q] + ys[q, cc]), int(ix[q, cc]), q,
                                      float(ys[q, cc])))
                cands.sort(key=lambda x: -x[0])
                pseq, plp = bseq.clone(), blp.clone()
                nh, nc = h.clone(), c.clone()
                for vix in range(K):
                    p, w, q, r = cands[vix]
                    bseq[:t - 1, vix] = pseq[:t - 1, q]
                    blp[:t - 1, vix] = plp[:t - 1, q]
                    nh[0, vix], nc[0, vix] = h[0, q], c[0, q]
                    bseq[t - 1, vix] = w
                    blp[t - 1, vix] = r
                    bsum[vix] = p
                    if w == 0 or t == T - 2:
                        ppl = math.exp(-p / (t - 1)) if t > 1 else 10000
                        done.append((ppl, bseq[:, vix].clone(), blp[:, vix].clone()))
                h, c = nh, nc
                it = bseq[t - 1]
            o, (h, c) = m.core.rnn(torch.cat([m.embed(it), v], 1)[None], (h, c))
            logprobs = F.log_softmax(m.logit(o[0]), -1)
        done.sort(key=lambda x: x[0])  # stable: earliest harvested wins ties
        seqs.append(done[0][1])
        lps.append(done[0][2])
    return torch.stack(seqs), torch.stack(lps)


@pytest.mark.parametrize('K', [2, 5])
def test_beam_search_matches_per_video_spec(K):
    m = _model(seed=K).eval()
    feats = _feats(4, seed=K)
    with torch.no_grad():
        seq, lp = m.sample(feats, {'beam_size': K})
        rseq, rlp = _beam_spec(m, feats, K)
    assert seq.shape == (4, L)
    assert torch.equal(seq, rseq)
    torch.testing.assert_close(lp, rlp, rtol=1e-5, atol=1e-5)


def test_criteria():
    seq = torch.tensor([[5, 6, 0, 0], [7, 0, 3, 0]])
    assert reward_mask(seq).tolist() == [[1, 1, 1, 0], [1, 1, 0, 1]]
    lp = -torch.rand(2, 4)
    r = torch.tensor([2.0, -1.0])
    loss = RewardCriterion()(seq, lp, r)
    m = reward_mask(seq)
    assert float(loss) == pytest.approx(float(-(lp * r[:, None] * m).sum() / m.sum()))
    # (N, T) reward like the reference broadcast
    loss2 = RewardCriterion()(seq, lp, r[:, None].expand(2, 4))
    assert float(loss2) == pytest.approx(float(loss))
    # XE: full (N,T,V) and gathered (N,T) inputs agree; target/mask truncated
    logp = F.log_softmax(torch.randn(2, 3, 9), -1)
    tgt = torch.randint(0, 9, (2, 5))
    mask = torch.tensor([[1, 1, 1, 0, 0], [1, 1, 0, 0, 0]]).float()
    a = CrossEntropyCriterion()(logp, tgt, mask)
    b = CrossEntropyCriterion()(logp.gather(2, tgt[:, :3, None])[..., 0], tgt, mask)
    torch.testing.assert_close(a, b)
    manual = -(logp.gather(2, tgt[:, :3, None])[..., 0] * mask[:, :3]).sum() / mask[:, :3].sum()
    torch.testing.assert_close(a, manual)


def test_temporal_attention_model_runs():
    m = CaptionModel(_opt(num_chunks=4))
    seq = torch.randint(3, V, (6, L))
    seq[:, 0] = 1
    lp, _, _ = m(_feats(2, chunks=4), seq)
    lp.sum().backward()
    assert m.temporal_att is not None
    with torch.no_grad():
        s, _ = m.eval().sample(_feats(2, chunks=4), {'beam_size': 3})
    assert s.shape == (2, L)


@pytest.mark.parametrize('cell', ['lstm', 'gru', 'rnn'])
def test_engine_gate_packing_maps(cell):
    """Packed gate layout of the fused engine (decoder_engine.gate_maps): src
    and dst are inverse on the used rows, unused slots read the zero row, the
    slot code decodes (as csrc/kernels/adam.hip packed_gate_row does) to the
    same packed rows, and a packed GEMM reproduces the cell's pre-activations
    slot by slot (GRU: n_x and n_h kept apart)."""
    from cst_captioning_amd.models.decoder_engine import CELLS, DecoderEngine, gate_maps
    H, K = 8, 5
    _, G, _, _ = CELLS[cell]
    (src_ie, dst_ie, code_ie), (src_hh, dst_hh, code_hh) = gate_maps(cell, H)
    for src, dst, code in ((src_ie, dst_ie, code_ie), (src_hh, dst_hh, code_hh)):
        assert src.shape == (4 * H,) and dst.shape == (G * H,)
        assert torch.equal(src[dst], torch.arange(G * H))
        assert (src == G * H).sum() == (4 - G) * H
        rows = torch.arange(G * H)
        g = rows // H
        assert torch.equal(dst, (rows - g * H) * 4 + ((code >> (2 * g)) & 3))
    torch.manual_seed(0)
    w_ih, w_hh = torch.randn(G * H, K), torch.randn(G * H, H)
    x, h = torch.randn(3, K), torch.randn(3, H)
    a_x = (x @ DecoderEngine.pack_rows(w_ih, src_ie).t()).view(3, H, 4)
    a_h = (h @ DecoderEngine.pack_rows(w_hh, src_hh).t()).view(3, H, 4)
    px, ph = (x @ w_ih.t()).view(3, G, H), (h @ w_hh.t()).view(3, G, H)
    if cell == 'gru':  # slots r, z, n_x, n_h
        torch.testing.assert_close((a_x + a_h)[..., :2], (px + ph)[:, :2].transpose(1, 2))
        torch.testing.assert_close((a_x + a_h)[..., 2], px[:, 2])
        torch.testing.assert_close((a_x + a_h)[..., 3], ph[:, 2])
    else:
        torch.testing.assert_close((a_x + a_h)[..., :G], (px + ph).transpose(1, 2))
        assert (a_x[..., G:] == 0).all() and (a_h[..., G:] == 0).all()
    # pack_rows along another dim (the video gate table (B, C, G*H))
    gv = torch.randn(2, 3, G * H, requires_grad=True)
    pk = DecoderEngine.pack_rows(gv, src_ie, 2)
    assert pk.shape == (2, 3, 4 * H)
    pk.sum().backward()
    assert torch.equal(gv.grad, torch.ones_like(gv))
