"""One decode step through ``decode_step_test``: the tiled decode launch
(csrc/kernels/vocab.hip vocab_tr_block + vocab_combine_kernel) against fp32
PyTorch.

  * teacher-forced step with the exp store and the recurrent GEMM (+ video
    gates): LSE, target log-prob, E = exp(x - eoff) rows, pre = h W_hh^T +
    vgate, at the headline shape and at a row count that is not a multiple
    of the 64-row tiles;
  * step 0's fp16 logits rows (entries past V hold -inf);
  * greedy selection = argmax of the fp32 logits;
  * multinomial sampling: chi-square of 10,240 draws against softmax;
  * the combine's token selection and cell epilogue for each selection mode,
    with and without the end-of-sequence rules, at 1,280 / 1,000 / 64 rows
    (the greedy baseline's shape): the cell against an fp32 PyTorch LSTM
    cell, teacher forcing, the "all rows ended" stop.

(A fused form with the combine folded into the decode launch -- merge and
cell in the launch's recurrent tiles after in-launch waits -- measured
slower, 58.0 vs 35.5 + 14.4 us per step at 1,280 rows and 28.7 vs 7.9 + 8.4
us at 64, profiles/r4/README_r4.md, and was removed.)

The reference decoder step is /root/reference/model.py:281 (logit Linear),
:326-337 (log_softmax, multinomial / max) and :234-271 (LSTM step, the
all-rows-ended stop and the per-row mask of sample())."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'
E0 = torch.empty(0)


def _ops():
    from cst_captioning_amd import _ext
    return _ext.ops()


def _inputs(R, V, H=512, vdiv=20, seed=0, wscale=0.1):
    g = torch.Generator(device=DEV).manual_seed(seed)
    hd = torch.randn(R, H, device=DEV, generator=g).bfloat16()
    h = (torch.rand(R, H, device=DEV, generator=g) * 2 - 1).bfloat16()
    W = (torch.randn(V, H, device=DEV, generator=g) * wscale).bfloat16()
    b = torch.randn(V, device=DEV, generator=g) * 0.5
    whh = (torch.randn(4 * H, H, device=DEV, generator=g) / H ** 0.5).bfloat16()
    vg = torch.randn((R + vdiv - 1) // vdiv, 4 * H, device=DEV, generator=g)
    tgt = torch.randint(0, V, (R,), device=DEV, generator=g)
    return hd, h, W, b, whh, vg, tgt


def _ref_logits(hd, W, b):
    return hd.float() @ W.float().t() + b


def _step(ops, hd, h, W, b, whh, vg, vdiv, tgt, eoff, save, mode, step, rng,
          ptab=E0, c_prev=E0, drop_p=0.0, cell=0, eos=0, unfinished=E0, ss_prob=0.0):
    return ops.decode_step_test(hd, h, W, b, whh, vg, vdiv, tgt, eoff, save, mode, step, rng,
                                ptab, c_prev, drop_p, cell, eos, unfinished, ss_prob)


@pytest.mark.parametrize('R', [1280, 1000])
def test_teacher_forced_exp_store_and_recurrent(R):
    ops = _ops()
    V, H, vdiv = 10509, 512, 20
    R = R - R % vdiv
    hd, h, W, b, whh, vg, tgt = _inputs(R, V, H, vdiv)
    x = _ref_logits(hd, W, b)
    lse_ref = torch.logsumexp(x, 1)
    g = torch.Generator(device=DEV).manual_seed(7)
    eoff = lse_ref + torch.randn(R, device=DEV, generator=g) * 2  # a previous step's LSE
    rng = torch.tensor([11, 22], dtype=torch.int32, device=DEV)
    pre_ref = h.float() @ whh.float().t() + vg.repeat_interleave(vdiv, 0)
    e_ref = torch.exp(x - eoff[:, None])
    out = _step(ops, hd, h, W, b, whh, vg, vdiv, tgt, eoff, 2, 0, 3, rng)
    lse, tok, gsel, gxe, saved, pre, n = out[:7]
    assert int(n) == (V + 127) // 128
    torch.testing.assert_close(lse, lse_ref, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(gxe, x.gather(1, tgt[:, None]).squeeze(1) - lse_ref,
                               rtol=1e-5, atol=2e-4)
    assert (tok == tgt).all()  # mode 0: teacher forcing
    torch.testing.assert_close(saved[:, :V].float(), e_ref, rtol=1e-2, atol=1e-30)
    assert (saved[:, V:].float() == 0).all()
    torch.testing.assert_close(pre, pre_ref, rtol=1e-5, atol=1e-4)


def test_fp16_logits_rows():
    ops = _ops()
    R, V = 1280, 10509
    hd, h, W, b, whh, vg, tgt = _inputs(R, V, seed=1)
    x = _ref_logits(hd, W, b)
    rng = torch.tensor([5, 6], dtype=torch.int32, device=DEV)
    out = _step(ops, hd, h, W, b, E0, E0, 1, tgt, E0, 1, 0, 0, rng)
    lse, saved = out[0], out[4]
    torch.testing.assert_close(saved[:, :V].float(), x, rtol=2e-3, atol=2e-3)
    assert torch.isinf(saved[:, V:].float()).all() and (saved[:, V:].float() < 0).all()
    torch.testing.assert_close(lse, torch.logsumexp(x, 1), rtol=1e-5, atol=1e-4)


def test_greedy_is_argmax():
    ops = _ops()
    R, V = 1280, 10509
    hd, h, W, b, whh, vg, tgt = _inputs(R, V, seed=2)
    x = _ref_logits(hd, W, b)
    rng = torch.tensor([1, 2], dtype=torch.int32, device=DEV)
    out = _step(ops, hd, h, W, b, E0, E0, 1, E0, E0, 0, 2, 0, rng)
    tok, gsel = out[1], out[2]
    ref = x.argmax(1)
    top2 = x.topk(2, 1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-3  # rows without a near-tie
    assert (tok[clear] == ref[clear]).all()
    lp = torch.log_softmax(x, 1).gather(1, tok[:, None]).squeeze(1)
    torch.testing.assert_close(gsel, lp, rtol=1e-5, atol=2e-4)


def test_sampling_matches_softmax():
    from scipy.stats import chi2
    ops = _ops()
    R, V, H = 1280, 1000, 512  # V not a multiple of the 128-entry tiles
    g = torch.Generator(device=DEV).manual_seed(3)
    row = torch.randn(1, H, device=DEV, generator=g)
    hd = row.expand(R, H).contiguous().bfloat16()
    W = (torch.randn(V, H, device=DEV, generator=g) * 0.06).bfloat16()
    b = torch.randn(V, device=DEV, generator=g) * 0.5
    x = _ref_logits(hd[:1], W, b)[0]
    p = torch.softmax(x.double(), 0)
    counts = torch.zeros(V, dtype=torch.float64, device=DEV)
    for step in range(8):
        rng = torch.tensor([1000 + step, 77], dtype=torch.int32, device=DEV)
        out = _step(ops, hd, E0, W, b, E0, E0, 1, E0, E0, 0, 1, step, rng)
        tok, gsel = out[1], out[2]
        counts += torch.bincount(tok, minlength=V).double()
        lp = torch.log_softmax(x, 0)[tok]
        torch.testing.assert_close(gsel, lp, rtol=1e-5, atol=2e-4)
    N = counts.sum()
    exp = p * N
    big = exp >= 5
    obs_b, exp_b = counts[big], exp[big]
    rest_o, rest_e = counts[~big].sum(), exp[~big].sum()
    stat = ((obs_b - exp_b) ** 2 / exp_b).sum()
    dof = int(big.sum()) - 1
    if rest_e >= 5:
        stat = stat + (rest_o - rest_e) ** 2 / rest_e
        dof += 1
    pval = chi2.sf(float(stat), dof)
    assert pval > 1e-4, (float(stat), dof, pval)


def _cell_inputs(R, V, H, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    ptab = (torch.randn(V, 4 * H, device=DEV, generator=g) * 0.5).half()  # (the engine's fp16 table)
    c_prev = torch.randn(R, H, device=DEV, generator=g)
    return ptab, c_prev


# (mode, eos, with unfinished mask, save): teacher forcing with the exp
# store, MIXER sampling with the all-rows-ended counter, greedy with the
# per-row finished mask, scheduled sampling, greedy with a dead previous step
CASES = [(0, 1, False, 2), (1, 1, False, 2), (2, 0, True, 0), (3, 1, False, 2), (2, 2, True, 0)]


@pytest.mark.parametrize('R,vdiv', [(1280, 20), (1000, 20), (64, 1)])
@pytest.mark.parametrize('mode,eos,unf,save', CASES)
def test_combine_cell_matches_fp32(R, vdiv, mode, eos, unf, save):
    ops = _ops()
    V, H = 10509, 512
    hd, h, W, b, whh, vg, tgt = _inputs(R, V, H, vdiv, seed=11 + mode)
    ptab, c_prev = _cell_inputs(R, V, H, seed=5)
    eoff = torch.logsumexp(_ref_logits(hd, W, b), 1) + 1.0 if save == 2 else E0
    rng = torch.tensor([123, 456], dtype=torch.int32, device=DEV)
    mask0 = (torch.rand(R, device=DEV) > 0.3).to(torch.uint8) if unf else None
    um = mask0.clone() if unf else E0
    o = _step(ops, hd, h, W, b, whh, vg, vdiv, tgt, eoff, save, mode, 4, rng, ptab=ptab,
              c_prev=c_prev, drop_p=0.5, cell=0, eos=eos, unfinished=um, ss_prob=0.5)
    torch.cuda.synchronize()
    tok = o[1]
    if eos == 2:
        assert (tok == 0).all()  # every row ended at the previous step
    if mode == 0 and eos != 2:
        assert torch.equal(tok, tgt * mask0 if unf else tgt)  # teacher forcing
    if unf:  # rows stay finished; a finished row gets token 0
        assert torch.equal(um.bool(), mask0.bool() & (tok > 0))
    if eos == 1:  # the step's "some row is alive" flag
        assert bool((o[11].view(3, -1)[2] != 0).any()) == bool((tok != 0).any())
    # the cell against fp32 PyTorch: gates = h W_hh^T + vgate + P[token]
    pre = h.float() @ whh.float().t() + vg.repeat_interleave(vdiv, 0)[:R]
    gates = (pre + ptab[tok].float()).view(R, H, 4)
    i_, f_, g_, o_ = (gates[..., k] for k in range(4))
    c_ref = torch.sigmoid(f_) * c_prev + torch.sigmoid(i_) * torch.tanh(g_)
    h_ref = torch.sigmoid(o_) * torch.tanh(c_ref)
    torch.testing.assert_close(o[8], c_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(o[7].float(), h_ref, rtol=1e-2, atol=1e-2)
    hd_out = o[9].float()
    kept = hd_out != 0
    assert 0.4 < kept.float().mean().item() < 0.6  # dropout 0.5 on h
    torch.testing.assert_close(hd_out[kept], 2 * o[7].float()[kept], rtol=1e-2, atol=1e-2)
