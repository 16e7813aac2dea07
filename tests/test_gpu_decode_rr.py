"""Row-resident decode launch (csrc/kernels/vocab_rr.h) against fp32 PyTorch
and against the tiled launch it replaces (vocab.hip vocab_tr_block), one
decode step through ``decode_step_test`` (launch + combine, no cell):

  * teacher-forced step with the exp store and the recurrent GEMM (+ video
    gates): LSE, target log-prob, E = exp(x - eoff) rows and pre = h W_hh^T +
    vgate, at the headline shape and at a row count that is not a multiple of
    the 256-row groups;
  * step 0's fp16 logits rows (entries past V hold -inf);
  * greedy selection = argmax of the fp32 logits;
  * multinomial sampling: chi-square of 10,240 draws against softmax, and the
    sampled token's log-prob.

The reference decoder step is /root/reference/model.py:281 (logit Linear)
and :326-337 (log_softmax, multinomial / max)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


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
    vg = torch.randn(R // vdiv, 4 * H, device=DEV, generator=g)
    tgt = torch.randint(0, V, (R,), device=DEV, generator=g)
    return hd, h, W, b, whh, vg, tgt


def _ref_logits(hd, W, b):
    return hd.float() @ W.float().t() + b


def _n_tiles(V):
    return (V + 127) // 128


@pytest.mark.parametrize('R', [1280, 1000])
def test_rr_teacher_forced_exp_store_and_recurrent(R):
    ops = _ops()
    V, H, vdiv = 10509, 512, 20
    hd, h, W, b, whh, vg, tgt = _inputs(R, V, H, vdiv)
    x = _ref_logits(hd, W, b)
    lse_ref = torch.logsumexp(x, 1)
    g = torch.Generator(device=DEV).manual_seed(7)
    eoff = lse_ref + torch.randn(R, device=DEV, generator=g) * 2  # a previous step's LSE
    rng = torch.tensor([11, 22], dtype=torch.int32, device=DEV)
    pre_ref = h.float() @ whh.float().t() + vg.repeat_interleave(vdiv, 0)
    e_ref = torch.exp(x - eoff[:, None])
    outs = {}
    for rr in (1, 0):
        lse, tok, gsel, gxe, saved, pre, n = ops.decode_step_test(
            hd, h, W, b, whh, vg, vdiv, tgt, eoff, 2, 0, 3, rng, rr)
        outs[rr] = (lse, gxe, saved, pre, int(n))
        torch.testing.assert_close(lse, lse_ref, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(gxe, x.gather(1, tgt[:, None]).squeeze(1) - lse_ref,
                                   rtol=1e-5, atol=2e-4)
        assert (tok == tgt).all()  # mode 0: teacher forcing
        e = saved[:, :V].float()
        torch.testing.assert_close(e, e_ref, rtol=1e-2, atol=1e-30)
        assert (saved[:, V:].float() == 0).all()
        torch.testing.assert_close(pre, pre_ref, rtol=1e-5, atol=1e-4)
    assert outs[1][4] != _n_tiles(V), 'the row-resident launch did not run'
    assert outs[0][4] == _n_tiles(V)
    # the two launch forms agree with each other to fp32 reassociation
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(outs[1][3], outs[0][3], rtol=1e-6, atol=1e-5)
    diff = (outs[1][2].float() - outs[0][2].float()).abs()
    assert (diff <= 2 ** -7 * outs[0][2].float().abs() + 1e-30).all()  # <= 1 bf16 ulp


def test_rr_fp16_logits_rows():
    ops = _ops()
    R, V = 1280, 10509
    hd, h, W, b, whh, vg, tgt = _inputs(R, V, seed=1)
    x = _ref_logits(hd, W, b)
    rng = torch.tensor([5, 6], dtype=torch.int32, device=DEV)
    lse, tok, gsel, gxe, saved, pre, n = ops.decode_step_test(
        hd, h, W, b, torch.empty(0), torch.empty(0), 1, tgt, torch.empty(0), 1, 0, 0, rng, 1)
    assert int(n) != _n_tiles(V)
    torch.testing.assert_close(saved[:, :V].float(), x, rtol=2e-3, atol=2e-3)
    assert torch.isinf(saved[:, V:].float()).all() and (saved[:, V:].float() < 0).all()
    torch.testing.assert_close(lse, torch.logsumexp(x, 1), rtol=1e-5, atol=1e-4)


def test_rr_greedy_is_argmax():
    ops = _ops()
    R, V = 1280, 10509
    hd, h, W, b, whh, vg, tgt = _inputs(R, V, seed=2)
    x = _ref_logits(hd, W, b)
    rng = torch.tensor([1, 2], dtype=torch.int32, device=DEV)
    lse, tok, gsel, gxe, saved, pre, n = ops.decode_step_test(
        hd, h, W, b, torch.empty(0), torch.empty(0), 1, torch.empty(0), torch.empty(0), 0, 2, 0,
        rng, 1)
    assert int(n) != _n_tiles(V)
    ref = x.argmax(1)
    top2 = x.topk(2, 1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-3  # rows without a near-tie
    assert (tok[clear] == ref[clear]).all()
    lp = torch.log_softmax(x, 1).gather(1, tok[:, None]).squeeze(1)
    torch.testing.assert_close(gsel, lp, rtol=1e-5, atol=2e-4)


def test_rr_sampling_matches_softmax():
    from scipy.stats import chi2
    ops = _ops()
    R, V, H = 1280, 1000, 512  # V not a multiple of the 64-entry units
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
        lse, tok, gsel, gxe, saved, pre, n = ops.decode_step_test(
            hd, torch.empty(0), W, b, torch.empty(0), torch.empty(0), 1, torch.empty(0),
            torch.empty(0), 0, 1, step, rng, 1)
        assert int(n) != _n_tiles(V)
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
