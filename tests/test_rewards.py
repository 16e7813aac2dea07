"""Reward arithmetic against the golden values of SURVEY.md §4.3.

The goldens were captured from the reference ``get_cst_reward`` /
``get_self_critical_reward`` (``/root/reference/utils.py:169-324``) with a
fake scorer whose score is the caption length.
"""
import numpy as np
import pytest
import torch

from cst_captioning_amd.reward.rewards import (cst_from_scores, get_cst_reward,
                                               get_self_critical_reward, scst_from_scores)


class LengthScorer:
    """compute_score(gts, res) -> (mean, per-hyp caption length)."""

    def compute_score(self, gts, res):
        s = np.array([len(r['caption'][0].split()) for r in res], dtype=np.float64)
        return s.mean(), s


B, S, T = 2, 3, 5


def _model_res():
    # rows of lengths [1, 2, 3] for every video (tokens >= 3, no EOS inside)
    res = np.zeros((B * S, T), dtype=np.int64)
    for i in range(B * S):
        n = i % S + 1
        res[i, :n] = 5 + np.arange(n)
    return res


def _gts():
    return [np.array([[1, 5, 6, 0, 0, 0]]) for _ in range(B)]


BCMR = np.array([[1., 2., 3.], [4., 5., 6.]])


def test_cst_scb_baseline2():
    r, m, b = get_cst_reward(_model_res(), _gts(), LengthScorer(), BCMR, expand_feat=1,
                             seq_per_img=S, scb_captions=2, scb_baseline=2, use_mixer=1)
    assert r.shape == (B * S, T)
    np.testing.assert_allclose(r[:, 0], [-0.5, 0.5, 1.5, -0.5, 0.5, 1.5])
    assert (r == r[:, :1]).all()
    assert m == pytest.approx(2.0) and b == pytest.approx(1.5)


def test_cst_scb_baseline1():
    r, m, b = get_cst_reward(_model_res(), _gts(), LengthScorer(), BCMR, expand_feat=1,
                             seq_per_img=S, scb_captions=2, scb_baseline=1, use_mixer=1)
    np.testing.assert_allclose(r[:, 0], [-0.5, 0.5, 1.5, -3.5, -2.5, -1.5])
    assert m == pytest.approx(2.0) and b == pytest.approx(3.5)


def test_wxe_reward_is_gt_consensus():
    r, m, b = get_cst_reward(_model_res(), _gts(), LengthScorer(), BCMR, expand_feat=1,
                             seq_per_img=S, scb_captions=0, scb_baseline=1, use_mixer=0)
    np.testing.assert_allclose(r[:, 0], [1, 2, 3, 4, 5, 6])
    assert m == pytest.approx(3.5) and b == 0


def test_scst_greedy_length2():
    greedy = np.zeros((B * S, T), dtype=np.int64)
    greedy[:, :2] = [7, 8]
    r, m, g = get_self_critical_reward(_model_res(), greedy, _gts(), LengthScorer(),
                                       expand_feat=1, seq_per_img=S)
    assert r.shape == (B * S, T)
    np.testing.assert_allclose(r[:, 0], [-1, 0, 1, -1, 0, 1])
    assert m == pytest.approx(2.0) and g == pytest.approx(2.0)


@pytest.mark.parametrize('baseline', [1, 2])
def test_device_and_host_baselines_agree(baseline):
    rng = np.random.RandomState(0)
    scores = rng.rand(4, 20)
    bcmr = rng.rand(4, 20)
    rn, mn, bn = cst_from_scores(scores, bcmr, 7, baseline)
    rt, mt, bt = cst_from_scores(torch.from_numpy(scores), torch.from_numpy(bcmr), 7, baseline)
    np.testing.assert_allclose(rt.numpy(), rn, rtol=1e-12)
    assert float(mt) == pytest.approx(mn) and float(bt) == pytest.approx(bn)
    rs, _, _ = scst_from_scores(torch.from_numpy(scores), torch.from_numpy(bcmr))
    np.testing.assert_allclose(rs.numpy(), scores - bcmr)


def test_scb_baseline_invalid():
    with pytest.raises(ValueError):
        cst_from_scores(np.ones((2, 3)), None, 2, 1)
    with pytest.raises(ValueError):
        cst_from_scores(np.ones((2, 3)), np.ones((2, 3)), 2, 3)
