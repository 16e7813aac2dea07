"""CST / SCST / WXE rewards.

Semantics of ``get_cst_reward`` (``/root/reference/utils.py:229-324``) and
``get_self_critical_reward`` (``utils.py:169-226``), split into two layers so
that the same arithmetic runs on the host (numpy, reference parity) and on
the device (torch tensors on HBM, no host round trip):

  1. *scoring*: a score per hypothesis (CIDEr-D from the GPU kernel, or any
     reference-style scorer on the CPU via :func:`score_hypotheses`);
  2. *baseline*: :func:`cst_from_scores` / :func:`scst_from_scores` turn the
     scores into per-sequence rewards plus the two logged means.

The reward is constant over time; the reference broadcasts it to
``(rows, T)`` with ``np.repeat`` (``utils.py:226,322``).  Here it stays one
value per row and the loss broadcasts it.
"""
import numpy as np
import torch

from ..utils.text import array_to_str


def _hyp_video(i, n_rows, seq_per_img, expand_feat):
    # utils.py:200-206, 266-272.  With expand_feat=1 hypothesis i belongs to
    # video (i % n_rows) // seq_per_img.
    if expand_feat == 1:
        return (i % n_rows) // seq_per_img
    return i % n_rows


def score_hypotheses(scorer, hyps, gts, seq_per_img, expand_feat=1, use_eos=0,
                     n_rows=None):
    """Score token-id hypotheses against per-video GT label rows on the CPU.

    ``hyps``: (N, T) int array.  ``gts``: list (one per video) of (ncap, L)
    label arrays.  Returns an (N,) float64 array.  The scorer follows the
    reference call convention (``compute_score(gts_dict, res)``).
    """
    hyps = np.asarray(hyps)
    n = hyps.shape[0]
    n_rows = n if n_rows is None else n_rows
    refs = [[array_to_str(r, use_eos) for r in g] for g in gts]
    res = [{'image_id': i, 'caption': [array_to_str(hyps[i], use_eos)]} for i in range(n)]
    gts_map = {i: refs[_hyp_video(i, n_rows, seq_per_img, expand_feat)] for i in range(n)}
    if hasattr(scorer, 'compute_score_tokens'):
        return np.asarray(scorer.compute_score_tokens(gts_map, res), dtype=np.float64)
    _, scores = scorer.compute_score(gts_map, res)
    if isinstance(scores, list) and len(scores) and isinstance(scores[0], (list, np.ndarray)):
        scores = scores[-1]  # Bleu: keep Bleu_4 (utils.py:211-213)
    return np.asarray(scores, dtype=np.float64)


def _lib(x):
    return torch if isinstance(x, torch.Tensor) else np


def cst_from_scores(scores, bcmrscores=None, scb_captions=20, scb_baseline=1):
    """Consensus baseline (``utils.py:292-324``).

    ``scores``: (B, S) scores of the rewarded sequences (samples, or the GT
    consensus scores themselves in WXE mode).  ``bcmrscores``: (B, S) GT
    consensus scores (needed for ``scb_baseline=1``).
    Returns ``(reward (B*S,), m_score, b_score)``; the means are 0-dim
    tensors for tensor input, floats for numpy input.
    """
    L = _lib(scores)
    if scb_captions > 0:
        if scb_baseline == 1:
            if bcmrscores is None:
                raise ValueError('scb_baseline=1 needs the GT consensus scores')
            ref = bcmrscores
            m_score = scores.mean()
            b_score = bcmrscores.mean()
        elif scb_baseline == 2:
            ref = scores
            m_score = scores.mean()
            b_score = None
        else:
            raise ValueError('unknown scb_baseline!')
        low = L.sort(ref, axis=1) if L is np else torch.sort(ref, dim=1).values
        low = low[:, :scb_captions]
        base = low.mean(axis=1) if L is np else low.mean(dim=1)
        if scb_baseline == 2:
            b_score = low.mean()
        reward = scores - base[:, None]
    else:
        m_score = scores.mean()
        b_score = 0.0 if L is np else torch.zeros((), dtype=scores.dtype,
                                                  device=scores.device)
        reward = scores + 0
    reward = reward.reshape(-1)
    if L is np:
        return reward, float(m_score), float(b_score)
    return reward, m_score, b_score


def scst_from_scores(sample_scores, greedy_scores):
    """Self-critical reward (``utils.py:215-224``): sample - greedy."""
    reward = sample_scores - greedy_scores
    m, g = sample_scores.mean(), greedy_scores.mean()
    if isinstance(reward, np.ndarray):
        return reward, float(m), float(g)
    return reward, m, g


def get_cst_reward(model_res, data_gts, scorer, bcmrscores=None, expand_feat=1,
                   seq_per_img=20, scb_captions=20, scb_baseline=1, use_eos=0,
                   use_mixer=0):
    """Host-side drop-in for the reference ``utils.get_cst_reward``; returns
    rewards broadcast to ``(rows, T)`` like the reference."""
    model_res = np.asarray(model_res)
    if bcmrscores is None or use_mixer == 1:
        scores = score_hypotheses(scorer, model_res, data_gts, seq_per_img,
                                  expand_feat, use_eos).reshape(-1, seq_per_img)
    else:
        scores = np.array(bcmrscores, dtype=np.float64, copy=True)
    reward, m, b = cst_from_scores(scores, None if bcmrscores is None else
                                   np.asarray(bcmrscores, dtype=np.float64),
                                   scb_captions, scb_baseline)
    return np.repeat(reward[:, None], model_res.shape[1], 1), m, b


def get_self_critical_reward(model_res, greedy_res, data_gts, scorer, expand_feat=1,
                             seq_per_img=20, use_eos=0):
    """Host-side drop-in for the reference ``utils.get_self_critical_reward``."""
    model_res = np.asarray(model_res)
    greedy_res = np.asarray(greedy_res)
    n = model_res.shape[0]
    both = np.concatenate([_pad_to(model_res, greedy_res.shape[1]),
                           _pad_to(greedy_res, model_res.shape[1])], 0)
    scores = score_hypotheses(scorer, both, data_gts, seq_per_img, expand_feat,
                              use_eos, n_rows=n)
    reward, m, g = scst_from_scores(scores[:n], scores[n:])
    return np.repeat(reward[:, None], model_res.shape[1], 1), m, g


def _pad_to(a, width):
    if a.shape[1] >= width:
        return a
    out = np.zeros((a.shape[0], width), dtype=a.dtype)
    out[:, :a.shape[1]] = a
    return out
