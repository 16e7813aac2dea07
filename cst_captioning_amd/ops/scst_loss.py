"""Fused SCST / CST loss (``csrc/kernels/loss.hip``): the reward (self-critical,
or the consensus baseline of CST), the reference's reward mask and the
REINFORCE loss in one launch forward and one backward (reference
``utils.py:215-224`` and ``292-324``, ``model.py`` RewardCriterion,
``train.py:182-194, 223-246`` for the logged means).  Same arithmetic as
:func:`~cst_captioning_amd.reward.rewards.scst_from_scores` /
:func:`~cst_captioning_amd.reward.rewards.cst_from_scores` followed by
:class:`~cst_captioning_amd.models.criteria.RewardCriterion`, fp32."""
import torch

from .. import _ext


class _SCSTLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, seq, lp, sample, greedy, cst):
        lp32 = lp.detach().float().contiguous()
        if cst is None:
            loss, out, reward = _ext.ops().scst_loss_forward(seq, lp32, sample.float().contiguous(),
                                                             greedy.float().contiguous())
        else:
            S, k = cst
            bref = (greedy.float().contiguous().reshape(-1) if greedy is not None
                    else torch.empty(0, device=lp.device))
            loss, out, reward = _ext.ops().cst_loss_forward(seq, lp32,
                                                            sample.float().contiguous().reshape(-1),
                                                            bref, S, k)
        ctx.save_for_backward(seq, reward, out)
        ctx.mark_non_differentiable(reward, out)
        return loss, reward, out

    @staticmethod
    def backward(ctx, dloss, _dr, _do):
        seq, reward, out = ctx.saved_tensors
        dlp = _ext.ops().scst_loss_backward(seq, reward, out, dloss.float().reshape(1).contiguous())
        return None, dlp, None, None, None


class _XELossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, labels, lp, off):
        loss, out, cnt = _ext.ops().xe_loss_forward(labels, lp.detach().float().contiguous(), off)
        ctx.save_for_backward(cnt, out)
        ctx.T = lp.size(1)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        cnt, out = ctx.saved_tensors
        dlp = _ext.ops().xe_loss_backward(cnt, out, dloss.float().reshape(1).contiguous(), ctx.T)
        return None, dlp, None


def xe_loss(labels, logprobs, off=1):
    """CrossEntropyCriterion(logprobs, labels[:, off:], masks[:, off:]) with
    the loader's masks (caption plus EOS: positions < nonzeros + 1,
    ``data/dataset.py`` gather) computed from the full label rows in the same
    launch: ``logprobs`` (R, T) are the gathered GT log-probs of label columns
    off .. off + T - 1."""
    return _XELossFn.apply(labels.contiguous(), logprobs, int(off))


def scst_loss(seq, logprobs, sample_scores, greedy_scores):
    """(loss, reward (R,), m, b): ``greedy_scores`` per row (R,) or per
    video (R / rows-per-video,)."""
    loss, reward, out = _SCSTLossFn.apply(seq.contiguous(), logprobs, sample_scores,
                                          greedy_scores, None)
    return loss, reward, out[1], out[2]


def cst_loss(seq, logprobs, scores, bcmrscores, scb_captions, scb_baseline):
    """(loss, reward (R,), m, b) of the CST recipe: ``scores`` (B, S) of the
    rewarded rows, ``bcmrscores`` (B, S) GT consensus scores (needed for
    ``scb_baseline=1``), the baseline the mean of each video's
    ``scb_captions`` lowest reference scores (0: no baseline)."""
    B, S = scores.shape
    if scb_captions > 0 and scb_baseline not in (1, 2):
        raise ValueError('unknown scb_baseline!')
    if scb_captions > 0 and scb_baseline == 1 and bcmrscores is None:
        raise ValueError('scb_baseline=1 needs the GT consensus scores')
    bref = bcmrscores if (scb_captions > 0 and scb_baseline == 1) else None
    loss, reward, out = _SCSTLossFn.apply(seq.contiguous(), logprobs, scores, bref,
                                          (int(S), min(int(scb_captions), int(S))))
    return loss, reward, out[1], out[2]
