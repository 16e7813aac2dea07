"""Fused SCST loss (``csrc/kernels/loss.hip``): self-critical reward, the
reference's reward mask and the REINFORCE loss in one launch forward and one
backward (reference ``utils.py:215-224``, ``model.py`` RewardCriterion,
``train.py:223-246`` for the logged means).  Same arithmetic as
:func:`~cst_captioning_amd.reward.rewards.scst_from_scores` followed by
:class:`~cst_captioning_amd.models.criteria.RewardCriterion`, fp32."""
import torch

from .. import _ext


class _SCSTLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, seq, lp, sample, greedy):
        loss, out, reward = _ext.ops().scst_loss_forward(seq, lp.detach().float().contiguous(),
                                                         sample.float().contiguous(),
                                                         greedy.float().contiguous())
        ctx.save_for_backward(seq, reward, out)
        ctx.mark_non_differentiable(reward, out)
        return loss, reward, out

    @staticmethod
    def backward(ctx, dloss, _dr, _do):
        seq, reward, out = ctx.saved_tensors
        dlp = _ext.ops().scst_loss_backward(seq, reward, out, dloss.float().reshape(1).contiguous())
        return None, dlp, None, None


def scst_loss(seq, logprobs, sample_scores, greedy_scores):
    """(loss, reward (R,), m, b): ``greedy_scores`` per row (R,) or per
    video (R / rows-per-video,)."""
    loss, reward, out = _SCSTLossFn.apply(seq.contiguous(), logprobs, sample_scores,
                                          greedy_scores)
    return loss, reward, out[1], out[2]
