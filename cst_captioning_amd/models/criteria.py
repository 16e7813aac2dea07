"""Loss criteria.

  * CrossEntropyCriterion -- ``/root/reference/model.py:26-43``: masked NLL,
    target/mask truncated to the prediction length.
  * RewardCriterion       -- ``model.py:7-23``: REINFORCE
    ``-sum(logp * reward * mask) / sum(mask)`` with mask = ``seq > 0``
    shifted right by one and a leading 1 (the first EOS is rewarded).

Both also accept *gathered* log-probs (what the fused HIP engine returns:
``logp[r, t]`` of the token of interest), so no ``(R, T, V)`` tensor is
needed.
"""
import torch
import torch.nn as nn


def reward_mask(seq):
    m = (seq > 0).float()
    return torch.cat([m.new_ones(m.size(0), 1), m[:, :-1]], 1)


class CrossEntropyCriterion(nn.Module):
    def forward(self, pred, target, mask):
        """pred: (N, T, V) log-probs, or (N, T) log-probs already gathered at
        ``target``."""
        T = pred.size(1)
        target = target[:, :T]
        mask = mask[:, :T].float()
        lp = pred if pred.dim() == 2 else pred.gather(2, target.unsqueeze(2)).squeeze(2)
        return -(lp * mask).sum() / mask.sum()


class RewardCriterion(nn.Module):
    def forward(self, seq, logprobs, reward):
        """seq, logprobs: (N, T).  reward: (N, T) as in the reference or (N,)
        (constant over time)."""
        mask = reward_mask(seq)
        if reward.dim() == 1:
            reward = reward[:, None]
        return -(logprobs * reward * mask).sum() / mask.sum()
