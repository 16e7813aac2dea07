from .caption_model import CaptionModel
from .criteria import CrossEntropyCriterion, RewardCriterion, reward_mask
from .modules import FeatPool, FeatExpander, RNNUnit, MANet, TemporalAttention

__all__ = ['CaptionModel', 'CrossEntropyCriterion', 'RewardCriterion', 'reward_mask',
           'FeatPool', 'FeatExpander', 'RNNUnit', 'MANet', 'TemporalAttention']
