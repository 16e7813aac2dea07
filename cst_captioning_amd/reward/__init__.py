from .cider_d_cpu import CiderD, Cider, precook, document_frequency, load_df_file
from .rewards import (cst_from_scores, scst_from_scores, score_hypotheses, get_cst_reward,
                      get_self_critical_reward)

__all__ = ['CiderD', 'Cider', 'precook', 'document_frequency', 'load_df_file',
           'cst_from_scores', 'scst_from_scores', 'score_hypotheses', 'get_cst_reward',
           'get_self_critical_reward']
