from .text import (EOS, BOS, UNK, array_to_str, sequence_tokens, decode_sequence,
                   compute_avglogp)
from .schedules import lr_at, adjust_learning_rate, ss_prob, mixer_from, scb_captions
from .timers import PhaseTimer

__all__ = ['EOS', 'BOS', 'UNK', 'array_to_str', 'sequence_tokens', 'decode_sequence',
           'compute_avglogp', 'lr_at', 'adjust_learning_rate', 'ss_prob', 'mixer_from',
           'scb_captions', 'PhaseTimer']
