"""Offline preprocessing (reference components P1-P7).

Each module has a ``main(argv)`` CLI with the reference script's positional
arguments; ``python -m cst_captioning_amd.prepro.<module> ...``.
"""
from .standalize import standalize_yt2t, standalize_msrvtt, standalize_tvvtt
from .tokenize import tokenize_caption, group_and_tokenize
from .vocab import build_vocab, SPECIALS, EOS_TOKEN, BOS_TOKEN, UNK_TOKEN
from .labels import build_label_store, encode_captions, final_captions
from .cocofmt import to_cocofmt
from .ciderdf import (pack_ngram, unpack_ngram_keys, df_from_token_refs, index_refs, save_df,
                      load_packed_df)
from .evalscores import compute_consensus_scores, save_scores, load_scores
