"""Token-sequence helpers.

Semantics follow the reference helpers:
  * ``array_to_str``     -- ``/root/reference/utils.py:135-152``
  * ``decode_sequence``  -- ``/root/reference/utils.py:78-95``
  * ``compute_avglogp``  -- ``/root/reference/utils.py:99-111``

Token conventions (``build_vocab.py:41-42``): ``<end>`` = 0 (EOS and padding),
``<start>`` = 1 (BOS), ``<unk>`` = 2.
"""
import numpy as np

EOS = 0
BOS = 1
UNK = 2


def sequence_tokens(arr, use_eos=0):
    """The token ids that the reward string of ``arr`` contains.

    BOS is skipped; scanning stops at the first EOS, which is kept when
    ``use_eos`` is set (so a sample is rewarded for emitting its first EOS).
    """
    out = []
    for x in arr:
        x = int(x)
        if x == EOS:
            if use_eos:
                out.append(EOS)
            break
        if x == BOS:
            continue
        out.append(x)
    return out


def array_to_str(arr, use_eos=0):
    """Index string used as CIDEr-D input, e.g. ``[5,6,7,0,9] -> '5 6 7'``
    (``'5 6 7 0'`` with ``use_eos=1``)."""
    return ' '.join(str(x) for x in sequence_tokens(arr, use_eos))


def decode_sequence(ix_to_word, seq):
    """Map an ``N x D`` id matrix to sentences, stopping at the first EOS."""
    seq = np.asarray(seq)
    out = []
    for row in seq:
        words = []
        for ix in row:
            ix = int(ix)
            if ix <= 0:
                break
            w = ix_to_word[ix] if ix in ix_to_word else ix_to_word[str(ix)]
            words.append(w.decode() if isinstance(w, bytes) else w)
        out.append(' '.join(words))
    return out


def compute_avglogp(seq, logseq, eos_token=EOS):
    """Mean log-prob of each row up to and including its first EOS."""
    seq = np.asarray(seq)
    logseq = np.asarray(logseq)
    out = []
    for i in range(seq.shape[0]):
        vals = []
        for j in range(seq.shape[1]):
            vals.append(float(logseq[i, j]))
            if int(seq[i, j]) == eos_token:
                break
        out.append(sum(vals) / len(vals) if vals else 0)
    return out
