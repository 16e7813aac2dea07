"""P6: CIDEr-D document frequencies over token-index n-grams.

``/root/reference/compute_ciderdf.py:56-140``: every reference caption is
turned into its token **index** string (``'<unk>'``-mapped words followed by
``<end>``; the ``<start>`` the reference builds is overwritten at
``compute_ciderdf.py:115-116``, so BOS never appears), n-grams n<=4 are
counted once per video, and ``ref_len`` is the number of videos.

Besides the reference pickle (tuple-of-string keys) this writes an ``.npz``
with the n-grams packed into uint64 keys -- the form the on-GPU CIDEr-D
hash table consumes: token ``t`` of an n-gram occupies bits ``16*i`` as
``t + 1`` (so 0 marks an unused slot and the key is exact, collision-free,
for vocabularies up to 65534 words).
"""
import argparse
import json
import pickle
from collections import defaultdict

import numpy as np

from .vocab import EOS_TOKEN, UNK_TOKEN, build_vocab

MAX_VOCAB_FOR_PACKING = 65534


def pack_ngram(tokens):
    key = 0
    for i, t in enumerate(tokens):
        t = int(t)
        if not 0 <= t < MAX_VOCAB_FOR_PACKING:
            raise ValueError('token id %d cannot be packed' % t)
        key |= (t + 1) << (16 * i)
    return key


def unpack_ngram_keys(keys):
    out = []
    for k in np.asarray(keys, dtype=np.uint64).tolist():
        toks = []
        while k:
            toks.append(str((k & 0xFFFF) - 1))
            k >>= 16
        out.append(tuple(toks))
    return out


def ngram_set(token_ids, n=4):
    s = set()
    for k in range(1, n + 1):
        for i in range(len(token_ids) - k + 1):
            s.add(tuple(token_ids[i:i + k]))
    return s


def df_from_token_refs(refs_per_video, n=4):
    """refs_per_video: list (videos) of lists (captions) of int id lists.
    Returns ({packed_key: df}, ref_len)."""
    df = defaultdict(float)
    for refs in refs_per_video:
        seen = set()
        for r in refs:
            seen |= ngram_set(list(r), n)
        for g in seen:
            df[pack_ngram(g)] += 1.0
    return dict(df), len(refs_per_video)


def index_refs(videos, wtoi):
    """Index captions the way compute_ciderdf.py does (no BOS, + EOS)."""
    eos = wtoi[EOS_TOKEN]
    unk = wtoi[UNK_TOKEN]
    return [[[wtoi.get(w, unk) for w in toks] + [eos] for toks in v['processed_tokens']]
            for v in videos]


def save_df(path_pkl, packed_df, ref_len, write_pickle=True):
    keys = np.fromiter(packed_df.keys(), dtype=np.uint64, count=len(packed_df))
    vals = np.fromiter(packed_df.values(), dtype=np.float32, count=len(packed_df))
    npz = path_pkl[:-4] + '.npz' if path_pkl.endswith('.pkl') else path_pkl + '.npz'
    np.savez(npz, keys=keys, values=vals, ref_len=np.int64(ref_len))
    if write_pickle:
        tuple_df = defaultdict(float)
        for k, v in zip(unpack_ngram_keys(keys), vals.tolist()):
            tuple_df[k] = v
        with open(path_pkl, 'wb') as f:
            pickle.dump({'document_frequency': tuple_df, 'ref_len': ref_len}, f,
                        protocol=pickle.HIGHEST_PROTOCOL)
    return npz


def load_packed_df(path):
    """(keys uint64, values float32, ref_len) from a df file.

    ``.npz`` is read without pickle.  A reference-format ``.pkl`` goes
    through the restricted unpickler (plain containers and numbers only)."""
    if path.endswith('.pkl'):
        npz = path[:-4] + '.npz'
        try:
            z = np.load(npz, allow_pickle=False)
            return z['keys'], z['values'], int(z['ref_len'])
        except FileNotFoundError:
            from ..utils.safe_pickle import safe_load
            d = safe_load(path)
            keys = np.array([pack_ngram([int(t) for t in g]) for g in d['document_frequency']],
                            dtype=np.uint64)
            vals = np.array(list(d['document_frequency'].values()), dtype=np.float32)
            return keys, vals, int(d['ref_len'])
    z = np.load(path, allow_pickle=False)
    return z['keys'], z['values'], int(z['ref_len'])


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('captions_json')
    p.add_argument('output_pkl')
    p.add_argument('--output_words', action='store_true')
    p.add_argument('--vocab_json', default=None)
    a = p.parse_args(argv)
    with open(a.captions_json) as f:
        videos = json.load(f)
    if a.vocab_json:
        with open(a.vocab_json) as f:
            vocab = json.load(f)
    else:
        vocab = build_vocab(videos, 0)
    wtoi = {w: i for i, w in enumerate(vocab)}
    packed, ref_len = df_from_token_refs(index_refs(videos, wtoi))
    save_df(a.output_pkl, packed, ref_len)
    if a.output_words:
        from ..reward.cider_d_cpu import document_frequency
        words = [[' '.join([w if w in wtoi else UNK_TOKEN for w in t] + [EOS_TOKEN])
                  for t in v['processed_tokens']] for v in videos]
        with open(a.output_pkl.replace('.pkl', '_words.pkl', 1), 'wb') as f:
            pickle.dump({'document_frequency': document_frequency(words), 'ref_len': ref_len},
                        f, protocol=pickle.HIGHEST_PROTOCOL)
    return packed, ref_len


if __name__ == '__main__':
    main()
