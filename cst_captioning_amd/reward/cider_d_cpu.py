"""CPU CIDEr / CIDEr-D scorer (fp64 oracle).

The reference calls the external ``pyciderevalcap.ciderD.ciderD.CiderD``
(``/root/reference/train.py:121``, ``utils.py:194-198,260-264``) and coco
``Cider`` (``compute_scores.py:68``).  Neither package is vendored or
installable here, so this module implements the published CIDEr-D
definition (Vedantam et al. 2015, as in the ruotianluo/cider package;
spec restated in SURVEY.md §2.2):

  * n-grams n = 1..4 over whitespace tokens, counted per sentence;
  * ``vec[n][g] = tf(g) * (log(ref_len) - log(max(1, df(g))))``;
  * ``norm[n] = ||vec[n]||_2``; the "length" is the number of **bigram**
    occurrences (a quirk of the upstream code, kept);
  * per ref: ``val[n] = sum_g min(vh, vr) * vr / (|vh| |vr|)`` times the
    Gaussian length penalty ``exp(-(lh - lr)^2 / (2 sigma^2))``, sigma = 6;
  * score = 10 * mean_n(sum_refs val[n]) / n_refs.

``CiderD`` (df from a file, clipping + penalty) and ``Cider`` (corpus df,
no clipping, no penalty) share the machinery.  Parity with the real package
is "parity unpinned" (the package is not available in this image); the GPU
kernel is tested against this oracle.
"""
import math
from collections import defaultdict

import numpy as np

from ..utils.safe_pickle import safe_load

NGRAM_N = 4
SIGMA = 6.0


def precook(sentence, n=NGRAM_N):
    """n-gram counts of a whitespace-tokenised sentence: {tuple: count}."""
    words = sentence.split()
    counts = defaultdict(int)
    for k in range(1, n + 1):
        for i in range(len(words) - k + 1):
            counts[tuple(words[i:i + k])] += 1
    return counts


def document_frequency(refs_per_item):
    """df over items: the number of items whose refs contain the n-gram."""
    df = defaultdict(float)
    for refs in refs_per_item:
        seen = set()
        for ref in refs:
            seen.update(precook(ref).keys())
        for g in seen:
            df[g] += 1
    return df


class _CiderBase:
    clipped = True

    def __init__(self, n=NGRAM_N, sigma=SIGMA):
        self.n = n
        self.sigma = sigma
        self.document_frequency = None
        self.log_ref_len = None

    def _vec(self, counts):
        vec = [dict() for _ in range(self.n)]
        norm = [0.0] * self.n
        length = 0
        df = self.document_frequency
        for g, tf in counts.items():
            k = len(g) - 1
            d = df.get(g, 0.0)
            v = float(tf) * (self.log_ref_len - math.log(max(1.0, d)))
            vec[k][g] = v
            norm[k] += v * v
            if k == 1:
                length += tf
        return vec, [math.sqrt(x) for x in norm], length

    def _sim(self, vh, nh, lh, vr, nr, lr):
        delta = float(lh - lr)
        val = np.zeros(self.n)
        for k in range(self.n):
            ref = vr[k]
            acc = 0.0
            for g, x in vh[k].items():
                y = ref.get(g, 0.0)
                acc += (min(x, y) if self.clipped else x) * y
            if nh[k] != 0 and nr[k] != 0:
                acc /= (nh[k] * nr[k])
            if self.clipped:
                acc *= math.exp(-(delta ** 2) / (2 * self.sigma ** 2))
            val[k] = acc
        return val

    def score_one(self, hyp, refs):
        vh, nh, lh = self._vec(precook(hyp, self.n))
        total = np.zeros(self.n)
        for r in refs:
            vr, nr, lr = self._vec(precook(r, self.n))
            total += self._sim(vh, nh, lh, vr, nr, lr)
        s = float(np.mean(total)) / len(refs)
        return s * 10.0

    def _prepare_df(self, gts, keys):
        pass

    def compute_score(self, gts, res):
        """Reference calling convention.

        ``gts``: {id: [ref strings]}.  ``res``: a list of
        ``{'image_id': id, 'caption': [hyp]}`` (CiderD) or a dict
        {id: [hyp]} (coco Cider).  Returns ``(mean, ndarray of scores)``.
        """
        if isinstance(res, dict):
            items = [(k, res[k][0]) for k in res]
        else:
            items = [(r['image_id'], r['caption'][0]) for r in res]
        self._prepare_df(gts, [k for k, _ in items])
        scores = np.array([self.score_one(h, gts[k]) for k, h in items])
        return float(np.mean(scores)) if len(scores) else 0.0, scores


class CiderD(_CiderBase):
    """CIDEr-D with document frequencies loaded from a precomputed table.

    ``df`` may be a path to the reference's ``*_ciderdf.pkl``
    (``compute_ciderdf.py:123-129``: {'document_frequency', 'ref_len'}), a
    dict of that shape, or the string 'corpus' (df from the refs being
    scored, as coco does).
    """
    clipped = True

    def __init__(self, df='corpus', n=NGRAM_N, sigma=SIGMA):
        super().__init__(n, sigma)
        self.df_mode = 'corpus'
        if isinstance(df, dict):
            self._load(df)
        elif df != 'corpus':
            self._load(load_df_file(df))

    def _load(self, d):
        self.df_mode = 'file'
        self.document_frequency = dict(d['document_frequency'])
        self.log_ref_len = math.log(float(d['ref_len']))

    def _prepare_df(self, gts, keys):
        if self.df_mode == 'corpus':
            # one ref set per scored item, as the upstream scorer accumulates them
            self.document_frequency = dict(document_frequency([gts[k] for k in keys]))
            self.log_ref_len = math.log(float(len(keys)))


class Cider(_CiderBase):
    """coco-caption CIDEr: corpus df, no clipping, no length penalty."""
    clipped = False

    def _prepare_df(self, gts, keys):
        self.document_frequency = dict(document_frequency([gts[k] for k in keys]))
        self.log_ref_len = math.log(float(len(keys)))


def load_df_file(path):
    """Load a df table.

    ``.npz`` (written by this framework: keys/values arrays) is read with
    ``allow_pickle=False``.  A reference-format ``.pkl`` (tuples of strings
    -> floats) goes through the restricted unpickler, which resolves no
    globals beyond plain containers and numbers.
    """
    if str(path).endswith('.npz'):
        z = np.load(path, allow_pickle=False)
        from ..prepro.ciderdf import unpack_ngram_keys
        keys = unpack_ngram_keys(z['keys'])
        return {'document_frequency': dict(zip(keys, z['values'].tolist())),
                'ref_len': int(z['ref_len'])}
    return safe_load(path)
