"""Language metrics: BLEU-1..4, METEOR, ROUGE-L, CIDEr.

The reference evaluates with the external coco-caption package
(``/root/reference/utils.py:114-132``: ``COCOEvalCap``; scorers
``pycocoevalcap.{bleu,meteor,rouge,cider}``), which needs Java for the PTB
tokenizer and for METEOR.  Neither Java nor the package exists in this
image, so this module re-implements the metrics from their definitions:

  * BLEU   -- corpus BLEU with "closest" reference length and the
              per-sentence scores coco reports (tiny=1e-15, small=1e-9);
  * ROUGE-L-- LCS F-measure, beta = 1.2, max precision/recall over refs;
  * CIDEr  -- coco CIDEr (corpus df, no clipping/penalty), via
              :mod:`..reward.cider_d_cpu`;
  * METEOR -- exact + stem matching (the Snowball English / Porter2
              stemmer METEOR 1.5 uses, :mod:`.stem`) with the METEOR 1.5
              English parameters (alpha .85, beta .2, gamma .6; stem weight .6).
              WordNet synonyms/paraphrases are not available, so this is an
              approximation (parity unpinned); if ``java`` and a METEOR jar
              are found (``METEOR_JAR`` env var) the real scorer is used.

Tokenisation approximates the PTB tokenizer + coco punctuation removal.
"""
import logging
import math
import os
import re
import shutil
import subprocess
from collections import Counter

import numpy as np

from ..reward.cider_d_cpu import Cider
from .stem import stem

_PUNCT = {"''", "'", "``", "`", "-lrb-", "-rrb-", "-lcb-", "-rcb-", ".", "?", "!", ",",
          ":", "-", "--", "...", ";"}
_TOKEN_RE = re.compile(r"\.\.\.|--|``|''|[A-Za-z0-9]+(?:'[A-Za-z]+)?|'[A-Za-z]+|[^\sA-Za-z0-9]")


def ptb_tokenize(sentence):
    toks = _TOKEN_RE.findall(sentence.lower())
    return ' '.join(t for t in toks if t not in _PUNCT)


def _ngrams(words, n):
    c = Counter()
    for k in range(1, n + 1):
        for i in range(len(words) - k + 1):
            c[tuple(words[i:i + k])] += 1
    return c


class Bleu:
    def __init__(self, n=4):
        self.n = n

    def compute_score(self, gts, res):
        n = self.n
        tiny, small = 1e-15, 1e-9
        per = [[] for _ in range(n)]
        tot_guess, tot_correct = [0] * n, [0] * n
        tot_test = tot_ref = 0
        for key in res:
            hyp = res[key][0].split()
            refs = [r.split() for r in gts[key]]
            maxc = Counter()
            for r in refs:
                for g, c in _ngrams(r, n).items():
                    maxc[g] = max(maxc[g], c)
            tlen = len(hyp)
            rlen = min((abs(len(r) - tlen), len(r)) for r in refs)[1]
            hc = _ngrams(hyp, n)
            guess = [max(0, tlen - k) for k in range(n)]
            correct = [0] * n
            for g, c in hc.items():
                correct[len(g) - 1] += min(c, maxc.get(g, 0))
            tot_test += tlen
            tot_ref += rlen
            b = 1.0
            for k in range(n):
                tot_guess[k] += guess[k]
                tot_correct[k] += correct[k]
                b *= (correct[k] + tiny) / (guess[k] + small)
                per[k].append(b ** (1.0 / (k + 1)))
            ratio = (tlen + tiny) / (rlen + small)
            if ratio < 1:
                for k in range(n):
                    per[k][-1] *= math.exp(1 - 1 / ratio)
        bleus = []
        b = 1.0
        for k in range(n):
            b *= (tot_correct[k] + tiny) / (tot_guess[k] + small)
            bleus.append(b ** (1.0 / (k + 1)))
        ratio = (tot_test + tiny) / (tot_ref + small)
        if ratio < 1:
            bleus = [x * math.exp(1 - 1 / ratio) for x in bleus]
        return bleus, per


def _lcs(a, b):
    if len(a) < len(b):
        a, b = b, a
    prev = [0] * (len(b) + 1)
    for x in a:
        cur = [0] * (len(b) + 1)
        for j, y in enumerate(b):
            cur[j + 1] = prev[j] + 1 if x == y else max(prev[j + 1], cur[j])
        prev = cur
    return prev[-1]


class Rouge:
    beta = 1.2

    def calc_score(self, cand, refs):
        c = cand.split()
        precs, recs = [], []
        for r in refs:
            rt = r.split()
            l = _lcs(rt, c)
            precs.append(l / float(len(c)) if c else 0.0)
            recs.append(l / float(len(rt)) if rt else 0.0)
        p, r = max(precs), max(recs)
        if p != 0 and r != 0:
            b2 = self.beta ** 2
            return ((1 + b2) * p * r) / float(r + b2 * p)
        return 0.0

    def compute_score(self, gts, res):
        scores = np.array([self.calc_score(res[k][0], gts[k]) for k in res])
        return float(np.mean(scores)), scores




_METEOR_WARNED = False


class Meteor:
    alpha, beta, gamma = 0.85, 0.2, 0.6
    w_exact, w_stem = 1.0, 0.6

    def __init__(self):
        jar = os.environ.get('METEOR_JAR')
        self.java = bool(jar and os.path.isfile(jar) and shutil.which('java'))
        self.jar = jar
        global _METEOR_WARNED
        if not self.java and not _METEOR_WARNED:
            _METEOR_WARNED = True
            logging.getLogger(__name__).warning(
                'METEOR: java or $METEOR_JAR missing -- using the native approximation '
                '(parity with coco-caption METEOR unpinned)')

    def _align(self, h, r):
        used = [False] * len(r)
        pairs = []
        for stage, key in ((self.w_exact, lambda w: w), (self.w_stem, stem)):
            for i, w in enumerate(h):
                if any(p[0] == i for p in pairs):
                    continue
                kw = key(w)
                cands = [j for j in range(len(r)) if not used[j] and key(r[j]) == kw]
                if not cands:
                    continue
                prev = max((p for p in pairs if p[0] < i), default=None)
                want = prev[1] + 1 if prev else 0
                j = min(cands, key=lambda j: (abs(j - want), j))
                used[j] = True
                pairs.append((i, j, stage))
        return sorted(pairs)

    def _stats(self, h, r):
        """Sufficient statistics of one (hypothesis, reference) alignment:
        (weighted matches, hypothesis words, reference words, chunks, matched
        pairs) -- what the jar's SCORE line hands to its EVAL aggregate."""
        pairs = self._align(h, r) if h and r else []
        m = sum(p[2] for p in pairs)
        chunks = 0
        if pairs:
            chunks = 1
            for a, b in zip(pairs[:-1], pairs[1:]):
                if not (b[0] == a[0] + 1 and b[1] == a[1] + 1):
                    chunks += 1
        return (m, len(h), len(r), chunks, len(pairs))

    def _score(self, st):
        m, lh, lr, chunks, npairs = st
        if m <= 0 or lh <= 0 or lr <= 0:
            return 0.0
        P, R = m / lh, m / lr
        fmean = P * R / (self.alpha * P + (1 - self.alpha) * R)
        frag = chunks / float(npairs)
        pen = self.gamma * frag ** self.beta
        return (1 - pen) * fmean

    def _segment(self, h, r):
        return self._score(self._stats(h, r))

    def compute_score(self, gts, res):
        """(corpus score, per-segment scores).  Per segment the best reference
        is kept; the corpus score is computed from the summed statistics of
        those alignments, as Meteor 1.5's EVAL command aggregates them
        (coco-caption reports that number, /root/reference/utils.py:114-132),
        not the mean of the segment scores."""
        if self.java:
            return self._java_score(gts, res)
        seg, tot = [], [0, 0, 0, 0, 0]
        for k in res:
            h = res[k][0].split()
            best = max((self._stats(h, r.split()) for r in gts[k]), key=self._score)
            seg.append(self._score(best))
            tot = [a + b for a, b in zip(tot, best)]
        return self._score(tuple(tot)), np.array(seg)

    def _java_score(self, gts, res):  # pragma: no cover - needs java + jar
        proc = subprocess.Popen(['java', '-jar', '-Xmx2G', self.jar, '-', '-', '-stdio', '-l',
                                 'en', '-norm'], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                universal_newlines=True)
        lines = []
        for k in res:
            proc.stdin.write('SCORE ||| %s ||| %s\n' % (' ||| '.join(gts[k]), res[k][0]))
            proc.stdin.flush()
            lines.append(proc.stdout.readline().strip())
        proc.stdin.write('EVAL ||| %s\n' % ' ||| '.join(lines))
        proc.stdin.flush()
        scores = [float(proc.stdout.readline().strip()) for _ in lines]
        total = float(proc.stdout.readline().strip())
        proc.stdin.close()
        proc.wait()
        return total, np.array(scores)


def evaluate_captions(gts_raw, res_raw):
    """COCOEvalCap equivalent: tokenize, then BLEU/METEOR/ROUGE_L/CIDEr.

    ``gts_raw``: {id: [raw ref captions]}, ``res_raw``: {id: raw caption}.
    """
    gts = {k: [ptb_tokenize(c) for c in v] for k, v in gts_raw.items()}
    res = {k: [ptb_tokenize(v)] for k, v in res_raw.items()}
    out = {}
    bleus, _ = Bleu(4).compute_score(gts, res)
    for i, b in enumerate(bleus):
        out['Bleu_%d' % (i + 1)] = b
    out['METEOR'] = Meteor().compute_score(gts, res)[0]
    out['ROUGE_L'] = Rouge().compute_score(gts, res)[0]
    out['CIDEr'] = Cider().compute_score(gts, res)[0]
    return out
