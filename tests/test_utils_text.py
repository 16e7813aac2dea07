"""Token helpers and schedules (reference utils.py / train.py formulas)."""
import math

import numpy as np

from cst_captioning_amd.config import default_opts
from cst_captioning_amd.utils import (array_to_str, decode_sequence, compute_avglogp, lr_at,
                                      ss_prob, mixer_from, scb_captions)


def test_array_to_str_matches_reference_probe():
    # SURVEY.md §2.1 P20 [probe]: '5 6 7' / '5 6 7 0'
    arr = [1, 5, 6, 7, 0, 9, 9]
    assert array_to_str(arr, 0) == '5 6 7'
    assert array_to_str(arr, 1) == '5 6 7 0'
    assert array_to_str([0, 4], 0) == ''
    assert array_to_str([0, 4], 1) == '0'
    assert array_to_str([5, 1, 6], 0) == '5 6'  # BOS skipped anywhere
    assert array_to_str([5, 6, 7], 1) == '5 6 7'  # truncated: no EOS


def test_decode_sequence_and_avglogp():
    vocab = {0: '<end>', 1: '<start>', 2: '<unk>', 3: 'a', 4: 'dog'}
    seq = np.array([[3, 4, 0, 3], [4, 0, 0, 0]])
    assert decode_sequence(vocab, seq) == ['a dog', 'dog']
    lp = np.array([[-1.0, -2.0, -3.0, -9.0], [-4.0, -5.0, -9.0, -9.0]])
    assert compute_avglogp(seq, lp) == [-2.0, -4.5]


def test_schedules():
    o = default_opts(learning_rate=1e-3, lr_update=10)
    assert lr_at(o, 9) == 1e-3 and abs(lr_at(o, 25) - 1e-5) < 1e-12
    o = default_opts(use_ss=1, use_ss_after=2, ss_k=30.0, ss_max_prob=0.25)
    assert ss_prob(o, 1) == 0.0
    ep = 40
    ann = 30.0 / (30.0 + math.exp((ep - 2) / 30.0))
    assert abs(ss_prob(o, ep) - min(1 - ann, 0.25)) < 1e-12
    o = default_opts(mixer_from=-1, use_rl_after=3, mixer_descrease_every=2)
    assert mixer_from(o, 3, 30) == 29 and mixer_from(o, 4, 30) == 29
    assert mixer_from(o, 5, 30) == 28 and mixer_from(o, 200, 30) == 1
    o = default_opts(scb_captions=-1, use_cst_after=0, cst_increase_every=5)
    assert scb_captions(o, 0, 20) == 1 and scb_captions(o, 5, 20) == 2
    assert scb_captions(o, 1000, 20) == 19


def test_snowball_english_stemmer():
    """METEOR's stem stage (eval/stem.py): Snowball English (Porter2) stems of
    the algorithm's published examples and caption-style words."""
    from cst_captioning_amd.eval.stem import stem
    pairs = dict(consign='consign', consigned='consign', consigning='consign',
                 consignment='consign', consisted='consist', consistency='consist',
                 knackeries='knackeri', generously='generous', generation='generat',
                 running='run', happily='happili', caresses='caress', ponies='poni',
                 ties='tie', cried='cri', hoped='hope', hopping='hop', agreed='agre',
                 feed='feed', skies='sky', dying='die', gaps='gap', gas='gas', kiwis='kiwi',
                 luxuriated='luxuri', dancing='danc', riding='ride', people='peopl',
                 beautiful='beauti', relational='relat', conditional='condit',
                 sensibility='sensibl', fruitlessly='fruitless', hopefulness='hope',
                 communication='communic', arsenal='arsenal', news='news', controlled='control')
    assert {w: stem(w) for w in pairs} == pairs


def test_meteor_matches_stems():
    from cst_captioning_amd.eval.metrics import Meteor
    m = Meteor()
    exact = m._segment('a man is riding a horse'.split(), 'a man is riding a horse'.split())
    stemmed = m._segment('a man rides horses'.split(), 'a man riding a horse'.split())
    none = m._segment('a man rides horses'.split(), 'a woman cooks food'.split())
    assert exact > stemmed > none > 0


def test_meteor_corpus_score_aggregates_statistics():
    """The corpus METEOR is computed from the summed alignment statistics of
    each segment's best reference (Meteor 1.5 EVAL), so a long segment weighs
    more than a short one; it is not the mean of the segment scores.  (Parity
    with the jar itself is unpinned: no java here.)"""
    from cst_captioning_amd.eval.metrics import Meteor
    m = Meteor()
    gts = {0: ['a man is riding a horse on the beach near the sea'],
           1: ['a cat', 'a dog sleeps']}
    res = {0: ['a man is riding a horse on the beach near the sea'], 1: ['the bird']}
    corpus, seg = m.compute_score(gts, res)
    assert seg[0] > 0.5 and seg[1] == 0.0
    # mean of the segments would be ~0.5; the aggregate follows the matched words
    mean = float(seg.mean())
    assert corpus > mean + 0.1, (corpus, mean)
    st = [max((m._stats(res[k][0].split(), r.split()) for r in gts[k]), key=m._score)
          for k in res]
    tot = tuple(sum(x) for x in zip(*st))
    assert abs(corpus - m._score(tot)) < 1e-12
