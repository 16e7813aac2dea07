"""Reference-API surface for users switching from the reference scripts.

The reference exposes its pieces as flat modules (``dataloader.DataLoader``,
``utils.*``, ``model.*``).  This module gives the same call signatures on top
of the MI355X-native components, so reference-style driver code keeps
working:

* :class:`DataLoader` -- ``DataLoader(opt_dict)`` with the reference keys
  (``label_h5``, ``feat_h5``, ``batch_size``, ``seq_per_img``, ``num_chunks``,
  ``mode``, ``cocofmt_file``, ``bcmrscores_pkl``, ``eval_metric``) and every
  getter of ``/root/reference/dataloader.py:15-218`` (``close``,
  ``get_feat_size``, ``get_num_feats``, ``get_cocofmt_file`` included).  The
  split is HBM-resident (``data/dataset.py``); pass ``device='cuda'`` to get
  device tensors straight from ``get_batch``.
* ``score`` / ``load_gt_refs`` / ``compute_score`` / ``language_eval`` /
  ``get_self_critical_reward2`` -- ``/root/reference/utils.py:31-166`` (the
  last is dead code in the reference, kept for API completeness).
* Re-exports of the model, criteria, reward and text helpers under their
  reference names.
"""
import json

import numpy as np

from .data.dataset import CaptionLoader, VideoCaptionDataset
from .eval import load_gt_refs, language_eval as _language_eval
from .eval.metrics import Bleu, Meteor, Rouge
from .models import (CaptionModel, CrossEntropyCriterion, RewardCriterion, FeatPool,
                     FeatExpander, RNNUnit, MANet)
from .reward import CiderD, Cider, get_cst_reward, get_self_critical_reward
from .utils import adjust_learning_rate, array_to_str, decode_sequence, compute_avglogp

__all__ = ['DataLoader', 'score', 'load_gt_refs', 'compute_score', 'language_eval',
           'get_self_critical_reward', 'get_self_critical_reward2', 'get_cst_reward',
           'adjust_learning_rate', 'array_to_str', 'decode_sequence', 'compute_avglogp',
           'CaptionModel', 'CrossEntropyCriterion', 'RewardCriterion', 'FeatPool',
           'FeatExpander', 'RNNUnit', 'MANet', 'CiderD', 'Cider']


class DataLoader(CaptionLoader):
    """``DataLoader(opt)`` of ``/root/reference/dataloader.py:18-76``.

    ``opt`` is a dict; ``label_h5`` / ``feat_h5`` name label and feature files
    in the reference layout (h5 where h5py is installed, else ``.npz`` with the
    same dataset names, ``data/formats.py``).  ``opt['dataset']`` may instead
    hold a ready :class:`VideoCaptionDataset` (e.g. ``make_synthetic``).
    Extra keys: ``device`` (default ``'cpu'``), ``rank``/``world_size`` (DP
    sharding), ``seed``.
    """

    def __init__(self, opt):
        ds = opt.get('dataset')
        if ds is None:
            ds = VideoCaptionDataset.from_files(
                opt['label_h5'], list(opt['feat_h5']), num_chunks=opt.get('num_chunks', 1),
                bcmrscores_file=opt.get('bcmrscores_pkl'),
                eval_metric=opt.get('eval_metric', 'CIDEr'),
                cocofmt_file=opt.get('cocofmt_file'))
        elif opt.get('cocofmt_file'):
            ds.cocofmt_file = opt['cocofmt_file']
        super().__init__(ds, opt.get('batch_size', 128), opt.get('seq_per_img', 1),
                         mode=opt.get('mode', 'train'), device=opt.get('device', 'cpu'),
                         rank=opt.get('rank', 0), world_size=opt.get('world_size', 1),
                         seed=opt.get('seed', 123))
        self.word_embedding_size = opt.get('word_embedding_size', 512)
        self.num_chunks = ds.num_chunks
        self.bcmrscores_pkl = opt.get('bcmrscores_pkl')

    # getters the base loader does not carry (dataloader.py:78-81, 190-195, 217-218)
    def close(self):
        """Files are read once at construction; nothing stays open."""
        self.ds._device_cache.clear()

    def get_feat_size(self):
        return sum(self.ds.feat_dims)

    def get_num_feats(self):
        return len(self.ds.feat_dims)

    def get_cocofmt_file(self):
        return self.ds.cocofmt_file

    @property
    def vocab(self):
        return self.ds.vocab

    @property
    def num_videos(self):
        return self.ds.num_videos

    @property
    def seq_length(self):
        return self.ds.seq_length

    @property
    def feat_dims(self):
        return self.ds.feat_dims


def score(ref, hypo):
    """BLEU-1..4 / METEOR / ROUGE-L / CIDEr of ``hypo`` against ``ref``
    (both ``{id: [sentences]}``, already tokenized) -- ``utils.py:31-47``."""
    scorers = [(Bleu(4), ['Bleu_1', 'Bleu_2', 'Bleu_3', 'Bleu_4']), (Meteor(), 'METEOR'),
               (Rouge(), 'ROUGE_L'), (Cider(), 'CIDEr')]
    out = {}
    for scorer, method in scorers:
        s, _ = scorer.compute_score(ref, hypo)
        if isinstance(method, list):
            out.update(zip(method, s))
        else:
            out[method] = s
    return out


def compute_score(gt_refs, predictions, scorer):
    """Score ``[{'image_id', 'caption'}]`` with a CIDEr-style scorer
    (``compute_score(gts, res_list)``) -- ``utils.py:58-74``."""
    hypo = [{'image_id': p['image_id'], 'caption': [p['caption']]} for p in predictions]
    ref = {p['image_id']: gt_refs[p['image_id']] for p in predictions}
    return scorer.compute_score(ref, hypo)


def language_eval(gold_file, pred_file):
    """``utils.py:114-132``: ``pred_file`` is a JSON file of
    ``[{'image_id', 'caption'}]`` or that list itself."""
    if isinstance(pred_file, str):
        with open(pred_file) as f:
            pred_file = json.load(f)
    return _language_eval(gold_file, pred_file)


def get_self_critical_reward2(model_res, greedy_res, gt_refs, scorer):
    """Dead helper of ``utils.py:155-166``, reproduced as is: it passes its
    arguments to ``compute_score(gt_refs, predictions, scorer)`` swapped, so
    ``model_res`` / ``greedy_res`` fill the refs slot and ``gt_refs`` the
    predictions slot.  Returns the two mean scores."""
    _, model_scores = compute_score(model_res, gt_refs, scorer)
    _, greedy_scores = compute_score(greedy_res, gt_refs, scorer)
    return float(np.mean(model_scores)), float(np.mean(greedy_scores))
