"""Evaluation: language metrics and the reference-style ``language_eval``."""
import json

from .metrics import Bleu, Rouge, Meteor, ptb_tokenize, evaluate_captions


def load_gt_refs(cocofmt_file):
    """{image_id: [captions]} from a coco-format file (``utils.py:50-55``)."""
    with open(cocofmt_file) as f:
        d = json.load(f)
    out = {}
    for a in d['annotations']:
        out.setdefault(a['image_id'], []).append(a['caption'])
    return out


def language_eval(gold, predictions):
    """Score ``[{'image_id', 'caption'}]`` against a coco-format file or a
    ``{image_id: [captions]}`` dict; returns metrics rounded to 5 places like
    ``/root/reference/utils.py:114-132``."""
    refs = load_gt_refs(gold) if isinstance(gold, str) else gold
    res = {p['image_id']: p['caption'] for p in predictions}
    gts = {k: refs[k] for k in res}
    return {k: round(v, 5) for k, v in evaluate_captions(gts, res).items()}


__all__ = ['Bleu', 'Rouge', 'Meteor', 'ptb_tokenize', 'evaluate_captions', 'load_gt_refs',
           'language_eval']
