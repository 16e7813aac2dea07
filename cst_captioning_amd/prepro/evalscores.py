"""P7: GT consensus scores ("bcmrscores").

``/root/reference/compute_scores.py:37-110``: for caption slot ``i`` of every
video (videos in sorted-id order), score that caption against the video's
references -- with ``remove_in_ref`` the caption itself is left out -- under
BLEU-4, METEOR, ROUGE-L and coco CIDEr.  Output ``{metric: (N, S)}``.

Improvement over the reference (README TODO): videos
with fewer than ``seq_per_img`` captions are supported by cycling their
captions (slot ``i`` uses caption ``i % ncap``), so MSVD-style data works.
Results are saved as ``.npz`` (no pickle needed to read them back); a
``.pkl`` path also gets the reference-format pickle.
"""
import argparse
import os
import pickle

import numpy as np

from ..eval import load_gt_refs
from ..eval.metrics import Bleu, Meteor, Rouge, ptb_tokenize
from ..reward.cider_d_cpu import Cider

METRICS = ('Bleu_4', 'METEOR', 'ROUGE_L', 'CIDEr')


def compute_consensus_scores(gt_refs, seq_per_img=20, remove_in_ref=True, tokenize=True,
                             metrics=METRICS):
    videos = sorted(gt_refs.keys())
    refs = {v: [ptb_tokenize(c) if tokenize else c for c in gt_refs[v]] for v in videos}
    out = {m: np.zeros((len(videos), seq_per_img)) for m in metrics}
    scorers = {'Bleu_4': Bleu(4), 'METEOR': Meteor(), 'ROUGE_L': Rouge(), 'CIDEr': Cider()}
    for i in range(seq_per_img):
        preds = {v: [refs[v][i % len(refs[v])]] for v in videos}
        if remove_in_ref:
            gts_i = {}
            for v in videos:
                j = i % len(refs[v])
                rest = refs[v][:j] + refs[v][j + 1:]
                gts_i[v] = rest if rest else refs[v]
        else:
            gts_i = refs
        for m in metrics:
            _, s = scorers[m].compute_score(gts_i, preds)
            if m == 'Bleu_4':
                s = s[-1]
            out[m][:, i] = np.asarray(s)
    return out


def save_scores(path, scores):
    npz = path[:-4] + '.npz' if path.endswith('.pkl') else path
    np.savez(npz, **scores)
    if path.endswith('.pkl'):
        with open(path, 'wb') as f:
            pickle.dump(scores, f, protocol=pickle.HIGHEST_PROTOCOL)
    return npz


def load_scores(path, metric='CIDEr'):
    """One metric's (N, S) matrix, read from the ``.npz`` written beside a
    ``.pkl`` (no unpickling).  A reference-written ``.pkl`` with no ``.npz``
    beside it goes through the restricted unpickler (arrays and containers
    only)."""
    npz = path[:-4] + '.npz' if path.endswith('.pkl') else path
    if path.endswith('.pkl') and not os.path.exists(npz):
        from ..utils.safe_pickle import safe_load
        z = safe_load(path)
        if metric == 'CIDEr' and metric not in z and 'cider' in z:
            metric = 'cider'
        return np.asarray(z[metric], dtype=np.float64)
    z = np.load(npz, allow_pickle=False)
    if metric == 'CIDEr' and metric not in z.files and 'cider' in z.files:
        metric = 'cider'  # dataloader.py:70-71
    return np.asarray(z[metric], dtype=np.float64)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('cocofmt_file')
    p.add_argument('output_pkl')
    p.add_argument('--seq_per_img', type=int, default=20)
    p.add_argument('--remove_in_ref', action='store_true')
    a = p.parse_args(argv)
    scores = compute_consensus_scores(load_gt_refs(a.cocofmt_file), a.seq_per_img,
                                      a.remove_in_ref)
    save_scores(a.output_pkl, scores)
    return scores


if __name__ == '__main__':
    main()
