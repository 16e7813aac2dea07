"""GT consensus scores ("bcmrscores", prepro/evalscores.py: coco CIDEr of
each GT caption against the video's other captions, remove_in_ref) of the
bench's synthetic MSR-VTT dataset (seed 123, 6,513 videos x 20 captions,
V = 10,509), computed once on the CPU and cached as .npz for bench.py's
CST_MS_SCB field (the reference reads them from a file too,
/root/reference/dataloader.py:62-71)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from cst_captioning_amd.data import make_synthetic
from cst_captioning_amd.prepro.evalscores import compute_consensus_scores


def main(out, seed=123, videos=6513, vocab=10509):
    t = time.time()
    ds = make_synthetic('msrvtt', num_videos=videos, vocab_size=vocab, seed=seed)
    s = compute_consensus_scores(ds.gt_refs, 20, True, tokenize=False, metrics=('CIDEr',))['CIDEr']
    np.savez_compressed(out, CIDEr=s.astype(np.float32), seed=seed, videos=videos, vocab=vocab)
    print('bcmr', s.shape, 'mean %.4f' % s.mean(), '%.1f s' % (time.time() - t))


if __name__ == '__main__':
    main(sys.argv[1])
