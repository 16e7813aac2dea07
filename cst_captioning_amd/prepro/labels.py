"""P4: encode captions as fixed-length label rows.

``/root/reference/create_sequencelabel.py:21-105``: each caption becomes
``<start> w... <end>`` with out-of-vocabulary words mapped to ``<unk>``,
truncated to ``max_length`` (so a long caption can lose its ``<end>``),
zero padded (0 = ``<end>``).  The label store holds ``labels (M, L)``,
``label_start_ix / label_end_ix (N)``, ``label_length / label_to_video (M)``,
``videos (N)`` and ``vocab (V)``.

Files are written with :func:`..data.formats.save_label_file`: ``.h5`` when
h5py is importable (reference format), otherwise ``.npz`` with the same
dataset names.  ``np.string_`` (removed in NumPy 2) is not used.
"""
import argparse
import json

import numpy as np

from .vocab import BOS_TOKEN, EOS_TOKEN, UNK_TOKEN


def final_captions(tokens_list, wtoi, with_bos=True):
    out = []
    for toks in tokens_list:
        cap = [BOS_TOKEN] if with_bos else []
        cap += [w if w in wtoi else UNK_TOKEN for w in toks]
        cap.append(EOS_TOKEN)
        out.append(cap)
    return out


def encode_captions(videos, max_length, wtoi):
    n = len(videos)
    m = sum(len(v['final_captions']) for v in videos)
    labels = np.zeros((m, max_length), dtype=np.int64)
    start = np.zeros(n, dtype=np.int64)
    end = np.zeros(n, dtype=np.int64)
    length = np.zeros(m, dtype=np.int64)
    to_video = np.zeros(m, dtype=np.int64)
    row = 0
    for i, v in enumerate(videos):
        caps = v['final_captions']
        if not caps:
            raise ValueError('video %r has no captions' % v.get('video_id'))
        start[i] = row
        for cap in caps:
            ids = [wtoi[w] for w in cap[:max_length]]
            labels[row, :len(ids)] = ids
            length[row] = min(max_length, len(cap))
            to_video[row] = i
            row += 1
        end[i] = row
    return labels, start, end, length, to_video


def build_label_store(vocab, videos, max_length):
    wtoi = {w: i for i, w in enumerate(vocab)}
    for v in videos:
        v['final_captions'] = final_captions(v['processed_tokens'], wtoi)
    store = {'videos': np.array([str(v['video_id']) for v in videos]),
             'vocab': np.array(vocab)}
    if videos and len(videos[0]['captions']) > 0:
        lab, s, e, ln, tv = encode_captions(videos, max_length, wtoi)
        store.update(labels=lab, label_start_ix=s, label_end_ix=e, label_length=ln,
                     label_to_video=tv)
    return store


def main(argv=None):
    from ..data.formats import save_label_file
    p = argparse.ArgumentParser()
    p.add_argument('vocab_json')
    p.add_argument('captions_json')
    p.add_argument('output_file')
    p.add_argument('--max_length', type=int, default=30)
    a = p.parse_args(argv)
    with open(a.vocab_json) as f:
        vocab = json.load(f)
    with open(a.captions_json) as f:
        videos = json.load(f)
    store = build_label_store(vocab, videos, a.max_length)
    return save_label_file(a.output_file, store)


if __name__ == '__main__':
    main()
