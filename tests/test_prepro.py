"""Preprocessing pipeline P1-P7 end to end on a tiny
MSR-VTT-shaped raw file, through the same CLIs the Makefile drives.

Reference behaviour: ``standalize_format.py``, ``preprocess_datainfo.py``,
``build_vocab.py``, ``create_sequencelabel.py``, ``convert_datainfo2cocofmt.py``,
``compute_ciderdf.py``, ``compute_scores.py`` under ``/root/reference``.
"""
import json
import os

import numpy as np
import pytest

from cst_captioning_amd.data.formats import load_label_file
from cst_captioning_amd.prepro import (ciderdf, cocofmt, evalscores, labels, standalize,
                                       tokenize, vocab)
from cst_captioning_amd.prepro.ciderdf import load_packed_df, pack_ngram


def _raw_msrvtt(path):
    videos, sents = [], []
    sid = 0
    for i in range(6):
        split = 'train' if i < 4 else 'validate'
        videos.append({'video_id': 'video%d' % i, 'id': i, 'split': split, 'category': i % 3,
                       'url': '', 'start time': 0, 'end time': 1})
        for j in range(3 + i % 2):
            sents.append({'sen_id': sid, 'video_id': 'video%d' % i,
                          'caption': 'A man, is Cooking food %d!  café' % (j % 2)})
            sid += 1
    sents.append({'sen_id': sid, 'video_id': 'video0', 'caption': 'rare words appear here once'})
    with open(path, 'w') as f:
        json.dump({'info': {'year': 2016}, 'videos': videos, 'sentences': sents}, f)


def test_tokenizer():
    assert tokenize.tokenize_caption('A man, is Cooking! café') == ['a', 'man', 'is',
                                                                        'cooking', 'caf']


def test_vocab_specials_first():
    vids = [{'processed_tokens': [['b', 'a', 'b'], ['c']]}]
    v = vocab.build_vocab(vids, 2)
    assert v[:3] == ['<end>', '<start>', '<unk>'] and v[3:] == ['b']


def test_encode_truncates_and_maps_unk():
    wtoi = {w: i for i, w in enumerate(['<end>', '<start>', '<unk>', 'a', 'b'])}
    vids = [{'video_id': 7, 'captions': ['x'], 'processed_tokens': [['a', 'zz', 'b', 'a']]}]
    store = labels.build_label_store(list(wtoi), vids, 4)
    # <start> a <unk> b  (truncated: the <end> is lost, like the reference)
    assert store['labels'].tolist() == [[1, 3, 2, 4]]
    assert store['label_length'].tolist() == [4]
    store6 = labels.build_label_store(list(wtoi), vids, 7)
    assert store6['labels'].tolist() == [[1, 3, 2, 4, 3, 0, 0]]


def test_pipeline_cli(tmp_path):
    d = str(tmp_path)
    raw = os.path.join(d, 'raw.json')
    _raw_msrvtt(raw)
    info = os.path.join(d, 'msrvtt_train_datainfo.json')
    standalize.main([raw, info, '--dataset', 'msrvtt2016', '--split', 'train'])
    di = json.load(open(info))
    assert [v['id'] for v in di['videos']] == [0, 1, 2, 3]
    assert all(c['video_id'] in (0, 1, 2, 3) for c in di['captions'])

    toks = os.path.join(d, 'msrvtt_train_proprocessedtokens.json')
    tokenize.main([info, toks])
    tv = json.load(open(toks))
    assert tv[0]['processed_tokens'][0] == ['a', 'man', 'is', 'cooking', 'food', '0', 'caf']

    vj = os.path.join(d, 'msrvtt_train_vocab.json')
    voc = vocab.main([toks, vj, '--word_count_threshold', '3'])
    assert 'rare' not in voc and 'cooking' in voc

    lab = os.path.join(d, 'msrvtt_train_sequencelabel.npz')
    labels.main([vj, toks, lab, '--max_length', '10'])
    st = load_label_file(lab)
    assert st['vocab'] == voc
    assert st['labels'].shape[1] == 10 and (st['labels'][:, 0] == 1).all()
    ncaps = st['label_end_ix'] - st['label_start_ix']
    assert ncaps.tolist() == [4, 4, 3, 4]
    assert (st['label_to_video'][st['label_start_ix']] == np.arange(4)).all()
    # the rare-word caption of video 0 maps OOV words to <unk>=2
    assert (st['labels'][st['label_start_ix'][0]:st['label_end_ix'][0]] == 2).any()

    coco = os.path.join(d, 'msrvtt_train_cocofmt.json')
    cocofmt.main([info, coco])
    cj = json.load(open(coco))
    assert len(cj['annotations']) == len(di['captions'])
    assert all(ord(ch) < 128 for a in cj['annotations'] for ch in a['caption'])

    dfp = os.path.join(d, 'msrvtt_train_ciderdf.pkl')
    ciderdf.main([toks, dfp, '--vocab_json', vj])
    keys, vals, ref_len = load_packed_df(dfp)
    assert ref_len == 4
    df = dict(zip(keys.tolist(), vals.tolist()))
    wtoi = {w: i for i, w in enumerate(voc)}
    # 'a man' appears in every train video; EOS-terminated n-grams are counted,
    # BOS-prefixed ones are not (compute_ciderdf.py:115-116)
    assert df[pack_ngram((wtoi['a'], wtoi['man']))] == 4
    assert df[pack_ngram((wtoi['caf'], 0))] == 4
    assert pack_ngram((1, wtoi['a'])) not in df

    sc = os.path.join(d, 'msrvtt_train_evalscores.pkl')
    evalscores.main([coco, sc, '--seq_per_img', '5'])
    cider = evalscores.load_scores(sc, 'CIDEr')
    assert cider.shape == (4, 5) and np.isfinite(cider).all()
    b4 = evalscores.load_scores(sc, 'Bleu_4')
    assert b4.shape == (4, 5)


def test_consensus_cycles_short_videos():
    refs = {0: ['a b c', 'a b d'], 1: ['x y z', 'x y z', 'x y w']}
    s = evalscores.compute_consensus_scores(refs, 4, True, tokenize=False,
                                            metrics=('CIDEr', 'ROUGE_L'))
    assert s['CIDEr'].shape == (2, 4)
    # slot i uses caption i % ncap: video 0 slots 0/2 and 1/3 coincide
    np.testing.assert_allclose(s['ROUGE_L'][0, 0], s['ROUGE_L'][0, 2])
    np.testing.assert_allclose(s['ROUGE_L'][0, 1], s['ROUGE_L'][0, 3])


@pytest.mark.parametrize('use_txt', [True])
def test_yt2t(tmp_path, use_txt):
    p = tmp_path / 'yt.txt'
    p.write_text('vid1\ta dog runs\nvid1\ta dog is running\nvid12\ta cat\n')
    out = standalize.standalize_yt2t(str(p))
    assert [v['id'] for v in out['videos']] == [1, 12]
    assert [c['video_id'] for c in out['captions']] == [1, 1, 12]
