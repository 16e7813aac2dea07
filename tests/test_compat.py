"""Reference-API facade (``cst_captioning_amd.compat``): ``DataLoader(opt)``
over label/feature files with the reference getters
(``/root/reference/dataloader.py:15-218``), and the ``utils.py`` scorer
helpers (``score``, ``compute_score``, ``language_eval`` from a file,
``get_self_critical_reward2``)."""
import json

import numpy as np
import torch

from cst_captioning_amd import compat
from cst_captioning_amd.data.formats import save_feature_file, save_label_file
from cst_captioning_amd.data.synthetic import make_synthetic
from cst_captioning_amd.prepro.labels import build_label_store


def _files(tmp_path, ncaps=(2, 3, 25)):
    vocab = ['<end>', '<start>', '<unk>'] + ['w%d' % i for i in range(10)]
    videos = []
    for i, n in enumerate(ncaps):
        toks = [['w%d' % ((i + j) % 10)] * (1 + j % 3) for j in range(n)]
        videos.append({'video_id': 100 + i, 'captions': [' '.join(t) for t in toks],
                       'processed_tokens': toks})
    st = build_label_store(vocab, videos, 6)
    lab = save_label_file(str(tmp_path / 'lab.npz'), st)
    rng = np.random.RandomState(0)
    f1 = save_feature_file(str(tmp_path / 'a.npz'), st['videos'],
                           rng.rand(len(ncaps), 4).astype(np.float32))
    f2 = save_feature_file(str(tmp_path / 'b.npz'), st['videos'],
                           rng.rand(len(ncaps), 7).astype(np.float32))
    return lab, [f1, f2]


def test_dataloader_opt_dict_and_getters(tmp_path):
    lab, feats = _files(tmp_path)
    loader = compat.DataLoader({'label_h5': lab, 'feat_h5': feats, 'batch_size': 2,
                                'seq_per_img': 20, 'mode': 'train', 'num_chunks': 1})
    assert loader.get_num_videos() == 3 and loader.get_batch_size() == 2
    assert loader.get_feat_dims() == [4, 7]
    assert loader.get_feat_size() == 11 and loader.get_num_feats() == 2
    assert loader.get_seq_length() == 6 and loader.get_seq_per_img() == 20
    assert loader.get_vocab()[0] == '<end>' and loader.get_vocab_size() == 13
    assert loader.get_cocofmt_file() is None
    data = loader.get_batch()
    assert [f.shape for f in data['feats']] == [(2, 1, 4), (2, 1, 7)]
    assert data['labels'].shape == (40, 6) and data['masks'].shape == (40, 6)
    assert len(data['ids']) == 2 and all(i in (100, 101, 102) for i in data['ids'])
    # mask = caption tokens + EOS (dataloader.py:158-163)
    n = (data['labels'] != 0).sum(1) + 1
    assert torch.equal(data['masks'].sum(1).long(), n)
    loader.get_batch()  # wraps the 3-video epoch
    assert loader.get_current_epoch() == 1
    loader.close()


def test_dataloader_accepts_ready_dataset():
    ds = make_synthetic('msvd', num_videos=6, vocab_size=40, seq_length=8, seed=0)
    loader = compat.DataLoader({'dataset': ds, 'batch_size': 3, 'seq_per_img': 4,
                                'mode': 'test'})
    assert loader.get_batch()['labels'].shape == (12, 8)
    assert loader.get_num_feats() == len(ds.feat_dims)


def test_score_and_language_eval_from_file(tmp_path):
    refs = {1: ['a man is playing a guitar', 'a person plays guitar'],
            2: ['a cat is sleeping', 'a cat sleeps on a bed']}
    hyps = {1: ['a man is playing a guitar'], 2: ['a dog is running']}
    s = compat.score(refs, hyps)
    assert set(s) == {'Bleu_1', 'Bleu_2', 'Bleu_3', 'Bleu_4', 'METEOR', 'ROUGE_L', 'CIDEr'}
    assert s['Bleu_1'] > 0.4
    coco = {'images': [{'id': 1}, {'id': 2}],
            'annotations': [{'image_id': k, 'caption': c, 'id': i}
                            for i, (k, cs) in enumerate(refs.items()) for c in cs],
            'type': 'captions', 'info': {}, 'licenses': []}
    gold = tmp_path / 'gold.json'
    gold.write_text(json.dumps(coco))
    preds = [{'image_id': 1, 'caption': 'a man is playing a guitar'},
             {'image_id': 2, 'caption': 'a cat is sleeping'}]
    pred = tmp_path / 'pred.json'
    pred.write_text(json.dumps(preds))
    out = compat.language_eval(str(gold), str(pred))
    assert out == compat.language_eval(str(gold), preds)
    assert out['CIDEr'] > 1.0 and out['Bleu_4'] > 0.5
    assert compat.load_gt_refs(str(gold)) == refs


def test_compute_score_and_dead_sc_reward2():
    refs = {0: ['5 6 7 0', '5 6 8 0'], 1: ['9 10 0', '9 11 0']}
    scorer = compat.CiderD(df='corpus')
    preds = [{'image_id': 0, 'caption': '5 6 7 0'}, {'image_id': 1, 'caption': '12 0'}]
    mean, per = compute = compat.compute_score(refs, preds, scorer)
    assert per.shape == (2,) and per[0] > per[1] and abs(mean - per.mean()) < 1e-12
    assert compute[0] == mean
    # the dead helper hands its arguments to compute_score in swapped order
    # (utils.py:157-158): "model_res" lands in the refs slot, "gt_refs" in the
    # predictions slot; reproduced as is
    m, g = compat.get_self_critical_reward2(refs, {0: ['12 0'], 1: ['12 0']}, preds, scorer)
    assert abs(m - mean) < 1e-12 and g < m
