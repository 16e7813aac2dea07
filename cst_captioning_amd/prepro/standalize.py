"""P1: convert raw dataset metadata into the standard datainfo JSON
``{'info', 'videos': [...], 'captions': [...]}``.

Behaviour of ``/root/reference/standalize_format.py`` (yt2t ``:17-65``,
msrvtt2016/2017 ``:68-106``, tvvtt ``:109-141``), written for Python 3 (the
reference's ``unicode`` call and its global ``args`` lookups are fixed,
SURVEY.md §2.8 item 8).
"""
import argparse
import itertools
import json
import logging
import os

logger = logging.getLogger(__name__)


def standalize_yt2t(input_file):
    """YouTube2Text NAACL15 split: ``vidN\\tcaption`` lines."""
    order, caps = [], {}
    with open(input_file, encoding='utf-8', errors='ignore') as f:
        for line in f:
            line = line.rstrip('\n')
            if not line:
                continue
            vid, cap = line.split('\t', 1)
            if vid not in caps:
                caps[vid] = []
                order.append(vid)
            caps[vid].append(cap)
    videos, captions = [], []
    counter = itertools.count()
    for vid in order:
        num = int(vid[3:])
        videos.append({'category': 'unknown', 'video_id': vid, 'id': num,
                       'start_time': -1, 'end_time': -1, 'url': ''})
        for cap in caps[vid]:
            captions.append({'id': next(counter), 'video_id': num, 'caption': cap})
    return {'info': {}, 'videos': videos, 'captions': captions}


def standalize_msrvtt(input_file, dataset='msrvtt2016', split='train', val2016_json=None):
    """MSR-VTT; 2017 train = all 2017 train videos minus the val2016 ones."""
    with open(input_file) as f:
        info = json.load(f)
    if split == 'val':
        split = 'validate'
    out = {'info': info.get('info', {})}
    if dataset == 'msrvtt2017' and split == 'train':
        with open(val2016_json) as f:
            v16 = json.load(f)
        held = {v['video_id'] for v in v16['videos'] if v['split'] == 'validate'}
        out['videos'] = [v for v in info['videos'] if v['video_id'] not in held]
    else:
        out['videos'] = [v for v in info['videos'] if v['split'] == split]
    ids = {v['video_id']: v['id'] for v in out['videos']}
    out['captions'] = [{'id': c['sen_id'], 'video_id': ids[c['video_id']],
                        'caption': c['caption']}
                       for c in info['sentences'] if c['video_id'] in ids]
    return out


def standalize_tvvtt(input_file, split='train'):
    """TRECVID VTT metadata: each provided set is its own split."""
    key = {'train': 'train2016', 'val': 'test2016', 'test': 'test2017'}[split]
    with open(input_file) as f:
        info = json.load(f)[key]
    videos = [{'category': 'unknown', 'video_id': str(v), 'id': v, 'start_time': -1,
               'end_time': -1, 'url': ''} for v in info['videos']]
    return {'info': {}, 'videos': videos, 'captions': info['captions']}


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('input_file')
    p.add_argument('output_json')
    p.add_argument('--split', type=str, default='train')
    p.add_argument('--dataset', default='yt2t',
                   choices=['yt2t', 'msrvtt2016', 'msrvtt2017', 'tvvtt'])
    p.add_argument('--val2016_json', type=str)
    a = p.parse_args(argv)
    if a.dataset in ('msrvtt2016', 'msrvtt2017'):
        out = standalize_msrvtt(a.input_file, a.dataset, a.split, a.val2016_json)
    elif a.dataset == 'yt2t':
        out = standalize_yt2t(a.input_file)
    else:
        out = standalize_tvvtt(a.input_file, a.split)
    d = os.path.dirname(a.output_json)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(a.output_json, 'w') as f:
        json.dump(out, f)
    return out


if __name__ == '__main__':
    logging.basicConfig(level=logging.INFO)
    main()
