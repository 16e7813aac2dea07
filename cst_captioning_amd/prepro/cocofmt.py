"""P5: datainfo -> COCO caption format for language evaluation.

``/root/reference/convert_datainfo2cocofmt.py:18-89`` (optionally keeping a
random subset of ``max_caption`` captions per video).
"""
import argparse
import json
import random


def remove_nonascii(s):
    return ''.join(ch for ch in s if ord(ch) < 128)


def to_cocofmt(datainfo, max_caption=0, rng=random):
    keep = None
    if max_caption > 0:
        per_video = {}
        for c in datainfo['captions']:
            per_video.setdefault(c['video_id'], []).append(c['id'])
        keep = set()
        for ids in per_video.values():
            keep.update(rng.sample(ids, min(max_caption, len(ids))))
    anns = [{'caption': remove_nonascii(c['caption']), 'image_id': c['video_id'],
             'id': c['id']}
            for c in datainfo['captions'] if keep is None or c['id'] in keep]
    return {'images': [{'id': v['id']} for v in datainfo['videos']], 'annotations': anns,
            'type': 'captions', 'info': datainfo.get('info', {}), 'licenses': 'n/a'}


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('input_json')
    p.add_argument('output_json')
    p.add_argument('--max_caption', type=int, default=0)
    a = p.parse_args(argv)
    with open(a.input_json) as f:
        out = to_cocofmt(json.load(f), a.max_caption)
    with open(a.output_json, 'w') as f:
        json.dump(out, f)
    return out


if __name__ == '__main__':
    main()
