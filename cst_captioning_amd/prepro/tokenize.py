"""P2: group captions per video and tokenise them.

Behaviour of ``/root/reference/preprocess_datainfo.py:19-65``: drop
non-ASCII characters, lowercase, strip ASCII punctuation, split on
whitespace.  Output: ``[{category, video_id, captions, processed_tokens}]``.
"""
import argparse
import json
import string

_TABLE = str.maketrans('', '', string.punctuation)


def tokenize_caption(caption):
    ascii_only = ''.join(ch for ch in caption if ord(ch) < 128)
    return ascii_only.lower().translate(_TABLE).strip().split()


def group_and_tokenize(datainfo):
    by_video = {}
    for ann in datainfo['captions']:
        by_video.setdefault(ann['video_id'], []).append(ann['caption'])
    videos = []
    for v in datainfo['videos']:
        caps = by_video.get(v['id'], [])
        videos.append({'category': v.get('category', 'unknown'), 'video_id': v['id'],
                       'captions': caps,
                       'processed_tokens': [tokenize_caption(c) for c in caps]})
    return videos


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('input_json')
    p.add_argument('output_json')
    a = p.parse_args(argv)
    with open(a.input_json) as f:
        videos = group_and_tokenize(json.load(f))
    with open(a.output_json, 'w') as f:
        json.dump(videos, f)
    return videos


if __name__ == '__main__':
    main()
