"""P3: vocabulary builder.

``/root/reference/build_vocab.py:23-52``: words with count >= threshold, in
first-seen order, after the three specials ``['<end>', '<start>', '<unk>']``
(EOS = 0 so that padding and end-of-sentence coincide).
"""
import argparse
import json
from collections import Counter

PAD_TOKEN = '<pad>'
UNK_TOKEN = '<unk>'
BOS_TOKEN = '<start>'
EOS_TOKEN = '<end>'
SPECIALS = [EOS_TOKEN, BOS_TOKEN, UNK_TOKEN]


def build_vocab(videos, word_count_threshold):
    counts = Counter()
    for v in videos:
        for toks in v['processed_tokens']:
            counts.update(toks)
    return SPECIALS + [w for w, n in counts.items() if n >= word_count_threshold]


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('input_json')
    p.add_argument('output_json')
    p.add_argument('--word_count_threshold', type=int, default=0)
    a = p.parse_args(argv)
    with open(a.input_json) as f:
        vocab = build_vocab(json.load(f), a.word_count_threshold)
    with open(a.output_json, 'w') as f:
        json.dump(vocab, f)
    return vocab


if __name__ == '__main__':
    main()
