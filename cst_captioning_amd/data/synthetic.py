"""Synthetic datasets with the shapes of MSR-VTT and MSVD.

There is no network (no datasets, no features), so benchmarks and
integration tests run on generated data that has the reference workload's
*shape*:

  * ``msrvtt``: 6,513 train videos, exactly 20 captions each, 4 modalities
    (ResNet-152 2048, C3D 4096, MFCC 1024, category GloVe 300 -- dims are
    the SURVEY.md §2.3 assumptions), vocabulary ~10.5k, max length 30;
  * ``msvd``: 1,200 videos with a *variable* number of captions (≈20-60,
    so ``ncap > S`` and ``ncap < S`` both occur), 2 modalities.

Captions are not noise: every video has a latent topic, features are a
topic embedding plus noise, and caption words are drawn from a Zipf law over
a topic-specific word permutation.  A model can therefore learn the task
(used by the "loss decreases / CIDEr improves" integration tests).
``caption_mode='template'`` makes the captions (nearly) a deterministic
function of the features: each topic has one template sentence of
topic-specific words, and every caption is that template with each word
replaced by a random topic word with probability 0.15 and the last word
dropped with probability 0.2 -- a greedy decoder that recovers the topic
from the features scores a high CIDEr-D, so learning curves separate from
noise (the Zipf captions' CIDEr-D stays near zero at the headline scale).

The generator goes through the real preprocessing code path
(tokens -> vocab -> label store -> df table), so synthetic artefacts are
exactly what ``prepro`` would write for a real dataset of that shape.
"""
import numpy as np

from ..prepro.vocab import SPECIALS
from ..prepro.labels import build_label_store
from ..prepro.ciderdf import df_from_token_refs
from .dataset import VideoCaptionDataset

MSRVTT_FEAT_DIMS = [2048, 4096, 1024, 300]
MSVD_FEAT_DIMS = [2048, 4096]


def _captions_for(rng, topic_perm, n_words, ncap, mean_len, max_words, zipf_a):
    caps = []
    for _ in range(ncap):
        n = int(np.clip(np.round(rng.normal(mean_len, 3.0)), 3, max_words))
        ranks = np.minimum(rng.zipf(zipf_a, size=n) - 1, n_words - 1)
        caps.append(['w%d' % topic_perm[r] for r in ranks])
    return caps


def _template_captions(rng, template, topic_perm, n_words, ncap):
    caps = []
    for _ in range(ncap):
        t = list(template)
        if len(t) > 4 and rng.rand() < 0.2:
            t = t[:-1]
        for k in range(len(t)):
            if rng.rand() < 0.15:
                t[k] = 'w%d' % topic_perm[min(rng.zipf(1.35) - 1, n_words - 1)]
        caps.append(t)
    return caps


def make_synthetic(kind='msrvtt', num_videos=None, vocab_size=10509, seq_length=30,
                   feat_dims=None, num_chunks=1, n_topics=64, seed=0, mean_len=9.3,
                   with_consensus=False, split='train', start_video_id=0, consensus_cols=20,
                   world_seed=None, caption_mode='zipf'):
    """``world_seed``: seed of the generative "world" (topic word
    distributions, topic feature embeddings); splits that share it are
    different videos of the same world, so a model trained on one
    generalises to the others.  None: drawn from ``seed`` (one stream)."""
    rng = np.random.RandomState(seed)
    wrng = rng if world_seed is None else np.random.RandomState(world_seed)
    if kind == 'msrvtt':
        num_videos = num_videos or 6513
        feat_dims = feat_dims or MSRVTT_FEAT_DIMS
        caps_per_video = lambda: 20
    elif kind == 'msvd':
        num_videos = num_videos or 1200
        feat_dims = feat_dims or MSVD_FEAT_DIMS
        caps_per_video = lambda: int(rng.randint(8, 61))
    else:
        raise ValueError('unknown synthetic dataset %r' % kind)
    n_words = vocab_size - len(SPECIALS)
    if n_words < 8:
        raise ValueError('vocab_size too small')
    # topic structure: a shared Zipf head + topic-specific tails
    topic_perm = [np.concatenate([np.arange(min(32, n_words)),
                                  wrng.permutation(np.arange(min(32, n_words), n_words))])
                  for _ in range(n_topics)]
    topics = rng.randint(n_topics, size=num_videos)
    if caption_mode not in ('zipf', 'template'):
        raise ValueError('caption_mode must be zipf or template')
    templates = None
    if caption_mode == 'template':  # one sentence of topic-specific words per topic
        templates = [['w%d' % topic_perm[k][32 + wrng.randint(min(400, n_words - 32))]
                      for _ in range(int(wrng.randint(6, 13)))] for k in range(n_topics)]
    # Every word appears in the vocab: word ids are w0..w{n_words-1}, and the
    # vocabulary is built in id order (threshold 0), so ids are stable.
    words = ['w%d' % i for i in range(n_words)]
    vocab = SPECIALS + words
    videos = []
    for i in range(num_videos):
        if templates is not None:
            toks = _template_captions(rng, templates[topics[i]], topic_perm[topics[i]], n_words,
                                      caps_per_video())
        else:
            toks = _captions_for(rng, topic_perm[topics[i]], n_words, caps_per_video(),
                                 mean_len, seq_length + 6, 1.35)
        videos.append({'video_id': start_video_id + i, 'captions': [' '.join(t) for t in toks],
                       'processed_tokens': toks, 'category': int(topics[i])})
    store = build_label_store(vocab, videos, seq_length)
    # features: topic embedding + noise (+ per-chunk jitter)
    feats = []
    for d in feat_dims:
        emb = wrng.normal(0, 1, size=(n_topics, d)).astype(np.float32)
        base = emb[topics] + 0.5 * rng.normal(0, 1, size=(num_videos, d)).astype(np.float32)
        f = np.repeat(base[:, None, :], num_chunks, axis=1)
        if num_chunks > 1:
            f = f + 0.25 * rng.normal(0, 1, size=f.shape).astype(np.float32)
        feats.append(np.maximum(f, 0) if d != 300 else f)  # ReLU-like CNN features
    # CIDEr-D df over index refs (compute_ciderdf.py semantics: no BOS, + EOS)
    wtoi = {w: i for i, w in enumerate(vocab)}
    eos = wtoi['<end>']
    refs_idx = [[[wtoi[w] for w in t] + [eos] for t in v['processed_tokens']] for v in videos]
    df = df_from_token_refs(refs_idx)
    keys = np.fromiter(df[0].keys(), dtype=np.uint64, count=len(df[0]))
    vals = np.fromiter(df[0].values(), dtype=np.float32, count=len(df[0]))
    gt_refs = {start_video_id + i: v['captions'] for i, v in enumerate(videos)}
    bcmr = None
    if with_consensus:
        from ..prepro.evalscores import compute_consensus_scores
        bcmr = compute_consensus_scores(gt_refs, consensus_cols, True, tokenize=False,
                                        metrics=('CIDEr',))['CIDEr']
    return VideoCaptionDataset(vocab, store['videos'], feats, store['labels'],
                               store['label_start_ix'], store['label_end_ix'], bcmr,
                               gt_refs=gt_refs, df=(keys, vals, df[1]))


def make_splits(kind='msrvtt', vocab_size=10509, seq_length=30, feat_dims=None,
                num_chunks=1, train_videos=None, eval_videos=None, seed=0,
                with_consensus=False, seq_per_img=20, caption_mode='zipf'):
    """(train, val, test) synthetic splits sharing one vocabulary."""
    # one generative world (topic vocabularies / feature embeddings) for all
    # three splits, different videos in each
    world = 10007 + seed
    tr = make_synthetic(kind, train_videos, vocab_size, seq_length, feat_dims, num_chunks,
                        seed=seed, with_consensus=with_consensus, consensus_cols=seq_per_img,
                        world_seed=world, caption_mode=caption_mode)
    n_eval = eval_videos or max(8, (train_videos or 600) // 10)
    va = make_synthetic(kind, n_eval, vocab_size, seq_length, feat_dims, num_chunks,
                        seed=seed + 1, start_video_id=10 ** 6, world_seed=world,
                        caption_mode=caption_mode)
    te = make_synthetic(kind, n_eval, vocab_size, seq_length, feat_dims, num_chunks,
                        seed=seed + 2, start_video_id=2 * 10 ** 6, world_seed=world,
                        caption_mode=caption_mode)
    # train df is the one used for CIDEr-D rewards on every split
    va.df = te.df = tr.df
    return tr, va, te
