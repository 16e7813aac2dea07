"""CIDEr-D reward scorer: on-GPU HIP kernel, or CPU scorers.

The reference scores every RL iteration on the CPU through the external
CiderD package: device->host copy of the samples, Python string building
(``utils.py:135-152``) and pure-Python n-gram scoring of 1,280 (CST) or
2,560 (SCST) hypotheses against ~20 references each (the
dominant hot spot).  Here:

  * the df table becomes an open-addressing hash table in HBM keyed by the
    exact packed n-gram (:func:`..prepro.ciderdf.pack_ngram`);
  * each video's reference n-gram vectors, norms and "lengths" are
    precomputed ONCE per dataset by the native host builder
    (``csrc/host/cider_tables.cpp``) and uploaded;
  * ``csrc/kernels/cider_d.hip`` scores one hypothesis per wavefront
    (token compaction with ballots, n-gram counting in LDS, df lookups,
    clipped cosine + length penalty against the video's refs).

So the self-critical loop never leaves HBM.  ``backend='cpu-ref'`` reproduces
the reference cost model (strings + Python scorer) and is what the
reference-semantics baseline uses; ``backend='cpu'`` is the native C++
scorer (same tables, fp64).
"""
import math

import numpy as np
import torch

from .. import _ext
from ..reward.cider_d_cpu import CiderD
from ..reward.rewards import score_hypotheses
from ..prepro.ciderdf import unpack_ngram_keys


class CiderDScorer:
    def __init__(self, dataset, use_eos=0, device='cpu', backend='auto'):
        if dataset.df is None:
            raise ValueError('dataset has no CIDEr-D document-frequency table')
        self.ds = dataset
        self.use_eos = int(use_eos)
        self.device = torch.device(device)
        keys, vals, ref_len = dataset.df
        self.keys = np.ascontiguousarray(keys, dtype=np.uint64)
        self.vals = np.ascontiguousarray(vals, dtype=np.float32)
        self.ref_len = ref_len
        self.log_ref_len = math.log(float(ref_len))
        if backend == 'auto':
            backend = 'gpu' if (self.device.type == 'cuda' and _ext.available()) else 'cpu-ref'
            if backend == 'cpu-ref' and _ext.host_available():
                backend = 'cpu'
        self.backend = backend
        self._tables = None
        self._oracle = None
        if backend in ('gpu', 'cpu'):
            self._build_tables()

    # -- table construction ------------------------------------------------------
    def _build_tables(self):
        lab = np.ascontiguousarray(self.ds.labels, dtype=np.int64)
        st = np.ascontiguousarray(self.ds.label_start_ix, dtype=np.int64)
        en = np.ascontiguousarray(self.ds.label_end_ix, dtype=np.int64)
        t = _ext.ops().cider_build_tables(torch.from_numpy(lab), torch.from_numpy(st),
                                          torch.from_numpy(en),
                                          torch.from_numpy(self.keys.view(np.int64)),
                                          torch.from_numpy(self.vals), self.log_ref_len,
                                          self.use_eos)
        # t: dict of CPU tensors
        if self.backend == 'gpu':
            t = {k: v.to(self.device) for k, v in t.items()}
        self._tables = t

    def _oracle_scorer(self):
        if self._oracle is None:
            df = dict(zip(unpack_ngram_keys(self.keys), self.vals.astype(np.float64).tolist()))
            self._oracle = CiderD({'document_frequency': df, 'ref_len': self.ref_len})
        return self._oracle

    # -- scoring -------------------------------------------------------------------
    def score(self, hyps, video_index):
        """hyps: (N, T) long tensor; video_index: (N,) dataset video indices.
        Returns (N,) float32 scores on ``hyps.device``."""
        if self.backend == 'gpu':
            return _ext.ops().cider_score(hyps.contiguous(), video_index.contiguous(),
                                          self._tables, self.log_ref_len, self.use_eos)
        if self.backend == 'cpu':
            s = _ext.ops().cider_score_cpu(hyps.detach().cpu().contiguous(),
                                           video_index.detach().cpu().contiguous(),
                                           self._tables, self.log_ref_len, self.use_eos)
            return s.to(hyps.device)
        # reference cost model: strings + pure-Python scorer on the host
        h = hyps.detach().cpu().numpy()
        v = video_index.detach().cpu().numpy()
        gts = [self.ds.gts_of(int(x)) for x in v]
        s = score_hypotheses(self._oracle_scorer(), h, gts, seq_per_img=1, expand_feat=1,
                             use_eos=self.use_eos)
        return torch.from_numpy(s.astype(np.float32)).to(hyps.device)

    def score_reference(self, hyps, video_index):
        """fp64 oracle (pure Python), for tests."""
        h = hyps.detach().cpu().numpy()
        v = video_index.detach().cpu().numpy()
        gts = [self.ds.gts_of(int(x)) for x in v]
        return score_hypotheses(self._oracle_scorer(), h, gts, seq_per_img=1, expand_feat=1,
                                use_eos=self.use_eos)


class GenericScorer:
    """Any reference-style scorer (Bleu_4 / METEOR / ROUGE_L) on the CPU,
    for ``--eval_metric`` values other than CIDEr (``train.py:119-124``)."""

    def __init__(self, dataset, scorer, use_eos=0):
        self.ds, self.scorer, self.use_eos = dataset, scorer, int(use_eos)
        self.backend = 'cpu-ref'

    def score(self, hyps, video_index):
        h = hyps.detach().cpu().numpy()
        v = video_index.detach().cpu().numpy()
        gts = [self.ds.gts_of(int(x)) for x in v]
        s = score_hypotheses(self.scorer, h, gts, seq_per_img=1, expand_feat=1,
                             use_eos=self.use_eos)
        return torch.from_numpy(s.astype(np.float32)).to(hyps.device)
