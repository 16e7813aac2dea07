"""Building blocks of the caption model.

State-dict keys and shapes match the reference:
``feat_pool.feat_list.{i}.0.{weight,bias}``, ``core.rnn.weight_{ih,hh}_l0``
(no biases, gate order i,f,g,o), ``manet.{f_feat_m,f_h_m,align_m}.*``.

  * FeatPool     -- ``/root/reference/model.py:46-69`` (generalised to keep
                    the chunk axis when ``num_chunks > 1``)
  * FeatExpander -- ``model.py:72-90`` (vectorised ``repeat_interleave``
                    instead of a Python loop over the batch)
  * RNNUnit      -- ``model.py:93-116``
  * MANet        -- ``model.py:119-142`` (Python-3 fix: integer block size;
                    attention applied to the un-attended features every step)
  * TemporalAttention -- new: the temporal attention the reference only
                    declares (``opts.py:241-245``, ``model.py:61-66``)
"""
import warnings

import torch
import torch.nn as nn
import torch.nn.functional as F


class FeatPool(nn.Module):
    """Per-modality ``Linear -> ReLU -> Dropout``, concatenated."""

    def __init__(self, feat_dims, out_size, dropout):
        super().__init__()
        self.feat_list = nn.ModuleList([
            nn.Sequential(nn.Linear(d, out_size), nn.ReLU(), nn.Dropout(dropout))
            for d in feat_dims])

    def forward(self, feats):
        """feats: list of (N, C, dim_i).  Returns (N, F*out) for C == 1 (the
        reference shape) or (N, C, F*out) for C > 1."""
        outs = [m(f) for m, f in zip(self.feat_list, feats)]
        out = torch.cat(outs, dim=-1)
        return out.squeeze(1) if out.size(1) == 1 else out


class FeatExpander(nn.Module):
    def __init__(self, n=1):
        super().__init__()
        self.n = n

    def forward(self, x):
        return x if self.n == 1 else x.repeat_interleave(self.n, dim=0)

    def set_n(self, n):
        self.n = n


class RNNUnit(nn.Module):
    def __init__(self, rnn_type, input_size, rnn_size, num_layers, dropout):
        super().__init__()
        self.rnn_type = rnn_type
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')  # dropout with 1 layer: a no-op, as in the reference
            self.rnn = getattr(nn, rnn_type.upper())(input_size, rnn_size, num_layers,
                                                     bias=False, dropout=dropout)

    def forward(self, xt, state):
        out, state = self.rnn(xt.unsqueeze(0), state)
        return out.squeeze(0), state


class MANet(nn.Module):
    """Modal attention: softmax over the F modality blocks of the video
    vector, conditioned on the hidden state."""

    def __init__(self, video_encoding_size, rnn_size, num_feats):
        super().__init__()
        self.video_encoding_size = video_encoding_size
        self.num_feats = num_feats
        self.f_feat_m = nn.Linear(video_encoding_size, num_feats)
        self.f_h_m = nn.Linear(rnn_size, num_feats)
        self.align_m = nn.Linear(num_feats, num_feats)

    def forward(self, x, h):
        w = F.softmax(self.align_m(torch.tanh(self.f_feat_m(x) + self.f_h_m(h[-1]))), dim=-1)
        block = self.video_encoding_size // self.num_feats
        return x * w.repeat_interleave(block, dim=1)


class TemporalAttention(nn.Module):
    """Additive attention over the ``C`` frame vectors of a video:
    ``alpha = softmax_c(w^T tanh(W_v v_c + W_h h))``, context
    ``sum_c alpha_c v_c``.  ``W_v v_c`` is precomputed once per video."""

    def __init__(self, video_encoding_size, rnn_size, att_size):
        super().__init__()
        self.f_feat = nn.Linear(video_encoding_size, att_size)
        self.f_h = nn.Linear(rnn_size, att_size, bias=False)
        self.align = nn.Linear(att_size, 1)

    def precompute(self, frames):
        return self.f_feat(frames)

    def forward(self, frames, pre, h):
        e = self.align(torch.tanh(pre + self.f_h(h)[:, None, :])).squeeze(-1)
        alpha = F.softmax(e, dim=1)
        return torch.bmm(alpha.unsqueeze(1), frames).squeeze(1), alpha
