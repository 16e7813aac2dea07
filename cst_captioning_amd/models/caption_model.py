"""CaptionModel: multi-modal video encoder + LSTM caption decoder.

API and checkpoint layout of ``/root/reference/model.py:145-512``:
``forward(feats, seq) -> (logprobs N x T x V, sample_seq, sample_logprobs)``,
``sample(feats, opt) -> (seq, seqLogprobs)``, the setters
``set_ss_prob / set_mixer_from / set_seq_per_img``, identical state_dict
keys, U(-0.1, 0.1) init of ``embed``/``logit`` and a zero logit bias.

Two implementations of the decoding loops live behind this API:

  * the methods in this file -- plain PyTorch ops, one time step at a time.
    They define the reference semantics (scheduled sampling, MIXER rollout
    without an after-EOS mask, early exit when every row emits EOS, greedy /
    multinomial ``sample`` with an ``unfinished`` mask, beam search with
    perplexity ranking) and run anywhere, including CPU;
  * :mod:`.decoder_engine` -- the fused HIP engine used on MI355X
    (``impl='hip'``), which reproduces the same semantics with MFMA kernels
    and no host synchronisation inside the time loop.

The beam search here is *batched over videos* (the reference runs one video
at a time with CPU sorts, ``model.py:382-466``) but keeps its semantics:
only beam 0 expands at the first step, beams that emitted EOS keep
expanding, every EOS / last-step beam is harvested, and the harvested beam
with the lowest ``exp(-sum logp / (t-1))`` wins (earliest on ties).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.text import BOS
from .modules import FeatPool, FeatExpander, RNNUnit, MANet, TemporalAttention


class CaptionModel(nn.Module):

    def __init__(self, opt):
        super().__init__()
        self.vocab_size = opt.vocab_size
        self.input_encoding_size = opt.input_encoding_size
        self.rnn_type = opt.rnn_type
        self.rnn_size = opt.rnn_size
        self.num_layers = opt.num_layers
        self.drop_prob_lm = opt.drop_prob_lm
        self.seq_length = opt.seq_length
        self.feat_dims = list(opt.feat_dims)
        self.num_feats = len(self.feat_dims)
        self.seq_per_img = opt.train_seq_per_img
        self.model_type = opt.model_type
        self.num_chunks = getattr(opt, 'num_chunks', 1)
        self.bos_index = BOS
        self.ss_prob = 0.0
        self.mixer_from = 0
        self.mask_after_eos = bool(getattr(opt, 'mask_after_eos', 0))

        self.embed = nn.Embedding(self.vocab_size, self.input_encoding_size)
        self.logit = nn.Linear(self.rnn_size, self.vocab_size)
        self.dropout = nn.Dropout(self.drop_prob_lm)
        self.init_weights()

        self.feat_pool = FeatPool(self.feat_dims, self.num_layers * self.rnn_size,
                                  self.drop_prob_lm)
        self.feat_expander = FeatExpander(self.seq_per_img)
        self.video_encoding_size = self.num_feats * self.num_layers * self.rnn_size
        opt.video_encoding_size = self.video_encoding_size
        if self.model_type == 'standard':
            in_size = self.input_encoding_size
            if self.video_encoding_size != self.input_encoding_size:
                raise ValueError("model_type 'standard' feeds the video vector as the first "
                                 'LSTM input: needs num_feats*rnn_size == input_encoding_size')
        else:
            in_size = self.input_encoding_size + self.video_encoding_size
        self.core = RNNUnit(self.rnn_type, in_size, self.rnn_size, self.num_layers,
                            self.drop_prob_lm)
        if self.model_type == 'manet':
            self.manet = MANet(self.video_encoding_size, self.rnn_size, self.num_feats)
        if self.num_chunks > 1:
            if self.model_type != 'concat':
                raise ValueError('temporal attention (num_chunks > 1) needs model_type concat')
            self.temporal_att = TemporalAttention(self.video_encoding_size, self.rnn_size,
                                                  self.rnn_size)
        self.impl = 'torch'
        self._engine = None

    # -- reference setters ----------------------------------------------------
    def set_ss_prob(self, p):
        self.ss_prob = p

    def set_mixer_from(self, t):
        self.mixer_from = t

    def set_seq_per_img(self, n):
        self.seq_per_img = n
        self.feat_expander.set_n(n)

    def init_weights(self):
        nn.init.uniform_(self.embed.weight, -0.1, 0.1)
        nn.init.uniform_(self.logit.weight, -0.1, 0.1)
        nn.init.constant_(self.logit.bias, 0)

    def init_hidden(self, n):
        w = next(self.parameters())
        z = w.new_zeros((self.num_layers, n, self.rnn_size))
        return (z, z.clone()) if self.rnn_type == 'lstm' else z

    # -- encoder / one decoder step --------------------------------------------
    def encode(self, feats):
        """(N, F*H) video vectors (or (N, C, F*H) frame vectors)."""
        return self.feat_pool(feats)

    def _video_ctx(self, video):
        if self.num_chunks > 1:
            return {'frames': video, 'pre': self.temporal_att.precompute(video)}
        return {'video': video}

    def _expand_ctx(self, ctx, n):
        return {k: v.repeat_interleave(n, dim=0) for k, v in ctx.items()}

    def _step(self, xt, ctx, state):
        if self.model_type == 'standard':
            return self.core(xt, state)
        h = state[0] if self.rnn_type == 'lstm' else state
        if self.num_chunks > 1:
            v, _ = self.temporal_att(ctx['frames'], ctx['pre'], h[-1])
        elif self.model_type == 'manet':
            v = self.manet(ctx['video'], h)
        else:
            v = ctx['video']
        return self.core(torch.cat([xt, v], 1), state)

    def _first_input(self, ctx):
        # 'standard': the video vector is the input of step -1
        return ctx['video']

    # -- teacher forcing / scheduled sampling / MIXER rollout -----------------
    def forward(self, feats, seq):
        if self.impl == 'hip' and self._engine is not None:
            return self._engine.forward_full(self, feats, seq)
        ctx = self._expand_ctx(self._video_ctx(self.encode(feats)), self.feat_expander.n)
        n = seq.size(0)
        state = self.init_hidden(n)
        outputs, sample_seq, sample_lp = [], [], []
        alive = None
        start = -1 if self.model_type == 'standard' else 0
        for t in range(start, seq.size(1) - 1):
            if t == -1:
                xt = self._first_input(ctx)
            else:
                if self.training and t >= 1 and self.ss_prob > 0.0:
                    it = seq[:, t].clone()
                    use = torch.rand(n, device=seq.device) < self.ss_prob
                    if use.any():
                        drawn = torch.multinomial(outputs[-1].detach().exp(), 1).view(-1)
                        it = torch.where(use, drawn, it)
                elif self.training and self.mixer_from > 0 and t >= self.mixer_from:
                    it = torch.multinomial(outputs[-1].detach().exp(), 1).view(-1)
                    if self.mask_after_eos:
                        alive = (it > 0) if alive is None else alive & (it > 0)
                        it = it * alive
                else:
                    it = seq[:, t].clone()
                if t >= 1:
                    sample_seq.append(it)
                    sample_lp.append(outputs[-1].gather(1, it.unsqueeze(1)).view(-1))
                if int(it.sum()) == 0:  # every sequence ended (EOS = 0)
                    break
                xt = self.embed(it)
            out, state = self._step(xt, ctx, state)
            if t >= 0:
                outputs.append(F.log_softmax(self.logit(self.dropout(out)), dim=-1))
        return (torch.stack(outputs, 1), torch.stack(sample_seq, 1),
                torch.stack(sample_lp, 1))

    # -- greedy / multinomial decoding ----------------------------------------
    def sample(self, feats, opt={}):
        beam_size = opt.get('beam_size', 1)
        if beam_size > 1:
            return self.sample_beam(feats, opt)
        if self.impl == 'hip' and self._engine is not None:
            return self._engine.sample(self, feats, opt)
        sample_max = opt.get('sample_max', 1)
        temperature = opt.get('temperature', 1.0)
        ctx = self._video_ctx(self.encode(feats))
        if opt.get('expand_feat', 0) == 1:
            ctx = self._expand_ctx(ctx, self.feat_expander.n)
        n = next(iter(ctx.values())).size(0)
        state = self.init_hidden(n)
        seq, seq_lp = [], []
        unfinished = None
        start = -1 if self.model_type == 'standard' else 0
        logprobs = None
        for t in range(start, self.seq_length - 1):
            if t == -1:
                xt = self._first_input(ctx)
            else:
                if t == 0:
                    it = torch.full((n,), self.bos_index, dtype=torch.long,
                                    device=next(self.parameters()).device)
                elif sample_max == 1:
                    lp_t, it = torch.max(logprobs.detach(), 1)
                else:
                    p = (logprobs.detach() / temperature).exp() if temperature != 1.0 \
                        else logprobs.detach().exp()
                    it = torch.multinomial(p, 1).view(-1)
                    lp_t = logprobs.gather(1, it.unsqueeze(1)).view(-1)
                xt = self.embed(it)
                if t >= 1:
                    unfinished = (it > 0) if unfinished is None else unfinished & (it > 0)
                    it = it * unfinished
                    seq.append(it)
                    seq_lp.append(lp_t.view(-1))
                    if int(unfinished.sum()) == 0:
                        break
            out, state = self._step(xt, ctx, state)
            logprobs = F.log_softmax(self.logit(out), dim=-1)
        return torch.stack(seq, 1), torch.stack(seq_lp, 1)

    # -- beam search (batched over videos, reference semantics) ----------------
    def sample_beam(self, feats, opt={}):
        if self.impl == 'hip' and self._engine is not None:
            return self._engine.sample_beam(self, feats, opt)
        K = opt.get('beam_size', 5)
        V = self.vocab_size
        T = self.seq_length
        if K > V:
            raise ValueError('beam_size > vocab_size')
        ctx0 = self._video_ctx(self.encode(feats))
        B = next(iter(ctx0.values())).size(0)
        dev = next(self.parameters()).device
        ctx = self._expand_ctx(ctx0, K)
        state = self.init_hidden(B * K)
        beam_seq = torch.zeros(B, K, T, dtype=torch.long, device=dev)
        beam_lp = torch.zeros(B, K, T, device=dev)
        beam_sum = torch.zeros(B, K, device=dev)
        best_ppl = torch.full((B,), math.inf, device=dev)
        best_seq = torch.zeros(B, T, dtype=torch.long, device=dev)
        best_lp = torch.zeros(B, T, device=dev)
        bidx = torch.arange(B, device=dev)[:, None]
        logprobs = None
        start = -1 if self.model_type == 'standard' else 0
        for t in range(start, T - 1):
            if t == -1:
                xt = self._first_input(ctx)
            elif t == 0:
                xt = self.embed(torch.full((B * K,), self.bos_index, dtype=torch.long,
                                           device=dev))
            else:
                lp = logprobs.float().view(B, K, V)
                ys, ix = lp.topk(K, dim=2)  # per beam, best words first
                rows = 1 if t == 1 else K
                # reference candidate order: for c (word rank): for q (beam)
                cand_p = (beam_sum[:, :rows, None] + ys[:, :rows, :]).transpose(1, 2)
                cand_p = cand_p.reshape(B, K * rows)
                order = torch.sort(cand_p, dim=1, descending=True, stable=True).indices[:, :K]
                q = order % rows
                c = order // rows
                tok = ix[bidx, q, c]
                raw = ys[bidx, q, c]
                beam_sum = cand_p.gather(1, order)
                beam_seq = beam_seq[bidx, q]
                beam_lp = beam_lp[bidx, q]
                beam_seq[:, :, t - 1] = tok
                beam_lp[:, :, t - 1] = raw
                src = (bidx * K + q).reshape(-1)
                state = tuple(s[:, src] for s in state) if isinstance(state, tuple) \
                    else state[:, src]
                done = (tok == 0) | (t == T - 2)
                ppl = torch.exp(-beam_sum / (t - 1)) if t > 1 else \
                    torch.full_like(beam_sum, 10000.0)
                for v in range(K):  # harvest in the reference's order (earliest wins ties)
                    upd = done[:, v] & (ppl[:, v] < best_ppl)
                    best_ppl = torch.where(upd, ppl[:, v], best_ppl)
                    best_seq = torch.where(upd[:, None], beam_seq[:, v], best_seq)
                    best_lp = torch.where(upd[:, None], beam_lp[:, v], best_lp)
                xt = self.embed(tok.reshape(-1))
            out, state = self._step(xt, ctx, state)
            logprobs = F.log_softmax(self.logit(out), dim=-1)
        return best_seq, best_lp
