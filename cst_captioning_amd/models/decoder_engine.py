"""Fused HIP decoder engine (MI355X path of :class:`CaptionModel`).

Wraps the C++ executor of ``csrc/engine.cpp`` (time loops) and the gfx950
kernels of ``csrc/kernels`` in one autograd Function, so a whole
rollout / teacher-forced pass is ONE node of the autograd graph:

  * forward : ``decoder_forward`` runs T decode steps, each = fused LSTM step
    (embedding gather + gate MFMA GEMM + cell) -> fused vocab projection
    (MFMA + LSE / Gumbel-max / argmax epilogue) -> row combine, and returns
    the chosen tokens plus the *gathered* log-probs ``G[r, t]`` of the tokens
    that the losses need (sampled tokens for REINFORCE, targets for XE).
    No ``R x T x V`` log-prob tensor exists.
  * backward: ``decoder_backward`` takes ``dL/dG`` and returns the weight
    gradients (vocab head batched over all T*R rows; LSTM recurrence in
    reverse).

What stays in PyTorch autograd: FeatPool (video encoder, 64 rows) and the
video gate term ``vgate = W_ih[:, E:] . v`` computed once per *video* (the
reference feeds the same video vector at every step to 20 identical rows,
``model.py:84-86,278``), whose gradient the engine returns summed over time
and rows.

Temporal attention (``num_chunks > 1``, the extension of the reference's
declared-only ``--num_chunks``, ``opts.py:241-245``): autograd computes, once
per batch, the per-frame gate table ``Gv[b, c] = W_ih[:, E:] . v_c`` and the
projected frames ``P = f_feat(v)``; every decode step runs the attention
kernel of ``csrc/kernels/attention.hip`` (scores from ``W_q h_{t-1}``,
softmax over frames, ``vgate_r = sum_c alpha_c Gv[b, c]``), and the backward
returns ``dGv, dP, dW_q, dw_a, db_a``.

Semantics match :class:`CaptionModel`'s PyTorch path (reference
``model.py:218-367``) with two documented differences that are
distribution-identical, not value-identical:
  * RNG: multinomial sampling is an exact two-level inverse-CDF draw
    (tile chosen by its probability mass, then a token inside the tile)
    driven by a murmur3-finaliser counter hash of (seed, row, step); dropout
    keep-masks come from the same kind of counter hash of (seed, step, row,
    column), regenerated in the backward (``csrc/common.h`` ``mix32``,
    ``dropout_keep``); the scheduled-sampling coin uses Philox4x32-10;
  * precision: bf16 MFMA operands, fp32 accumulation, cell state and
    softmax statistics in fp32.
Cells (``--rnn_type``, reference ``opts.py`` / ``model.py:93-116``): LSTM,
GRU and tanh RNN share every kernel; only the cell epilogues differ
(``csrc/common.h`` ``cell_fwd`` / ``cell_bwd``).  All three are packed into
4 pre-activation slots per hidden unit (packed gate row ``4u + slot``):
LSTM (i, f, g, o); GRU (r, z, n_x, n_h), where the input-side weights fill
slots r, z, n_x and the recurrent ones r, z, n_h, because GRU's candidate is
``tanh(n_x + r * n_h)``; RNN slot 0 only.  Unused slots are zero rows.

Model types (reference ``model.py:273-278``): ``concat`` (the video vector
enters every step's gates through ``vgate``), ``standard`` (the video
vector is the input of an extra step -1: autograd runs that one cell step
per video, and the engine starts from its state, returning the gradient
w.r.t. that initial state), and ``manet`` (modal attention,
``model.py:119-142``): the F modality blocks of the video vector are the
attention "frames" of the same kernels -- gate table ``Gv[b, f] =
W_iv[:, block f] . v_f``, projected input ``p = W_fm v + b_fm + b_hm``
(shared by every frame), query ``W_hm h_{t-1}`` and per-frame scorer rows
``A_m[f]`` / ``b_m[f]``; the scorer width F is zero-padded to 64 (the
query's GEMM tile), and the padded units contribute nothing.

Stacked layers (``num_layers > 1``, ``model.py:93-116``): layer 0 is the
fused pipeline above; each upper layer ``l`` runs one hipBLASLt GEMM
``dropout(h_{l-1}) W_ih_l^T`` and one step kernel (recurrent GEMM + cell) per
step, its weights packed as ``[W_ih_l | W_hh_l]`` (4H, 2H).  nn.LSTM's
inter-layer dropout uses the same counter hash as the vocab dropout, keyed
per layer, so the backward regenerates it.

Supported configuration: ``rnn_type lstm | gru | rnn``, ``model_type concat
| standard | manet`` (manet: at most 8 modalities), temporal attention with
``concat``, ``num_layers >= 1`` (> 1 with concat, no attention); other
configurations use the PyTorch path (``build_model`` decides).
"""
import os

import torch
import torch.nn.functional as F

from .. import _ext
from ..utils.text import BOS

SEL_GT, SEL_SAMPLE, SEL_GREEDY, SEL_SS = 0, 1, 2, 3
# teacher-forced training forwards on the XE decode launches (csrc/engine.cpp
# "XE all rows"); CSTCAP_XE_ROWS=0: the general per-step launches + combine
XE_ROWS = os.environ.get('CSTCAP_XE_ROWS', '1') != '0'

# cell id of csrc/common.h CellType, gate groups of the PyTorch weights, and
# the packed slot of each gate group on the input / recurrent side
CELLS = {'lstm': (0, 4, (0, 1, 2, 3), (0, 1, 2, 3)),
         'gru': (1, 3, (0, 1, 2), (0, 1, 3)),
         'rnn': (2, 1, (0,), (0,))}

ATT_MAX_CHUNKS = 32  # frames per video supported by csrc/kernels/attention.hip
MANET_MAX_FEATS = 8  # modalities with per-frame scorer weights (attention.hip)
MAX_LAYERS = 5  # bf16 shadow segments of the fused Adam pass (SHADOW_MAX_SEGS)


def engine_unsupported_reason(opt):
    """None when the fused engine runs this configuration, else why not."""
    layers = getattr(opt, 'num_layers', 1)
    mt = getattr(opt, 'model_type', 'concat')
    C = getattr(opt, 'num_chunks', 1)
    if getattr(opt, 'rnn_type', 'lstm') not in CELLS:
        return 'rnn_type %r (supported: lstm, gru, rnn)' % getattr(opt, 'rnn_type', None)
    if not 1 <= layers <= MAX_LAYERS:
        return 'num_layers %d (supported: 1..%d)' % (layers, MAX_LAYERS)
    if mt not in ('concat', 'standard', 'manet'):
        return 'model_type %r' % mt
    if opt.input_encoding_size % 64 or opt.rnn_size % 64:
        return 'input_encoding_size / rnn_size must be multiples of 64'
    if layers > 1 and (mt != 'concat' or C != 1):
        return 'stacked layers need model_type concat without temporal attention'
    if mt == 'manet' and (C != 1 or len(getattr(opt, 'feat_dims', [])) > MANET_MAX_FEATS):
        return 'manet needs num_chunks 1 and at most %d modalities' % MANET_MAX_FEATS
    if C > 1 and (C > ATT_MAX_CHUNKS or mt != 'concat'):
        return 'temporal attention needs model_type concat and num_chunks <= %d' % ATT_MAX_CHUNKS
    return None


def engine_supports(opt):
    return engine_unsupported_reason(opt) is None


def gate_maps(rnn_type, H):
    """Packing of a cell's gate-major PyTorch weights (rows ``g*H + u``) into
    packed gate rows ``4u + slot``, for the input and the recurrent side:
    (src (4H,) PyTorch row of each packed row, ``G*H`` = a zero row;
    dst (G*H,) packed row of each PyTorch row; slot code for the Adam
    shadow pass, 2 bits per gate group, ``csrc/kernels/adam.hip``)."""
    _, G, slots_ie, slots_hh = CELLS[rnn_type]
    u = torch.arange(H)
    out = []
    for slots in (slots_ie, slots_hh):
        src = torch.full((H, 4), G * H, dtype=torch.long)
        dst = torch.empty(G * H, dtype=torch.long)
        for g, k in enumerate(slots):
            src[:, k] = g * H + u
            dst[g * H:(g + 1) * H] = 4 * u + k
        out.append((src.view(-1), dst, sum(k << (2 * g) for g, k in enumerate(slots))))
    return out


class _DecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, vgate, w_ih, w_hh, emb_w, logit_w, logit_b, att_gv, att_pre, att_wq,
                att_wa, att_ba, h0, c0, eng, labels, bos, R, T, modes, ss_prob, drop_p,
                temperature, rng, vdiv, want_xe, use_counts, use_unfinished, save, want_full,
                *up_w):
        has_att = att_gv is not None
        dev = logit_b.device
        att = []
        if has_att:
            att = [att_gv.detach().float().contiguous(), att_pre.detach().float().contiguous(),
                   eng.wq, att_wa.detach().float().contiguous().view(-1),
                   att_ba.detach().float().contiguous().view(-1)]
        vg_in = torch.empty(0, device=dev) if has_att else vgate.detach().float().contiguous()
        state0 = []
        if h0 is not None:  # bf16 h (the recurrent GEMM operand), fp32 c
            state0 = [h0.detach().bfloat16().contiguous(), c0.detach().float().contiguous()]
        store_exp = bool(save and not want_full)
        # XE all rows (csrc/engine.cpp): teacher forcing of a training forward
        # runs one launch per step (vocabulary tiles of step t + the whole LSTM
        # step t+1) with the combines on a side stream
        xe_rows = bool(store_exp and want_xe and labels is not None and not has_att
                       and not state0 and eng.layers == 1 and XE_ROWS and T <= 64
                       and all(m == SEL_GT for m in modes[:T - 1]))
        outs = _ext.ops().decoder_forward(
            eng.wx, eng.emb, eng.ptab, eng.whh_q if has_att else eng.whh, eng.wlog,
            logit_b.detach().float().contiguous(),
            vg_in, vdiv,
            labels if labels is not None else torch.empty(0, dtype=torch.long),
            bos if bos is not None else torch.empty(0, dtype=torch.long), R, T, modes, ss_prob,
            drop_p, temperature, rng, save, want_xe, use_counts, use_unfinished, att, eng.cell,
            state0, eng.upper_operands(), store_exp, xe_rows)
        ctx.xe_rows = xe_rows
        xw = torch.empty(0, device=dev)  # X = E W: engine.launch_x after the rollout
        seq, g_sel, g_xe, lse = outs[:4]
        ctx.save_dims = (R, T, vdiv, want_xe)
        # training rollouts save E = exp(logit - previous step's LSE) (bf16) for
        # the dS-free backward; the full log-prob API keeps fp16 logits
        ctx.store_exp = bool(save and not want_full)
        full = None
        if want_full:
            # full (R, T, V) log-probs for the model(feats, seq) API, from the
            # logits the backward keeps anyway (fp16) and the fp32 LSE
            V = logit_b.numel()
            full = (outs[4][:, :, :V].float() - lse.unsqueeze(2)).permute(1, 0, 2).contiguous()
        ctx.eng = eng
        ctx.drop_p, ctx.rng = drop_p, rng
        # the backward recomputes exp-store rows out of bf16 range from the
        # vocab input and the logit weights / bias (vocab_grad.hip vgrad_fix)
        ctx.logit_b = logit_b.detach().float().contiguous() if save else None
        ctx.shapes = (w_ih.shape, emb_w.shape)
        ctx.has_att = has_att
        ctx.state0 = state0 if save else []
        # the video-gate node that produced THIS call's vgate (ops/featpool.py
        # VgHandoff: matched by the tensor's identity; any other pending
        # hand-off is dropped here)
        vg_pending = eng.__dict__.pop('_vg_pending', None)
        ctx.vg_ctx = (vg_pending if (save and not has_att and not state0 and vg_pending is not None
                                     and vg_pending.matches(vgate)) else None)
        ctx.att_saved = None
        ctx.xw_late = None
        if save:
            ctx.saved = (lse, *outs[4:9], seq, labels, bos, xw)
            if ctx.store_exp and eng.x_after_rollout and xw.numel() == 0:
                eng._x_pending = ctx  # launch_x computes X = E W for this forward
            if has_att:  # Gv, P, W_q, w_a, alpha_all, q_all, u_all (fp16 scorer values)
                ctx.att_saved = (att[0], att[1], att[2], att[3], outs[9], outs[10], outs[11])
            ctx.up_saved = outs[12 if has_att else 9:]  # (h, c, gates, hd_in) per upper layer
        else:
            ctx.saved = None
        ctx.att_shapes = (att_wa.shape, att_ba.shape) if has_att else None
        ctx.mark_non_differentiable(seq)
        if g_xe is None:
            g_xe = torch.zeros(0, device=g_sel.device)
        if full is None:
            full = torch.zeros(0, device=g_sel.device)
        return seq, g_sel, g_xe, full

    @staticmethod
    def backward(ctx, dseq, dg_sel, dg_xe, dfull):
        if ctx.saved is None:
            raise RuntimeError('decoder forward ran without saving activations')
        R, T, vdiv, want_xe = ctx.save_dims
        eng = ctx.eng
        if eng._x_pending is ctx:  # never handed to launch_x: do not keep ctx alive
            eng._x_pending = None
        lse, logits16, hdrop, gates, c_all, h_all, seq, labels, bos, xw = ctx.saved
        x_ev = None
        if ctx.xw_late is not None:  # X = E W launched after the rollout (launch_x)
            xw, x_ev = ctx.xw_late
            ctx.xw_late = None
        ctx.saved = None  # (the fp16-logits buffer is overwritten in place by dS)
        att = list(ctx.att_saved) if ctx.has_att else []
        ctx.att_saved = None
        g_sel = dg_sel.contiguous() if dg_sel is not None else None
        g_xe = dg_xe.contiguous() if (want_xe and dg_xe is not None and dg_xe.numel()) else None
        empty = torch.empty(0, device=lse.device)
        n_steps = logits16.shape[0]
        ds_bias = empty
        if not ctx.store_exp:
            # fp16 logits saved (full log-prob API): dense dS = G - p * sum_v G,
            # G = the gradient w.r.t. the full log-probs (+ the gathered terms),
            # written as bf16 into the logits buffer
            V = logit_b_numel = eng.V
            n_sel = g_sel.size(1) if g_sel is not None else 0
            # (n, R, V); a private dense copy: the incoming gradient may be an
            # expanded view (e.g. of full.sum()) or shared with other nodes
            if dfull is not None and dfull.numel():
                G = dfull.permute(1, 0, 2).float().clone(memory_format=torch.contiguous_format)
            else:
                G = torch.zeros(n_steps, R, V, device=lse.device)
            if g_sel is not None:
                G[:n_sel].scatter_add_(2, seq.t()[:n_sel].unsqueeze(2), g_sel.t().unsqueeze(2))
            if g_xe is not None:
                tgt = labels[:, 1:1 + n_steps].t().unsqueeze(2)
                G.scatter_add_(2, tgt, g_xe.t()[:n_steps].unsqueeze(2))
            p = torch.exp(logits16[:, :, :V].float() - lse.unsqueeze(2))
            dS = G - p * G.sum(2, keepdim=True)
            logits16.view(torch.bfloat16)[:, :, :V].copy_(dS)
            ds_bias = dS.to(torch.bfloat16).float().sum((0, 1))
            del G, p, dS
            g_sel = g_xe = None
            del logit_b_numel
        # input token of every step: it_0 = BOS / labels[:, 0], it_t = seq[:, t-1]
        first = labels[:, :1] if labels is not None else bos.view(-1, 1)
        toks = torch.cat([first, seq[:, :n_steps - 1]], 1).t().reshape(-1)
        # the vocab-head weight gradients go straight into their flat-bucket
        # slots (no autograd accumulate pass over the V x H gradient); under
        # data parallelism the backward also marks them final with an event
        # (engine set_grad_events), for the comm stream (parallel/dist.py)
        direct = getattr(eng, 'direct_grad_slots', None)
        if direct is not None:
            eng.check_direct_slots()
        if direct is not None:
            out_w, out_b, comm = direct['wlog'], direct['blog'], 0
        else:
            out_w, out_b, comm = empty, empty, 0
        # embedding / LSTM weight slots: written here instead of returned, which
        # saves autograd's zero-fill + accumulate passes over them.  The video
        # columns of W_ih still arrive through autograd (the gate-table path),
        # and add onto these disjoint token columns in either order.
        emb_direct = direct is not None and 'emb' in direct
        out_emb = direct['emb'] if emb_direct else empty
        # concat model with direct slots: the video-gate / FeatPool backward
        # and the W_ih / W_hh row unpacking run inside the engine, right after
        # the reverse loop (third streamed DP slice)
        vg_bwd, vg_nf, vg_p = [], 0, 0.0
        vg_ctx, ctx.vg_ctx = getattr(ctx, 'vg_ctx', None), None
        if (vg_ctx is not None and emb_direct and 'fp_w0' in direct and eng.layers == 1
                and not ctx.state0 and eng.wiv is not None):
            fc, xs, wsd, vg_p, vg_nf = vg_ctx.payload
            vg_bwd = ([eng.dst_ie, eng.dst_hh, direct['wih'], direct['whh'], eng.wiv, fc]
                      + [direct['fp_w%d' % f] for f in range(vg_nf)]
                      + [direct['fp_b%d' % f] for f in range(vg_nf)] + list(xs) + list(wsd))
        # the operand preparation above (token rows, contiguous gradients)
        # needs no X; it runs while the X stream still computes (3.362-3.402
        # vs 3.400-3.418 ms per step waiting first, profiles/r5/tail/), and so
        # does the backward's own X-independent prologue: the native call
        # waits for X itself (x_wait: the raw event handle)
        res = _ext.ops().decoder_backward(
            eng.wx, eng.wlog, eng.emb, lse, logits16, hdrop, gates, c_all, h_all, seq,
            labels if labels is not None else torch.empty(0, dtype=torch.long, device=lse.device),
            toks, g_sel if g_sel is not None else empty, g_xe if g_xe is not None else empty,
            ctx.drop_p, ctx.rng, out_w, out_b, comm, att, out_emb, ds_bias, eng.cell,
            ctx.state0, eng.upper_operands(ctx.up_saved), ctx.logit_b, eng.exp_fix_rows,
            vdiv, xw if ctx.store_exp else empty, vg_bwd, vg_nf, float(vg_p),
            0 if x_ev is None else int(x_ev.cuda_event), ctx.xe_rows)
        ctx.logit_b = None
        ctx.up_saved = None
        d_up = []
        if eng.layers > 1:  # packed [W_ih | W_hh] of each upper layer
            H = eng.H
            for dwu in res[len(res) - (eng.layers - 1):]:
                d_up += [dwu[:, :H].index_select(0, eng.dst_ie),
                         dwu[:, H:].index_select(0, eng.dst_hh)]
            res = res[:len(res) - (eng.layers - 1)]
        d_state = (None, None)
        if ctx.state0:
            d_state = (res[-2], res[-1])  # through W_hh, and the state carry
            res = res[:-2]
        ctx.state0 = []
        dWx, dWlog, dblog, d_emb, dvg = res[:5]
        if direct is not None:
            dWlog = dblog = None  # already in the gradient buffers
        if emb_direct:
            d_emb = None
        E = eng.E
        # packed gate rows -> the PyTorch weights' rows (unused slots dropped)
        if not vg_bwd:
            d_ie = dWx[:, :E].index_select(0, eng.dst_ie)
            d_hh = dWx[:, E:].index_select(0, eng.dst_hh)
        w_ih_shape, emb_shape = ctx.shapes
        if vg_bwd:  # (written by the engine)
            d_wih = d_whh = None
            vg_ctx.done = True  # the video-gate node's own backward is a no-op
        elif emb_direct:
            direct['wih'][:, :E].copy_(d_ie)
            direct['whh'].copy_(d_hh)
            d_wih = d_whh = None
        else:
            d_wih = torch.zeros(w_ih_shape, dtype=torch.float32, device=dWx.device)
            d_wih[:, :E] = d_ie
            d_whh = d_hh
        if ctx.has_att:
            d_gv, d_pre, d_wa, d_ba, d_wq = res[5:10]
            d_wa, d_ba = d_wa.view(ctx.att_shapes[0]), d_ba.view(ctx.att_shapes[1])
            return (None, d_wih, d_whh, d_emb, dWlog, dblog, d_gv, d_pre, d_wq, d_wa,
                    d_ba) + (None,) * 18
        d_vgate = dvg  # (R // vdiv, 4H): summed over steps and each video's rows
        return (d_vgate, d_wih, d_whh, d_emb, dWlog, dblog) + (None,) * 5 + d_state + \
            (None,) * 16 + tuple(d_up)


_AUX = {}


def _device_aux(dev):
    """Per-device side streams and events of the engine (token-table prefetch,
    X = E W after the rollout), created once."""
    import types
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _AUX:
        _AUX[key] = types.SimpleNamespace(
            ptab_stream=torch.cuda.Stream(device=dev), ptab_ev0=torch.cuda.Event(),
            ptab_ev1=torch.cuda.Event(), x_stream=torch.cuda.Stream(device=dev),
            x_ev0=torch.cuda.Event(), x_ev1=torch.cuda.Event(), x_pending={})
    return key


class DecoderEngine:
    @property
    def _aux(self):
        return _AUX[self._aux_key] if self._aux_key is not None else None

    @property
    def _x_pending(self):
        return self._aux.x_pending.get(id(self)) if self._aux is not None else None

    @_x_pending.setter
    def _x_pending(self, ctx):
        if self._aux is not None:
            self._aux.x_pending[id(self)] = ctx

    def __init__(self, model, opt):
        why = engine_unsupported_reason(opt)
        if why is not None:
            raise ValueError('fused engine: unsupported configuration: ' + why)
        if not _ext.available():
            raise RuntimeError('HIP extension not available')
        self.H = model.rnn_size
        self.E = model.input_encoding_size
        self.V = model.vocab_size
        self.manet = getattr(model, 'model_type', 'concat') == 'manet'
        # the attention kernels run temporal attention and MANet
        self.attention = getattr(model, 'num_chunks', 1) > 1 or self.manet
        self.standard = getattr(model, 'model_type', 'concat') == 'standard'
        dev = model.embed.weight.device
        H, E, V = self.H, self.E, self.V
        self.cell, G, _, _ = CELLS[model.rnn_type]
        self.gates = G
        (self.src_ie, self.dst_ie, self.slots_ie), (self.src_hh, self.dst_hh, self.slots_hh) = \
            [(a.to(dev), b.to(dev), c) for a, b, c in gate_maps(model.rnn_type, H)]
        self.model = model
        # bf16 shadow weights read by the kernels.  Persistent buffers, updated
        # IN PLACE (by the fused Adam pass, or refresh_weights()), so a captured
        # HIP graph always reads the live weights.
        A = 0
        if self.manet:  # scorer width F, zero-padded to the 64-row GEMM tile
            A = (model.num_feats + 63) // 64 * 64
        elif self.attention:
            A = model.temporal_att.f_h.weight.size(0)
        self.att_dim = A
        bf = dict(dtype=torch.bfloat16, device=dev)
        self.wx = torch.empty(4 * H, E + H, **bf)       # [W_ie | W_hh], packed gate rows
        self.whh_q = torch.empty(4 * H + A, H, **bf)    # [W_hh; W_q] (recurrent GEMM operand)
        self.whh = self.whh_q[:4 * H]
        self.wq = self.whh_q[4 * H:] if self.attention else None
        self.emb = torch.empty(V, E, **bf)
        self.wlog = torch.empty(V, H, **bf)
        # W_ih's video columns in packed gate rows (zero rows in unused gate
        # slots): the operand of the per-video gate term vg = fc W_iv^T and of
        # its backward dfc = dvg W_iv, written by the fused Adam pass like the
        # other shadows (no per-step conversion)
        fv = model.core.rnn.weight_ih_l0.size(1) - E
        self.wiv = torch.zeros(4 * H, fv, **bf) if fv > 0 and not self.standard else None
        # (fp16: the decode's cell epilogue gathers one row per caption row and
        # step; half the bytes of fp32, 11 significant bits for these O(1)
        # gate pre-activation terms)
        self.ptab = torch.empty(V, 4 * H, dtype=torch.float16, device=dev)
        # upper layers of a stacked decoder: packed [W_ih_l | W_hh_l] and a
        # contiguous copy of W_hh_l (the step kernel's B operand)
        self.layers = getattr(model, 'num_layers', 1)
        self.wup = [torch.empty(4 * H, 2 * H, **bf) for _ in range(self.layers - 1)]
        self.whh_up = [torch.empty(4 * H, H, **bf) for _ in range(self.layers - 1)]
        self.fused_refresh = False  # True once an optimizer writes the shadows
        # the input-token gate table is refreshed lazily: after_step() only
        # bumps weights_version; the next training step computes the table on
        # a side stream under its prologue (prefetch_ptab), every other user
        # recomputes a stale table first (ensure_ptab)
        self.weights_version = 0
        self._ptab_version = -1
        self._ptab_pending = False  # this step's prefetch is in flight (aux.ptab_ev1)
        # side streams / events (created here, never during a graph capture;
        # kept outside the instance so a deepcopy of the model stays possible)
        self._aux_key = _device_aux(dev) if dev.type == 'cuda' else None
        # running count of exp-store rows the backward recomputed because the
        # row's LSE jumped by > 60 between steps (csrc/kernels/vocab_grad.hip)
        self.exp_fix_rows = torch.zeros(1, dtype=torch.int32, device=dev)
        # X = E W after the rollout (launch_x): the trainer enables it for RL
        # steps and calls launch_x right after the rollout is enqueued; the
        # GEMM runs on the engine's own x_stream
        self.x_after_rollout = False
        self.direct_grad_slots = None
        self.direct_params = None
        self.direct_armed = False
        self.refresh_weights()

    # -- bf16 shadow weights ------------------------------------------------------
    def shadow_spec(self, bucket):
        """Shadow-copy segments of the flat parameter buffer for the fused
        Adam pass: (int64 CPU meta (n, 8), [dst, dst2] * n).  The fused pass
        never writes the unused (zero) gate slots."""
        m = self.model
        slot = {id(p): (off, n) for p, (off, n) in zip(bucket.params, bucket.slices)}
        rnn = m.core.rnn
        H, E = self.H, self.E
        empty = torch.empty(0, dtype=torch.bfloat16, device=self.wx.device)
        segs = [(m.logit.weight, 0, 0, self.wlog, empty, 0, 0, E),
                (m.embed.weight, 0, 0, self.emb, empty, 0, 0, E),
                (rnn.weight_ih_l0, 1, rnn.weight_ih_l0.size(1), self.wx,
                 empty if self.wiv is None else self.wiv,
                 0 if self.wiv is None else self.wiv.size(1), self.slots_ie, E),
                (rnn.weight_hh_l0, 2, H, self.wx, self.whh_q, H, self.slots_hh, E)]
        if self.attention:  # (MANet: the first F rows of the padded W_q)
            segs.append((self._query_weight(), 0, 0, self.wq, empty, 0, 0, E))
        for k in range(1, self.layers):  # packed [W_ih_k | W_hh_k]: "E" = H
            segs += [(getattr(rnn, 'weight_ih_l%d' % k), 1, H, self.wup[k - 1], empty, 0,
                      self.slots_ie, H),
                     (getattr(rnn, 'weight_hh_l%d' % k), 2, H, self.wup[k - 1],
                      self.whh_up[k - 1], H, self.slots_hh, H)]
        meta, dsts = [], []
        for p, kind, cols, d, d2, ld2, slots, e in segs:
            off, n = slot[id(p)]
            meta.append([off, n, kind, cols, H, e, ld2, slots])
            dsts += [d, d2]
        return torch.tensor(meta, dtype=torch.int64), dsts

    @torch.no_grad()
    def refresh_weights(self):
        """Rewrite every shadow from the fp32 parameters (after init or a
        checkpoint load; the optimizer keeps them fresh during training)."""
        m = self.model
        E = self.E
        w_ih = m.core.rnn.weight_ih_l0
        w_hh = m.core.rnn.weight_hh_l0
        self.wx[:, :E].copy_(self.pack_rows(w_ih[:, :E], self.src_ie))
        self.wx[:, E:].copy_(self.pack_rows(w_hh, self.src_hh))
        self.whh.copy_(self.wx[:, E:])
        if self.wiv is not None:
            self.wiv.copy_(self.pack_rows(w_ih[:, E:], self.src_ie))
        self.emb.copy_(m.embed.weight)
        self.wlog.copy_(m.logit.weight)
        if self.attention:
            q = self._query_weight()
            self.wq.copy_(F.pad(q, (0, 0, 0, self.att_dim - q.size(0))))
        H = self.H
        for k in range(1, self.layers):
            rnn = m.core.rnn
            self.wup[k - 1][:, :H].copy_(self.pack_rows(getattr(rnn, 'weight_ih_l%d' % k),
                                                        self.src_ie))
            self.wup[k - 1][:, H:].copy_(self.pack_rows(getattr(rnn, 'weight_hh_l%d' % k),
                                                        self.src_hh))
            self.whh_up[k - 1].copy_(self.wup[k - 1][:, H:])
        self.update_ptab()

    @staticmethod
    def pack_rows(w, src, dim=0):
        """rows (``dim``) of a gate-major PyTorch tensor in packed gate order,
        zeros in the unused slots (differentiable)"""
        pad = [0, 0] * (w.dim() - 1 - dim % w.dim()) + [0, 1]
        return F.pad(w, pad).index_select(dim, src)

    @torch.no_grad()
    def update_ptab(self):
        # input-token gate table P = emb . W_ie^T (V x 4H, packed gate order):
        # one GEMM per optimizer step instead of K=E of work in every decode step
        if self.emb.is_cuda:
            # the measured hipBLASLt choice (host/blaslt_tuned.cpp): PyTorch's
            # pick ran this 22 GFLOP product at 0.27 PF/s (81 us,
            # profiles/r6/steps_xe_after_fixes.txt)
            p32 = torch.empty(self.ptab.shape, dtype=torch.float32, device=self.emb.device)
            _ext.ops().gemm_bf16_tuned(p32, self.emb, False, self.wx[:, :self.E], True)
            self.ptab.copy_(p32)
        else:
            self.ptab.copy_(torch.mm(self.emb, self.wx[:, :self.E].t(), out_dtype=torch.float32))
        self._ptab_version = self.weights_version

    def prefetch_ptab(self):
        """Start of a training step: a stale table is recomputed on a side
        stream, concurrently with the step's batch gather / FeatPool prologue
        (the decode waits for it in ensure_ptab).  Graph-capturable: the fork
        and the join are both inside the captured step."""
        if self._ptab_version == self.weights_version or self._aux is None:
            return
        main = torch.cuda.current_stream(self.ptab.device)
        self._aux.ptab_ev0.record(main)
        self._aux.ptab_stream.wait_event(self._aux.ptab_ev0)
        with torch.cuda.stream(self._aux.ptab_stream):
            self.update_ptab()
            self._aux.ptab_ev1.record(self._aux.ptab_stream)
        self._ptab_pending = True

    def ensure_ptab(self):
        """Before a decode reads the table: join this step's prefetch, or
        recompute a stale table on the current stream."""
        if self._ptab_version != self.weights_version:
            self.update_ptab()
        elif self._ptab_pending:
            torch.cuda.current_stream(self.ptab.device).wait_event(self._aux.ptab_ev1)

    def current_ptab(self):
        self.ensure_ptab()
        return self.ptab

    def attach_optimizer(self, trainer):
        """The trainer's flat Adam writes the bf16 shadows in its update pass."""
        opt = trainer.optimizer
        if getattr(opt, 'supports_shadows', False):
            opt.set_shadows(*self.shadow_spec(trainer.bucket))
            self.fused_refresh = True
        self.refresh_weights()  # params were re-homed into the flat buffer

    def after_step(self):
        """The weights changed (an optimizer step ran, eagerly or inside a
        replayed graph): the gate table is stale from here on."""
        self.weights_version += 1
        self._ptab_pending = False
        if not self.fused_refresh:
            self.refresh_weights()

    def invalidate_ptab(self):
        """Mark the gate table stale: a graph captured next then always holds
        its refresh (prefetch_ptab), whatever an eval just computed."""
        self._ptab_version = -1
        self._ptab_pending = False

    def launch_x(self, stream=None):
        """X = E W of the last training forward (the vocab head's backward GEMM
        without the one-hot terms; see csrc/engine.cpp "X in the rollout") on
        ``stream``, after the rollout: the GEMM then runs while the rewards
        and the loss are computed, and the backward's reverse loop reads
        alpha X + the one-hot rows instead of waiting for the GEMM.  No-op
        unless a forward left one pending."""
        ctx, self._x_pending = self._x_pending, None
        if ctx is None or ctx.saved is None:
            return
        if stream is None:
            stream = self._aux.x_stream
        logits16 = ctx.saved[1]
        n, R, ldl = logits16.shape
        main = torch.cuda.current_stream(logits16.device)
        # allocated on the main stream, which waits for the GEMM (backward)
        # before anything else touches it or frees it, like the exp store
        xw = torch.empty(n, R, self.H, dtype=torch.float32, device=logits16.device)
        self._aux.x_ev0.record(main)  # the rollout (enqueued before this call) is done
        stream.wait_event(self._aux.x_ev0)
        with torch.cuda.stream(stream):
            _ext.ops().vocab_x(logits16, self.wlog, xw)
            from ..utils import stamps
            stamps.mark('x_end')
            self._aux.x_ev1.record(stream)
        ctx.xw_late = (xw, self._aux.x_ev1)

    # -- gradient slots written by the fused backward -------------------------------
    def set_direct_slots(self, slots, params):
        self.direct_grad_slots = slots
        self.direct_params = params
        self.direct_armed = True

    def arm_direct_slots(self):
        self.direct_armed = True

    def check_direct_slots(self):
        """The fused backward OVERWRITES the gradient slots: one backward per
        zero_grad(), and the slots must still be the parameters' .grad."""
        if not self.direct_armed:
            raise RuntimeError('second fused backward before the gradient bucket was zeroed: '
                               'direct gradient slots would be overwritten')
        for k, slot in self.direct_grad_slots.items():
            g = self.direct_params[k].grad
            if g is None or g.data_ptr() != slot.data_ptr():
                raise RuntimeError('parameter %r no longer has its flat-bucket slot as .grad '
                                   '(zero_grad(set_to_none=True) or a replaced .grad?); use the '
                                   'trainer bucket\'s zero_grad()' % k)
        self.direct_armed = False
        self._video_slots_ok = True

    def take_video_slots(self):
        """For the FeatPool / video-gate backward of the same pass (it runs
        after the decoder's): the direct slots, once, if the decoder backward
        verified them and the FeatPool parameters have slots too."""
        ok = getattr(self, '_video_slots_ok', False)
        self._video_slots_ok = False
        d = self.direct_grad_slots
        if not ok or d is None or 'fp_w0' not in d:
            return None
        return d

    def _rng(self, dev):
        # per-pass seeds {dropout, sampling} drawn ON the device (graph-safe:
        # a replayed graph advances the generator's offset)
        return torch.randint(0, 2 ** 31 - 1, (2,), dtype=torch.int32, device=dev)

    @staticmethod
    def _encode(model, feats):
        """FeatPool through the fused kernels (ops/featpool.py) when they
        cover the configuration, else the PyTorch module."""
        from ..ops.featpool import featpool, fused_ok
        if fused_ok(model.feat_pool, feats):
            return featpool(model.feat_pool, feats)
        return model.encode(feats)

    def _initial_state(self, model, feats):
        """model_type 'standard': one cell step per video on the video vector
        from a zero state (plain autograd ops, so it captures in a HIP graph;
        W_hh does not enter it).  Returns (h0, c0) per video, c0 = h0 for
        GRU / RNN (the kernels' state buffer)."""
        fc = self._encode(model, feats)  # (B, E), FeatPool dropout in train mode
        a = F.linear(fc, model.core.rnn.weight_ih_l0)
        if self.cell == 0:  # LSTM i, f, g, o with c' = 0
            i, _, g, o = a.chunk(4, 1)
            c = torch.sigmoid(i) * torch.tanh(g)
            return torch.sigmoid(o) * torch.tanh(c), c
        if self.cell == 1:  # GRU r, z, n with h' = 0
            _, z, n = a.chunk(3, 1)
            h = (1 - torch.sigmoid(z)) * torch.tanh(n)
        else:
            h = torch.tanh(a)
        return h, h

    def _vgate(self, model, feats, expand):
        if self.standard:  # no per-step video term
            B = feats[0].size(0)
            return model.logit.bias.new_zeros(B, 4 * self.H), B
        from ..ops.featpool import featpool_vgate, fused_ok
        if fused_ok(model.feat_pool, feats) and feats[0].size(1) == 1:
            vg = featpool_vgate(self, model, feats)  # one node: FeatPool + gate term
            return vg, vg.size(0)
        fc = self._encode(model, feats)  # (B, F*H), FeatPool dropout in train mode
        w_iv = model.core.rnn.weight_ih_l0[:, self.E:]
        vg = F.linear(fc, w_iv)
        return self.pack_rows(vg, self.src_ie, 1), fc.size(0)

    def upper_operands(self, saved=None):
        """Upper-layer operands of the native calls: forward / beam
        {[W_ih | W_hh], W_hh} per layer; backward {[W_ih | W_hh], h, c, gates,
        hd_in} per layer from the forward's saved tensors."""
        out = []
        for k in range(self.layers - 1):
            if saved is None:
                out += [self.wup[k], self.whh_up[k]]
            else:
                out += [self.wup[k], *saved[4 * k:4 * k + 4]]
        return out

    def _query_weight(self):
        m = self.model
        return m.manet.f_h_m.weight if self.manet else m.temporal_att.f_h.weight

    def _manet_inputs(self, model, feats):
        """MANet as attention over the F modality blocks (module docstring)."""
        x = self._encode(model, feats)  # (B, F*blk), FeatPool dropout in train mode
        B, Fm = x.size(0), model.num_feats
        blk = x.size(1) // Fm
        w_iv = model.core.rnn.weight_ih_l0[:, self.E:]
        gv = torch.einsum('bfk,gfk->bfg', x.view(B, Fm, blk), w_iv.view(-1, Fm, blk))
        gv = self.pack_rows(gv, self.src_ie, 2)
        mn, pad = model.manet, self.att_dim - Fm
        p = F.pad(mn.f_feat_m(x) + mn.f_h_m.bias, (0, pad))
        pre = p.unsqueeze(1).expand(B, Fm, self.att_dim)
        wq = F.pad(mn.f_h_m.weight, (0, 0, 0, pad))
        wa = F.pad(mn.align_m.weight, (0, pad))
        return (gv, pre, wq, wa, mn.align_m.bias), B

    def _att_inputs(self, model, feats):
        """Per-batch attention operands: per-frame gate table Gv (B, C, 4H)
        in packed gate order, projected frames P (B, C, A), and the scorer
        parameters (W_q, w_a, b_a) as autograd inputs of the Function."""
        if self.manet:
            return self._manet_inputs(model, feats)
        ta = model.temporal_att
        from ..ops.featpool import att_inputs, fused_ok
        if fused_ok(model.feat_pool, feats) and feats[0].dim() == 3:
            # one node: FeatPool + one bf16 GEMM for Gv and P (ops/featpool.py;
            # att8 4.597 / 4.584 vs 4.776 / 4.780 ms per step with the two fp32
            # Linears below and their autograd backward, profiles/r5/README_r5.md)
            gv, pre = att_inputs(self, model, feats)
            return (gv, pre, ta.f_h.weight, ta.align.weight.view(-1), ta.align.bias), gv.size(0)
        frames = self._encode(model, feats)  # (B, C, F*H), FeatPool dropout in train mode
        w_iv = model.core.rnn.weight_ih_l0[:, self.E:]
        # (fp32 GEMMs here: under bf16 autocast -- bf16 gradients too -- the
        # projected frames' bias gradient drifted to 8.8 % of the fp32
        # reference at H = 64, tests/test_gpu_attention.py; the fused node
        # keeps the gradients fp32 and rounds only the GEMM operands)
        gv = self.pack_rows(F.linear(frames, w_iv), self.src_ie, 2)
        pre = ta.precompute(frames)
        return (gv, pre, ta.f_h.weight, ta.align.weight.view(-1), ta.align.bias), frames.size(0)

    def _run(self, model, feats, labels, modes, want_xe, use_counts, use_unfinished,
             expand=True, ss_prob=0.0, drop=True, temperature=1.0, bos_rows=None,
             want_full=False, rows_per_video=None):
        if self.attention:
            att, B = self._att_inputs(model, feats)
            vg = None
        else:
            vg, B = self._vgate(model, feats, expand)
            att = (None,) * 5
        from ..utils import stamps
        stamps.mark_fwd('vgate')
        S = rows_per_video or (model.feat_expander.n if expand else 1)
        h0 = c0 = None
        if self.standard:
            h0, c0 = self._initial_state(model, feats)
            if S > 1:
                h0, c0 = h0.repeat_interleave(S, 0), c0.repeat_interleave(S, 0)
        R = labels.size(0) if labels is not None else B * S
        if labels is not None:
            T = labels.size(1) - 1
            bos = None
        else:
            T = model.seq_length - 1
            bos = torch.full((R,), BOS, dtype=torch.long, device=model.logit.bias.device)
        drop_p = model.drop_prob_lm if (model.training and drop) else 0.0
        m = model
        ws = (m.core.rnn.weight_ih_l0, m.core.rnn.weight_hh_l0, m.embed.weight, m.logit.weight,
              m.logit.bias)
        ups = []
        for k in range(1, self.layers):
            ups += [getattr(m.core.rnn, 'weight_ih_l%d' % k), getattr(m.core.rnn, 'weight_hh_l%d' % k)]
        # (inside Function.forward grad mode is off, so decide here)
        diff_in = [t for t in (vg, h0, c0) + tuple(att) if t is not None] + list(ws) + ups
        save = want_full or (torch.is_grad_enabled() and any(t.requires_grad for t in diff_in))
        self.ensure_ptab()
        return _DecoderFn.apply(vg, *ws, *att, h0, c0, self,
                                labels.contiguous() if labels is not None else None, bos, R, T,
                                modes, float(ss_prob), float(drop_p), float(temperature),
                                self._rng(m.logit.bias.device), S, want_xe, use_counts,
                                use_unfinished, save, want_full, *ups)

    # -- public entry points ------------------------------------------------------
    def rollout(self, model, feats, labels):
        """Reference ``forward(feats, seq)`` for RL: returns
        (sample_seq (R, T-1), sample_logprobs (R, T-1), None)."""
        T = labels.size(1) - 1
        modes = self._modes(model, T)
        mask_eos = getattr(model, 'mask_after_eos', False)
        seq, g_sel, _, _ = self._run(model, feats, labels, modes, want_xe=False, use_counts=True,
                                     use_unfinished=mask_eos, ss_prob=model.ss_prob)
        return seq, g_sel, None

    def teacher_forced(self, model, feats, labels):
        """Gathered log-probs of the GT targets ``labels[:, 1:]`` (R, T) --
        what CrossEntropyCriterion needs.  Honours scheduled sampling."""
        T = labels.size(1) - 1
        modes = self._modes(model, T, rl=False)
        _, _, g_xe, _ = self._run(model, feats, labels, modes, want_xe=True, use_counts=True,
                                  use_unfinished=False, ss_prob=model.ss_prob)
        return g_xe

    def _modes(self, model, T, rl=True):
        modes = []
        for t in range(T - 1):
            tok_idx = t + 1
            if model.training and model.ss_prob > 0.0:
                modes.append(SEL_SS)
            elif rl and model.training and model.mixer_from > 0 and tok_idx >= model.mixer_from:
                modes.append(SEL_SAMPLE)
            else:
                modes.append(SEL_GT)
        return modes

    def forward_full(self, model, feats, seq):
        """Reference ``forward(feats, seq)`` (``model.py:218-289``) on the
        engine: (log-probs (R, T, V), sample_seq (R, T-1), sample_logprobs
        (R, T-1)) with teacher forcing / scheduled sampling / MIXER sampling as
        the model's setters select.  The log-probs are the kernels' logits
        (kept in fp16 for the backward) minus the fp32 LSE; gradients w.r.t.
        them flow through the fused backward as a dense dS.  Difference: when
        every row has emitted EOS the reference stops early; here the
        remaining steps are computed on EOS inputs (tokens stay 0)."""
        T = seq.size(1) - 1
        modes = self._modes(model, T)
        mask_eos = getattr(model, 'mask_after_eos', False)
        s_seq, g_sel, _, full = self._run(model, feats, seq, modes, want_xe=True,
                                          use_counts=True, use_unfinished=mask_eos,
                                          ss_prob=model.ss_prob, want_full=True)
        return full, s_seq, g_sel

    @torch.no_grad()
    def sample(self, model, feats, opt):
        sample_max = opt.get('sample_max', 1)
        temperature = opt.get('temperature', 1.0)
        expand = opt.get('expand_feat', 0) == 1
        T = model.seq_length - 1
        modes = [SEL_GREEDY if sample_max == 1 else SEL_SAMPLE] * (T - 1)
        # (temporal attention, one greedy row per video: decoding each video on
        # two identical rows so the decode launch's MFMA attention applies
        # measured slower, 5.317 vs 5.197 ms per att8 step -- the doubled
        # greedy vocabulary work slows the concurrent sampled rollout,
        # profiles/r4/README_r4.md)
        seq, lp, _, _ = self._run(model, feats, None, modes, want_xe=False, use_counts=False,
                                  use_unfinished=True, expand=expand, drop=False,
                                  temperature=temperature)
        return seq, lp

    def _att_mfma_shape_ok(self, model):
        """The MFMA attention's shape limits (csrc/kernels/vocab.hip
        att_mfma_ok, shared scorer): frames <= 16, A % 64 == 0 and <= 1024,
        64 <= H <= 512 with H % 32 == 0."""
        C = getattr(model, 'num_chunks', 1)
        A, H = self.att_dim, self.H
        return 1 <= C <= 16 and A % 64 == 0 and A <= 1024 and H % 32 == 0 and 64 <= H <= 512

    @torch.no_grad()
    def sample_beam(self, model, feats, opt):
        """Batched on-GPU beam search (``csrc/kernels/beam.hip``) with the
        reference's selection / harvesting / perplexity-ranking semantics
        (``model.py:369-512``)."""
        K = opt.get('beam_size', 5)
        if K > 16:
            model.impl = 'torch'
            try:
                return model.sample_beam(feats, opt)
            finally:
                model.impl = 'hip'
        att = []
        if self.attention:
            (gv, pre, _, wa, ba), _ = self._att_inputs(model, feats)
            att = [gv.float().contiguous(), pre.float().contiguous(), self.wq,
                   wa.float().contiguous(), ba.float().contiguous()]
            vg = gv[:, 0]  # only its row count is read when attention is on
        else:
            vg, _ = self._vgate(model, feats, False)
        state0 = []
        if self.standard:
            h0, c0 = self._initial_state(model, feats)
            state0 = [h0.bfloat16().contiguous(), c0.float().contiguous()]
        self.ensure_ptab()
        blog = model.logit.bias.detach().float().contiguous()
        vg = vg.detach().float().contiguous()
        if (not state0 and self.layers == 1 and vg.is_cuda
                and os.environ.get('CSTCAP_BEAM_GRAPH', '1') != '0'
                and not torch.cuda.is_current_stream_capturing()):
            return self._beam_graphed(vg, blog, K, model.seq_length, att)
        seq, lp = _ext.ops().beam_search(self.wx, self.ptab, self.whh, self.wlog, blog, vg, K,
                                         model.seq_length, BOS, att, self.cell, state0,
                                         self.upper_operands())
        return seq, lp

    def _beam_graphed(self, vg, blog, K, T, att=()):
        """The whole beam decode (T-1 steps) replayed as one captured HIP
        graph per (shapes, K, T): the weights are the engine's persistent
        shadows (updated in place); the video gates, the fp32 logit bias and
        the per-batch attention operands (Gv, P, w_a, b_a; W_q is a shadow)
        are copied into the graph's own static buffers before each replay (the
        caller's tensors may be fresh temporaries, so the graph never reads
        the caller's memory), the outputs cloned out."""
        att = list(att)
        dyn = [i for i, t in enumerate(att) if t is not self.wq]  # per-call operands
        key = (tuple(vg.shape), tuple(blog.shape), int(K), int(T),
               tuple(tuple(t.shape) for t in att))
        cache = self.__dict__.setdefault('_beam_graphs', {})
        ent = cache.get(key)
        if ent is None:
            if len(cache) >= 4:
                cache.clear()
            static_vg, static_b = vg.clone(), blog.clone()
            static_att = [t.clone() if i in dyn else t for i, t in enumerate(att)]
            args = lambda: (self.wx, self.ptab, self.whh, self.wlog, static_b, static_vg, K, T,
                            BOS, static_att, self.cell, [], [])
            _ext.ops().beam_search(*args())  # (kernel attributes, allocator, outside capture)
            torch.cuda.synchronize(vg.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = _ext.ops().beam_search(*args())
            ent = cache[key] = (g, static_vg, static_b, static_att, out)
        g, static_vg, static_b, static_att, out = ent
        static_vg.copy_(vg)
        static_b.copy_(blog)
        for i in dyn:
            static_att[i].copy_(att[i])
        g.replay()
        return out[0].clone(), out[1].clone()
