"""Fused FeatPool (``csrc/kernels/featpool.hip``): every modality's
``Linear -> ReLU -> Dropout`` and the concat in two launches forward and one
backward, for the fused decoder engine (the PyTorch path keeps
:class:`~cst_captioning_amd.models.modules.FeatPool`).

Reference: ``/root/reference/model.py:46-69``.  Same function, parameters
and fp32 operands (split into bf16 hi + lo on the bf16 matrix cores, three
MFMAs per step: products within ~2^-16 of fp32); dropout masks come from a counter
hash of (seed, row, column) drawn on the device (graph-safe),
distribution-identical to ``nn.Dropout``.
"""
import torch

from .. import _ext


def fused_ok(pool, feats):
    """The fused kernels cover this call (else use the PyTorch module)."""
    if not feats or not feats[0].is_cuda or len(feats) > 8 or not _ext.host_available():
        return False
    lins = [m[0] for m in pool.feat_list]
    ps = {m[2].p for m in pool.feat_list}
    H = lins[0].out_features
    return (len(ps) == 1 and H % 64 == 0 and all(l.out_features == H for l in lins)
            and all(f.dtype == torch.float32 and f.size(-1) % 4 == 0 for f in feats)
            and all(l.bias is not None for l in lins))


def _rows(f):
    """(rows, d) view of a modality's features: rows with a unit column
    stride and 16-byte alignment are passed as they are (the kernels take a
    row stride), anything else as a contiguous copy."""
    x = f.reshape(-1, f.size(-1))
    if x.stride(-1) != 1 or x.stride(0) % 4 or x.data_ptr() % 16:
        x = x.contiguous()
    return x


class _FeatPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, rng, nf, *args):
        xs, ws, bs = args[:nf], args[nf:2 * nf], args[2 * nf:]
        out = _ext.ops().featpool_forward(list(xs), [w.detach() for w in ws],
                                          [b.detach() for b in bs], p, rng)
        ctx.p, ctx.nf = p, nf
        ctx.save_for_backward(out, *xs, *[w.detach() for w in ws])
        return out

    @staticmethod
    def backward(ctx, dout):
        out, *rest = ctx.saved_tensors
        nf = ctx.nf
        g = _ext.ops().featpool_backward(dout.contiguous(), out, list(rest[:nf]),
                                         list(rest[nf:]), ctx.p, [])
        return (None, None, None) + (None,) * nf + tuple(g[:nf]) + tuple(g[nf:])


class VgHandoff:
    """Hand-off between one :class:`_FeatPoolVgateFn` node and the decoder
    node that consumes ITS output: the payload the decoder backward needs to
    run this node's backward inside the engine, the identity of the vg tensor
    it belongs to (data pointer and shape: a decoder call with another vg
    ignores it), and ``done``, set by that decoder backward so this node's
    own backward becomes a no-op.  Kept on the node's ctx, not on the engine:
    a stale hand-off from a no-grad / eval call cannot leak into the next
    training step."""
    __slots__ = ('payload', 'key', 'done')

    def __init__(self, payload, vg):
        self.payload = payload
        self.key = (vg.data_ptr(), tuple(vg.shape))
        self.done = False

    def matches(self, vg):
        return vg is not None and self.key == (vg.data_ptr(), tuple(vg.shape))


class _FeatPoolVgateFn(torch.autograd.Function):
    """FeatPool + the video gate term of the fused engine in one node:
    ``vg = pack(FeatPool(x) . W_ih[:, E:]^T)`` (packed gate slots, see
    decoder_engine).  Backward: the FeatPool weight / bias gradients and the
    video columns of ``W_ih``'s gradient are written straight into their
    gradient-bucket slots when the trainer registered them (no autograd
    zero-fill / accumulate passes), else returned."""

    @staticmethod
    def forward(ctx, eng, p, rng, nf, record, *args):
        xs, ws, bs, w_ih = args[:nf], args[nf:2 * nf], args[2 * nf:3 * nf], args[3 * nf]
        wsd = [w.detach() for w in ws]
        fc = _ext.ops().featpool_forward(list(xs), wsd, [b.detach() for b in bs], p, rng)
        w_iv = w_ih.detach()[:, eng.E:]
        wiv = getattr(eng, 'wiv', None)
        if fc.is_cuda and wiv is not None:
            # bf16 operands (W_iv: the engine's packed shadow, rows already in
            # packed gate order, so the product IS the packed gate term), fp32
            # accumulate and output, the measured hipBLASLt choice
            # (host/blaslt_tuned.cpp): the fp32 product ran as an MT16x64 fp32
            # kernel, 39 us on the forward's critical path
            # (profiles/r6/steps_xe_after_fixes.txt); the decoder's other input
            # terms are bf16 products too
            vg = torch.empty(fc.size(0), wiv.size(0), device=fc.device)
            _ext.ops().gemm_bf16_tuned(vg, fc.to(torch.bfloat16), False, wiv, True)
        else:
            vg = eng.pack_rows(torch.mm(fc, w_iv.t()), eng.src_ie, 1)
        ctx.eng, ctx.p, ctx.nf, ctx.wih_shape = eng, p, nf, w_ih.shape
        ctx.save_for_backward(fc, *xs, *wsd)
        # the decoder forward that consumes vg takes these, so its backward
        # can run this node's backward inside the engine (vg_bwd); only when
        # this node is recorded for a backward (no hand-off from eval / beam)
        ctx.handoff = VgHandoff((fc, list(xs), wsd, p, nf), vg) if record else None
        eng._vg_pending = ctx.handoff
        return vg

    @staticmethod
    def backward(ctx, dvg):
        eng, nf = ctx.eng, ctx.nf
        h, ctx.handoff = ctx.handoff, None
        if h is not None and h.done:
            # the decoder backward already ran this node's backward (vg_bwd)
            # and wrote W_ih's video columns and the FeatPool gradient slots
            eng.take_video_slots()
            return (None,) * (5 + 4 * nf)
        fc, *rest = ctx.saved_tensors
        xs, ws = list(rest[:nf]), list(rest[nf:])
        E = eng.E
        dvg_u = dvg.index_select(1, eng.dst_ie)  # (B, G*H), PyTorch gate order
        w_iv = eng.model.core.rnn.weight_ih_l0.detach()[:, E:]
        dfc = torch.mm(dvg_u, w_iv)
        direct = eng.take_video_slots()
        if direct is not None:  # the decoder backward wrote W_ih's token columns
            torch.mm(dvg_u.t(), fc, out=direct['wih'][:, E:])
            outs = [direct['fp_w%d' % f] for f in range(nf)] + \
                   [direct['fp_b%d' % f] for f in range(nf)]
            _ext.ops().featpool_backward(dfc, fc, xs, ws, ctx.p, outs)
            return (None,) * (5 + 4 * nf)
        d_wih = fc.new_zeros(ctx.wih_shape)
        d_wih[:, E:] = dvg_u.t() @ fc
        g = _ext.ops().featpool_backward(dfc, fc, xs, ws, ctx.p, [])
        return (None,) * (5 + nf) + tuple(g[:nf]) + tuple(g[nf:]) + (d_wih,)


class _AttInputsFn(torch.autograd.Function):
    """Temporal attention's per-batch operands in one node: FeatPool over the
    C frames, then ONE bf16 GEMM (fp32 accumulate) against the stacked weight
    ``[W_ih[:, E:]; W_f]`` for the per-frame gate table ``Gv = pack(frames .
    W_iv^T)`` and the projected frames ``P = frames . W_f^T + b_f``
    (reference: ``/root/reference/model.py:119-142``; the module computes them
    as two fp32 Linears).  Backward: ``dframes = [dGv | dP] . [W_iv; W_f]``
    and ``[dW_iv; dW_f] = [dGv | dP]^T . frames`` as one bf16 GEMM each; W_ih's
    video columns and the FeatPool parameters are written straight into their
    gradient-bucket slots when the trainer registered them (as
    :class:`_FeatPoolVgateFn`), else returned."""

    @staticmethod
    def forward(ctx, eng, p, rng, nf, C, *args):
        xs, ws, bs = args[:nf], args[nf:2 * nf], args[2 * nf:3 * nf]
        w_ih, wf, bf = args[3 * nf:3 * nf + 3]
        wsd = [w.detach() for w in ws]
        fc = _ext.ops().featpool_forward(list(xs), wsd, [b.detach() for b in bs], p, rng)
        E, G4, A = eng.E, w_ih.size(0), wf.size(0)
        wcat = torch.empty(G4 + A, fc.size(1), dtype=torch.bfloat16, device=fc.device)
        wcat[:G4].copy_(w_ih.detach()[:, E:])
        wcat[G4:].copy_(wf.detach())
        fc16 = fc.to(torch.bfloat16)
        y = torch.mm(fc16, wcat.t(), out_dtype=torch.float32)  # (N * C, 4H + A)
        B = xs[0].size(0) // C
        gv = eng.pack_rows(y[:, :G4], eng.src_ie, 1).view(B, C, -1)
        pre = (y[:, G4:] + bf.detach()).view(B, C, A)
        ctx.eng, ctx.p, ctx.nf, ctx.wih_shape, ctx.G4 = eng, p, nf, w_ih.shape, G4
        ctx.save_for_backward(fc, fc16, wcat, *xs, *wsd)
        return gv, pre

    @staticmethod
    def backward(ctx, dgv, dpre):
        eng, nf, G4 = ctx.eng, ctx.nf, ctx.G4
        fc, fc16, wcat, *rest = ctx.saved_tensors
        xs, ws = list(rest[:nf]), list(rest[nf:])
        E, N = eng.E, fc.size(0)
        A = wcat.size(0) - G4
        dy = torch.empty(N, G4 + A, dtype=torch.bfloat16, device=fc.device)
        if dgv is not None:
            dy[:, :G4].copy_(dgv.reshape(N, -1).index_select(1, eng.dst_ie))  # PyTorch gate order
        else:
            dy[:, :G4].zero_()
        if dpre is not None:
            dpre = dpre.reshape(N, A)
            dy[:, G4:].copy_(dpre)
            dbf = dpre.sum(0)
        else:
            dy[:, G4:].zero_()
            dbf = None
        dfc = torch.mm(dy, wcat, out_dtype=torch.float32)
        direct = eng.take_video_slots()
        dyt = dy.t()
        dwf = torch.mm(dyt[G4:], fc16, out_dtype=torch.float32)
        if direct is not None:  # the decoder backward wrote W_ih's token columns
            torch.mm(dyt[:G4], fc16, out_dtype=torch.float32, out=direct['wih'][:, E:])
            outs = [direct['fp_w%d' % f] for f in range(nf)] + \
                   [direct['fp_b%d' % f] for f in range(nf)]
            _ext.ops().featpool_backward(dfc, fc, xs, ws, ctx.p, outs)
            return (None,) * (5 + 3 * nf) + (None, dwf, dbf)
        d_wih = fc.new_zeros(ctx.wih_shape)
        d_wih[:, E:] = torch.mm(dyt[:G4], fc16, out_dtype=torch.float32)
        g = _ext.ops().featpool_backward(dfc, fc, xs, ws, ctx.p, [])
        return (None,) * (5 + nf) + tuple(g[:nf]) + tuple(g[nf:]) + (d_wih, dwf, dbf)


def att_inputs(eng, model, feats):
    """Temporal attention operands (Gv (B, C, 4H) packed, P (B, C, A)) of the
    fused engine through :class:`_AttInputsFn` (train-mode FeatPool dropout as
    the module's)."""
    pool = model.feat_pool
    lins = [m[0] for m in pool.feat_list]
    p = float(pool.feat_list[0][2].p) if pool.training else 0.0
    dev = feats[0].device
    rng = _seeds(p, dev)
    xs = [_rows(f) for f in feats]
    ta = model.temporal_att
    return _AttInputsFn.apply(eng, p, rng, len(xs), feats[0].size(1), *xs, *[l.weight for l in lins],
                              *[l.bias for l in lins], model.core.rnn.weight_ih_l0,
                              ta.f_feat.weight, ta.f_feat.bias)


# Tests may pin the dropout seeds: a callable dev -> int32[2] device tensor
# (graph-vs-eager equivalence, tests/test_gpu_graph.py).  None = a fresh
# on-device draw per pass (graph-safe).
SEED_SOURCE = None


def _seeds(p, dev):
    if p <= 0:
        return torch.zeros(2, dtype=torch.int32, device=dev)
    if SEED_SOURCE is not None:
        return SEED_SOURCE(dev)
    return torch.randint(0, 2 ** 31 - 1, (2,), dtype=torch.int32, device=dev)


def featpool_vgate(eng, model, feats):
    """Packed video gate term (B, 4H) of the concat model through the fused
    FeatPool (train-mode dropout as the module's)."""
    pool = model.feat_pool
    lins = [m[0] for m in pool.feat_list]
    p = float(pool.feat_list[0][2].p) if pool.training else 0.0
    dev = feats[0].device
    rng = _seeds(p, dev)
    xs = [_rows(f) for f in feats]
    params = [l.weight for l in lins] + [l.bias for l in lins] + [model.core.rnn.weight_ih_l0]
    record = torch.is_grad_enabled() and any(t.requires_grad for t in params + xs)
    return _FeatPoolVgateFn.apply(eng, p, rng, len(xs), record, *xs, *params)


def featpool(pool, feats):
    """``pool(feats)`` through the fused kernels: feats list of (N, C, d_f)
    fp32 -> (N, F*H) for C == 1, else (N, C, F*H)."""
    lins = [m[0] for m in pool.feat_list]
    p = float(pool.feat_list[0][2].p) if pool.training else 0.0
    dev = feats[0].device
    rng = _seeds(p, dev)
    xs = [_rows(f) for f in feats]
    out = _FeatPoolFn.apply(p, rng, len(xs), *xs, *[l.weight for l in lins],
                            *[l.bias for l in lins])
    N, C = feats[0].shape[0], feats[0].shape[1]
    out = out.view(N, C, -1)
    return out.squeeze(1) if C == 1 else out
