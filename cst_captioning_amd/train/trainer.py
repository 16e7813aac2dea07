"""Training / validation driver.

Behaviour of ``/root/reference/train.py:45-418``:

  * loop ``while True``: batch -> scheduled-sampling / RL / MIXER / SCB
    schedules -> forward -> loss -> backward -> clip(0.25) -> Adam;
  * XE: teacher-forced cross entropy;
  * RL (``--use_rl 1`` from epoch ``use_rl_after``; 0 = the resume epoch):
      - SCST (``use_cst 0``): greedy decode baseline (``train.py:175-180``),
      - CST (``use_cst 1``): consensus baseline from GT or sample scores,
      - WXE (``use_cst 1, use_mixer 0``): precomputed GT scores as weights;
  * LR step decay on epoch change; validation + best-model checkpoint from
    ``save_checkpoint_from``; stop at ``max_epochs`` or after
    ``max_patience`` epochs without improvement.

MI355X-side changes (same semantics): the batch comes from HBM, the reward
is computed on the GPU (no host round trip), the greedy SCST baseline is
decoded once per video instead of once per (video, caption) row (FeatPool
dropout is applied before the x seq_per_img expansion, ``model.py:220-221``,
so the expanded rows are identical), gradients live in one flat bucket that
is all-reduced once per step (DP), and clip + Adam is one fused kernel.
Host synchronisation happens only at log / eval time.
"""
import json
import logging
import math
import os
import time

import numpy as np
import torch

from ..models import CrossEntropyCriterion, RewardCriterion
from ..ops.adam import FlatAdam
from ..ops.cider_d import CiderDScorer, GenericScorer
from ..parallel import FlatGradBucket
from ..reward.rewards import cst_from_scores, scst_from_scores
from ..utils import schedules, stamps
from ..utils.text import decode_sequence, compute_avglogp
from ..data.dataset import LazyGather
from ..utils.timers import PhaseTimer
from . import checkpoint as ckpt

logger = logging.getLogger(__name__)


def maybe_inject_fault(rank, it):
    """Fault injection for the recovery tests:
    ``CSTCAP_FAULT_INJECT=rank:iter:marker`` makes that rank die abruptly
    (``os._exit``, no cleanup, like a killed process) when it reaches
    iteration ``iter``, once: the marker file records that the fault fired,
    so the restarted job (torchrun ``--max-restarts``) runs through and resumes
    from the ``_last.pth`` sidecar."""
    spec = os.environ.get('CSTCAP_FAULT_INJECT')
    if not spec:
        return
    r, i, marker = spec.split(':', 2)
    if int(r) == rank and int(i) == it and not os.path.exists(marker):
        with open(marker, 'w') as f:
            f.write('rank %d killed at iter %d\n' % (rank, it))
        logger.error('fault injection: rank %d exits at iter %d', rank, it)
        os._exit(13)


def build_scorer(opt, dataset, device):
    metric = opt.eval_metric
    if metric in ('CIDEr', 'MSRVTT', 'Loss'):
        backend = 'auto'
        if getattr(opt, 'reward_device', 'gpu') == 'cpu':
            backend = 'cpu-ref'
        return CiderDScorer(dataset, use_eos=opt.use_eos, device=device, backend=backend)
    from ..eval.metrics import Bleu, Meteor, Rouge
    sc = {'Bleu_4': Bleu(4), 'METEOR': Meteor(), 'ROUGE_L': Rouge()}[metric]
    return GenericScorer(dataset, sc, opt.use_eos)


class Trainer:
    def __init__(self, opt, model, train_loader, val_loader=None, ctx=None, engine=None):
        from ..parallel import DistContext
        self.opt = opt
        self.model = model
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.ctx = ctx or DistContext()
        self.engine = engine
        self.device = self.ctx.device
        self.xe_criterion = CrossEntropyCriterion()
        self.rl_criterion = RewardCriterion()
        self.ctx.broadcast_module(model)
        # bucket order = the order the fused backward finalises gradients:
        # vocab head (under the reverse loop), embedding (post-loop tail), rest
        early = [model.logit.weight, model.logit.bias]
        # concat model on the engine: W_ih and the FeatPool parameters are
        # final shortly after the reverse loop (the engine runs the video-gate
        # backward there: decoder_engine ``vg_bwd``), a third streamed slice
        third = []
        if (engine is not None and not engine.attention and not engine.standard
                and engine.layers == 1 and hasattr(model, 'feat_pool')):
            third = [model.core.rnn.weight_ih_l0] + \
                [m[0].weight for m in model.feat_pool.feat_list] + \
                [m[0].bias for m in model.feat_pool.feat_list]
        self.bucket = FlatGradBucket(model.parameters(),
                                     first=early + [model.embed.weight] + third,
                                     world_size=self.ctx.world_size,
                                     wire=getattr(opt, 'grad_wire', 'fp32'),
                                     update=getattr(opt, 'dp_update', 'allreduce'))
        # Data parallelism: those two slices are all-reduced on a comm stream
        # as soon as the backward marks them final (events; external
        # event-record nodes in the captured graph), under the rest of the
        # backward, eager RCCL between replays (parallel/dist.py)
        if (engine is not None and self.ctx.enabled and self.device.type == 'cuda'
                and not getattr(opt, 'no_early_allreduce', 0) and self.bucket.wire == 'fp32'
                and not self.bucket.sharded):
            from .. import _ext
            self.bucket.set_groups([early, [model.embed.weight]] + ([third] if third else []),
                                   self.ctx, priority=getattr(opt, 'comm_priority', 'high'))
            _ext.ops().set_grad_events(True)
        if engine is not None:
            # the fused backward writes the vocab-head, embedding and LSTM
            # weight gradients straight into their bucket slots (one backward
            # per step: overwrite == accumulate onto the zeroed buffer)
            slot = {id(p): (off, n) for p, (off, n) in zip(self.bucket.params, self.bucket.slices)}
            rnn = model.core.rnn
            named = {'wlog': model.logit.weight, 'blog': model.logit.bias,
                     'emb': model.embed.weight, 'wih': rnn.weight_ih_l0, 'whh': rnn.weight_hh_l0}
            # FeatPool weights / biases: written by the fused FeatPool backward
            for i, m in enumerate(model.feat_pool.feat_list):
                named['fp_w%d' % i], named['fp_b%d' % i] = m[0].weight, m[0].bias
            engine.set_direct_slots(
                {k: self.bucket.grad[slot[id(p)][0]:slot[id(p)][0] + slot[id(p)][1]].view_as(p)
                 for k, p in named.items()}, named)
            self.bucket.on_zero = engine.arm_direct_slots
        if getattr(opt, 'honor_optim_flags', 0):
            betas, eps = (opt.optim_alpha, opt.optim_beta), opt.optim_epsilon
        else:
            betas, eps = (0.9, 0.999), 1e-8  # train.py:492 ignores --optim_*
        self.optimizer = FlatAdam(self.bucket, opt.learning_rate, betas, eps, opt.grad_clip)
        self.optimizer.grad_scale = self.bucket.grad_scale(self.ctx)
        if engine is not None:
            engine.attach_optimizer(self)
        self.scorer = None
        # SCST with the fused engine: X = E W launched right after the rollout
        # (engine.launch_x); False keeps the backward's own E' W GEMM (tests)
        self.use_x_after_rollout = True
        # XE steps: X = E W after the teacher-forced forward too (else the
        # backward computes it in reverse-order chunks under the loop)
        self.xe_x_after_forward = os.environ.get('CSTCAP_XE_XAFTER', '1') == '1'
        self._x_after_loss = False  # (xe_loss: X is launched after the loss)
        # PyTorch decoder path at --precision bf16: torch autocast (bf16 GEMMs /
        # LSTM, fp32 softmax), the same-precision baseline of the fused engine
        self.autocast_bf16 = (engine is None and self.device.type == 'cuda'
                              and getattr(opt, 'precision', 'bf16') == 'bf16')
        self.timer = PhaseTimer(enabled=bool(getattr(opt, 'profile_phases', 0)))
        self.infos = {'iter': 0, 'epoch': 0, 'start_epoch': 0, 'best_score': float('-inf'),
                      'best_iter': 0, 'best_epoch': opt.max_epochs}
        self.history = {}
        self.rl_training = False
        # HIP-graph step (see graph_step): captured step per schedule key
        self._graph = None
        self._graph_key = None
        self._graph_warm = {}
        self._ev_inputs = None

    # ------------------------------------------------------------------ RL ---
    def _ensure_scorer(self):
        if self.scorer is None:
            self.scorer = build_scorer(self.opt, self.train_loader.ds, self.device)
        return self.scorer

    def _decode_rollout(self, data):
        """Forward pass.  Returns (sample_seq, sample_logprobs, pred)."""
        m = self.model
        if self.engine is not None:
            return self.engine.rollout(m, data['feats'], data['labels'])
        pred, seq, lp = m(data['feats'], data['labels'])
        return seq, lp, pred

    def _greedy_scores(self, data, scorer, S, per_video=False):
        """SCST baseline scores, one per rewarded row (R,) (or, with
        per_video and the deduplicated greedy decode, one per video)."""
        opt, m = self.opt, self.model
        vid = data['video_index']
        if opt.expand_feat == 1 and getattr(opt, 'dedupe_greedy', 1):
            with torch.no_grad():
                g, _ = m.sample(data['feats'], {'sample_max': 1, 'expand_feat': 0})
            gs = scorer.score(g, vid)
            return gs if per_video else gs.repeat_interleave(S)
        with torch.no_grad():
            g, _ = m.sample(data['feats'], {'sample_max': 1, 'expand_feat': opt.expand_feat})
        gvid = vid.repeat_interleave(S) if opt.expand_feat == 1 else vid
        return scorer.score(g, gvid)

    def rl_loss(self, data, scb_captions):
        opt = self.opt
        S = self.train_loader.get_seq_per_img()
        scorer = self._ensure_scorer()
        vid_rows = data['video_index'].repeat_interleave(S)
        side = None
        if opt.use_cst == 0 and self.device.type == 'cuda':
            # The greedy baseline only depends on the inputs and the current
            # weights: decode + score it on a second HIP stream, concurrently
            # with the rollout on the main stream.
            if getattr(self, '_side_stream', None) is None:
                # (a high-priority stream for the greedy decode measured 4.5 ->
                # 8.7 ms per step: the queue priority throttles the rollout)
                self._side_stream = torch.cuda.Stream(device=self.device)
                self._ev_inputs = torch.cuda.Event()
                self._ev_greedy = torch.cuda.Event()
            side = self._side_stream
            main = torch.cuda.current_stream(self.device)
            # the batch's device part (a LazyGather inside a captured step) is
            # gathered HERE, on the main stream, before the event both decodes
            # order behind: gathered lazily by whichever decode touched it
            # first, the other stream would read it unordered
            gathered = (data['feats'], data['labels'])  # (LazyGather: gathers now)
            del gathered
            stamps.mark('gathered')
            inputs_ready = self._ev_inputs
            inputs_ready.record(main)
        # fused engine: reward, mask and REINFORCE loss in one launch
        # (ops/scst_loss.py), the greedy scores per video
        fused = self.engine is not None and opt.use_cst == 0 and self.device.type == 'cuda'

        def enqueue_greedy():
            inputs_ready.record(main)  # (everything main enqueued so far)
            side.wait_event(inputs_ready)
            with torch.cuda.stream(side):
                stamps.mark('greedy_begin')
                stamps.base('fwd_greedy')
                g = self._greedy_scores(data, scorer, S, per_video=fused)
                stamps.mark('greedy_end')
                self._ev_greedy.record(side)
            return g
        # The greedy branch is captured BEFORE the rollout.  A replayed graph's
        # nodes are submitted in capture order (~2.7 us each): captured after
        # the rollout, the greedy branch started only after the rollout's ~85
        # nodes, and with the X node below in the graph the runtime ran it
        # behind the rollout altogether (device stamps,
        # profiles/r3/README_r3.md "Node order of the replayed graph").
        if side is not None:
            greedy_scores = enqueue_greedy()
        stamps.base('fwd_sample')
        model_res, logprobs, _ = self._decode_rollout(data)
        stamps.mark('rollout_enq')
        if self.engine is not None:
            # the vocab head's X = E W on the engine's own stream once the
            # rollout is done, under the reward / loss computation
            # (engine.launch_x; on the greedy stream behind its decode, the
            # backward's deferred join crashed hipStreamEndCapture; launched
            # after the loss instead: same step time, profiles/r3/ab_xat_vhsched.txt)
            self.engine.launch_x()
        stamps.base(None)
        self.timer.mark('rollout')
        if opt.use_cst == 0:
            sample_scores = scorer.score(model_res, vid_rows)
            stamps.mark('sample_scores')
            if side is not None:
                main.wait_event(self._ev_greedy)
                greedy_scores.record_stream(main)
            else:
                greedy_scores = self._greedy_scores(data, scorer, S, per_video=fused)
            if fused:
                from ..ops.scst_loss import scst_loss
                loss, reward, m_score, b_score = scst_loss(model_res, logprobs, sample_scores,
                                                           greedy_scores)
                stamps.mark('loss')
                self.timer.mark('reward')
                return loss, {'reward': reward, 'm': m_score, 'b': b_score, 'seq': model_res}
            reward, m_score, b_score = scst_from_scores(sample_scores.float(),
                                                        greedy_scores.float())
        else:
            bcmr = data.get('bcmrscores')
            if bcmr is None or opt.use_mixer == 1:
                scores = scorer.score(model_res, vid_rows).float().view(-1, S)
            else:
                scores = bcmr.float()
            if self.engine is not None and self.device.type == 'cuda':
                # fused: consensus baseline, reward, mask and REINFORCE loss in
                # one launch (csrc/kernels/loss.hip, CST mode)
                from ..ops.scst_loss import cst_loss
                loss, reward, m_score, b_score = cst_loss(
                    model_res, logprobs, scores, None if bcmr is None else bcmr.float(),
                    scb_captions, opt.scb_baseline)
                stamps.mark('loss')
                self.timer.mark('reward')
                return loss, {'reward': reward, 'm': m_score, 'b': b_score, 'seq': model_res}
            reward, m_score, b_score = cst_from_scores(scores, bcmr, scb_captions,
                                                       opt.scb_baseline)
        self.timer.mark('reward')
        loss = self.rl_criterion(model_res, logprobs, reward.detach().to(logprobs.dtype))
        return loss, {'reward': reward, 'm': m_score, 'b': b_score, 'seq': model_res}

    def xe_loss(self, data):
        if self.engine is not None:
            lp = self.engine.teacher_forced(self.model, data['feats'], data['labels'])
            self.timer.mark('rollout')
            # (a batch whose masks were not set by hand: the loader's caption
            # masks, derived from the labels)
            derived = isinstance(data, LazyGather) and not dict.__contains__(data, 'masks')
            if self.device.type == 'cuda' and derived:
                # the masked cross-entropy with the loader's caption masks in
                # one launch (ops/scst_loss.py xe_loss); the vocab head's X =
                # E W follows the loss and its NaN-guard flag
                # (_forward_backward): the X GEMM holds every CU, so small
                # launches queued behind it waited for it (the masks' row
                # count: 388 us "long" reduction, profiles/r6/steps_xe.txt)
                from ..ops.scst_loss import xe_loss
                self._x_after_loss = True
                return xe_loss(data['labels'], lp, 1), {}
            # the vocab head's X = E W right after the teacher-forced forward,
            # on the engine's stream (as after an RL rollout): the backward's
            # reverse loop then starts on X instead of on its first chunk
            self.engine.launch_x()
            return self.xe_criterion(lp, data['labels'][:, 1:], data['masks'][:, 1:]), {}
        pred = self.model(data['feats'], data['labels'])[0]
        self.timer.mark('rollout')
        return self.xe_criterion(pred, data['labels'][:, 1:], data['masks'][:, 1:]), {}

    # --------------------------------------------------------------- step ---
    def _schedules(self, epoch):
        """Host-side per-epoch schedules (train.py:109-162): scheduled
        sampling, RL switch, MIXER start, SCB count.  Returns (mixer_from, scb)."""
        opt, m = self.opt, self.model
        ssp = schedules.ss_prob(opt, epoch)
        opt.ss_prob = ssp
        if ssp > 0 or opt.use_ss == 1:
            m.set_ss_prob(ssp)
        if opt.use_rl == 1 and epoch >= opt.use_rl_after and not self.rl_training:
            logger.info('Using RL objective...')
            self.rl_training = True
        mixer_from = opt.mixer_from
        if opt.use_mixer == 1 and self.rl_training:
            mixer_from = schedules.mixer_from(opt, epoch, opt.seq_length)
            m.set_mixer_from(mixer_from)
        scb = opt.scb_captions
        if opt.use_cst == 1 and self.rl_training:
            scb = schedules.scb_captions(opt, epoch, self.train_loader.get_seq_per_img())
        return mixer_from, scb

    def _forward_backward(self, data, mixer_from, scb):
        """zero_grad -> forward -> loss -> backward (+ the NaN-guard flag).
        Device work only: no host synchronisation (graph-capturable)."""
        opt, m = self.opt, self.model
        if self.engine is not None and self.device.type == 'cuda':
            self.engine.prefetch_ptab()  # under the prologue, on a side stream
        if self.engine is not None:
            # the vocab head's X = E W right after the rollout (RL: rl_loss ->
            # engine.launch_x) or the teacher-forced forward (XE: xe_loss), on
            # the engine's stream
            self.engine.x_after_rollout = bool(self.use_x_after_rollout and
                                               (self.rl_training or self.xe_x_after_forward))
        m.train()
        self.optimizer.zero_grad()
        m.set_seq_per_img(self.train_loader.get_seq_per_img())
        stamps.mark('step')
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=self.autocast_bf16):
            if self.rl_training:
                loss, extra = self.rl_loss(data, scb)
            else:
                loss, extra = self.xe_loss(data)
        # (the flag is enqueued before the backward: its few small launches run
        # while the backward's first operand, X = E W, is still computing,
        # instead of between the backward and the Adam pass)
        skip = None
        if getattr(opt, 'nan_guard', 1):
            skip = ~torch.isfinite(loss.detach())
            if self.ctx.enabled and not self.bucket.sharded:  # every rank must skip
                self.bucket.set_flag(skip)  # together: the flag rides the all-reduce
        if self._x_after_loss:
            self._x_after_loss = False
            self.engine.launch_x()
        stamps.base('bwd')
        loss.backward()
        stamps.base(None)
        stamps.mark('bwd_end')
        self.timer.mark('backward')
        extra.update(loss=loss.detach(), mixer_from=mixer_from, scb_captions=scb)
        return extra, skip

    def _apply_update(self, skip):
        """(after the gradient all-reduce) clip + Adam + weight shadows."""
        if getattr(self.opt, 'nan_guard', 1) and self.ctx.enabled:
            skip = self.bucket.flag_any()
        stamps.mark('adam_begin')
        self.optimizer.step(skip)
        stamps.mark('adam_end')
        if self.engine is not None:
            self.engine.after_step()
        stamps.mark('ptab_end')
        self.timer.mark('optimizer')

    def _sharded_update(self, skip):
        """--dp_update sharded (eager, between graph replays): reduce-scatter
        of the gradient sum, clip + Adam on this rank's 1/N shard (the global
        norm and every rank's skip flag through one 4 KB all-reduce), all-gather
        of the updated parameters, bf16 shadows refreshed from them."""
        gshard = self.bucket.reduce_scatter(self.ctx)
        self.timer.mark('allreduce')
        self.optimizer.step_sharded(self.ctx, gshard, skip)
        self.bucket.all_gather_params(self.ctx)
        if self.engine is not None:
            meta, dsts = self.optimizer._shadow
            if len(dsts):
                from .. import _ext
                _ext.ops().refresh_shadows(self.bucket.data, meta, dsts)
            self.engine.after_step()
        self.timer.mark('optimizer')

    def train_step(self, data, epoch):
        self.timer.reset()
        self.timer.mark('start')
        mixer_from, scb = self._schedules(epoch)
        if self._graph_enabled():
            out = self._graph_step(data, mixer_from, scb)
            if out is not None:
                return out
        self.bucket.begin_step()
        extra, skip = self._forward_backward(data, mixer_from, scb)
        self._check_grad_events()
        if self.bucket.sharded:
            self._sharded_update(skip)
            return extra
        self.bucket.all_reduce(self.ctx)
        self.timer.mark('allreduce')
        self._apply_update(skip)
        return extra

    # ------------------------------------------------------------ HIP graph ---
    # One training step replayed as ONE captured HIP graph (torch.cuda.CUDAGraph
    # is hipGraph on ROCm): feature encoder, rollout, concurrent greedy
    # baseline (second stream, joined by events), on-GPU CIDEr-D, reward,
    # backward (vocab head on a side stream), clip + Adam + bf16 weight shadows
    # and the input-token table.  The host then enqueues one graph launch per
    # step instead of ~600 kernel launches.  What makes the replay correct:
    #   * inputs are copied into static buffers before each replay;
    #   * RNG seeds are drawn on the device (graph-safe Philox offsets), the
    #     kernels read them from memory;
    #   * Adam's lr / step live on the device; the bf16 weight shadows and the
    #     token table are persistent buffers updated in place;
    #   * schedules that change the captured work (RL switch, MIXER start, SCB
    #     count, scheduled-sampling probability, batch shapes) key the graph:
    #     a new key is run eagerly once, then captured.
    # Under data parallelism the gradient all-reduce stays an eager RCCL call
    # between two graphs (forward/backward, then update).
    def _graph_enabled(self):
        return (self.engine is not None and self.device.type == 'cuda'
                and bool(getattr(self.opt, 'cuda_graph', 1)) and not self.timer.enabled)

    def _graph_signature(self, idx, mixer_from, scb):
        return (self.rl_training, mixer_from, scb, float(self.model.ss_prob),
                self.train_loader.get_seq_per_img(), tuple(tuple(t.shape) for t in idx))

    def _graph_step(self, data, mixer_from, scb):
        """Replay the captured step on this batch; None = run it eagerly."""
        idx = data.index_tensors() if hasattr(data, 'index_tensors') else None
        if idx is None:
            return None
        key = self._graph_signature(idx, mixer_from, scb)
        if key != self._graph_key:
            if self._graph_warm.get(key, 0) < 1:  # run a new schedule eagerly once
                self._graph_warm[key] = self._graph_warm.get(key, 0) + 1
                return None
            self._capture(data._loader, idx, key, mixer_from, scb)
        if not self._copy_flat(idx):
            for dst, src in zip(self._static_idx, idx):
                if src.data_ptr() != dst.data_ptr():  # (the loader uploads into them)
                    dst.copy_(src, non_blocking=True)
        self.optimizer.sync_lr()
        g_a, g_b = self._graph
        if g_b is not None:  # data parallel: the comm stream's lower bound
            self.bucket.mark_start()
            self.bucket.events_ok = self._graph_events_ok
        g_a.replay()
        if self.bucket.sharded:  # data parallel, sharded update: eager after the graph
            self._sharded_update(self._graph_skip)  # (calls engine.after_step)
        else:
            if g_b is not None:  # data parallel: eager all-reduce between the graphs
                self.bucket.all_reduce(self.ctx)
                g_b.replay()
            # the replayed update changed the weights on the device: the gate
            # table an eval may have refreshed since is stale again
            self.engine.after_step()
        return self._graph_out

    def _check_grad_events(self):
        """After a step's backward was enqueued or captured: did it record
        the event of every streamed DP slice?  If the streamed all-reduce is
        configured but an event is missing, the comm stream falls back to
        waiting for the whole step (correct, not overlapped) -- logged once."""
        ok = self.bucket.end_enqueue()
        if self.bucket.groups and not ok and not getattr(self, '_warned_events', False):
            self._warned_events = True
            logger.warning('the backward did not record every gradient-slice event: the DP '
                           'all-reduce waits for the whole step (no overlap)')
        return ok

    def _copy_flat(self, idx):
        """The loader's index tensors are consecutive pieces of one upload:
        one device copy into the static buffer instead of one per tensor."""
        flat = getattr(self, '_static_flat', None)
        if flat is None or len(idx) != len(self._static_idx) or not idx:
            return False
        t0 = idx[0]
        off = t0.data_ptr()
        for t, d in zip(idx, self._static_idx):
            if (t.dtype != d.dtype or t.shape != d.shape or not t.is_contiguous()
                    or t.data_ptr() != off or t.device != d.device):
                return False
            off += t.numel() * t.element_size()
        if t0.data_ptr() == flat.data_ptr():
            return True  # the loader uploaded into the static buffer itself
        n = flat.numel()
        if t0.storage_offset() + n > t0.untyped_storage().nbytes() // t0.element_size():
            return False
        flat.copy_(torch.as_strided(t0, (n,), (1,)), non_blocking=True)
        return True

    def _capture(self, loader, idx, key, mixer_from, scb):
        """Capture one step (batch gather + forward + backward [+ update]).
        Callers must not keep an earlier autograd graph alive (e.g. an
        un-freed loss tensor): its AccumulateGrad nodes stay bound to the
        default stream, and the cross-stream wait they add breaks the capture."""
        self._graph = self._graph_out = None
        torch.cuda.synchronize(self.device)
        # the captured step must refresh the gate table itself on every replay
        self.engine.invalidate_ptab()
        # one flat static buffer, refreshed by one device copy per replay
        # (uploading later batches straight into it measured neutral,
        # 3.558-3.563 vs 3.553-3.579 ms, profiles/r4/README_r4.md)
        flat = torch.cat([t.reshape(-1) for t in idx])
        self._static_flat = flat
        self._static_idx, off = [], 0
        for t in idx:
            self._static_idx.append(flat[off:off + t.numel()].view(t.shape))
            off += t.numel()
        pool = torch.cuda.graph_pool_handle()
        g_a = torch.cuda.CUDAGraph()
        self.bucket.begin_step(record_start=False)
        with torch.cuda.graph(g_a, pool=pool):
            # the batch gather is captured too, each part on first use
            batch = LazyGather(loader, self._static_idx)
            batch['video_index'] = self._static_idx[0]
            extra, skip = self._forward_backward(batch, mixer_from, scb)
            if not self.ctx.enabled:
                self._apply_update(skip)
        # every replay runs the captured record nodes of the slice events
        self._graph_events_ok = self._check_grad_events()
        g_b = None
        if self.ctx.enabled and not self.bucket.sharded:
            g_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_b, pool=pool):
                self._apply_update(skip)
        self._graph, self._graph_key, self._graph_out = (g_a, g_b), key, extra
        self._graph_skip = skip
        logger.info('captured the training step as a HIP graph (%s)',
                    'two graphs around the all-reduce' if g_b is not None else 'one graph')

    # --------------------------------------------------------------- loop ---
    def resume(self):
        opt = self.opt
        path = ckpt.resolve_start_from(opt.start_from, opt.model_file or '')
        last = ckpt.last_path(opt.model_file) if opt.model_file else None
        if last and getattr(opt, 'save_last', 1) and os.path.exists(last):
            s = ckpt.load_checkpoint(last, map_location=self.device)
            self.model.load_state_dict(s['model'])
            self.optimizer.load_state_dict(s['optimizer'])
            pr = s.get('per_rank')
            if pr is not None and len(pr) == self.ctx.world_size:
                self.train_loader.load_state_dict(pr[self.ctx.rank]['loader'])
                ckpt.restore_rng(pr[self.ctx.rank]['rng'])
                if self.val_loader is not None and 'val_loader' in pr[self.ctx.rank]:
                    self.val_loader.load_state_dict(pr[self.ctx.rank]['val_loader'])
            else:  # written by a run with another world size: shared state only
                self.train_loader.load_state_dict(s['loader'])
                ckpt.restore_rng(s['rng'])
            self.infos = s['infos']
            extra = s.get('extra') or {}
            self.history = extra.get('history', {})
            self._exact_resume = extra
            logger.info('Resumed exactly from %s (iter %d)', last, self.infos['iter'])
            # the sidecar records whether that epoch's validation already ran
            return extra.get('checked', True)
        if path and os.path.exists(path):
            logger.info('Loading state from: %s', path)
            s = ckpt.load_checkpoint(path, map_location=self.device)
            self.model.load_state_dict(s['model'])
            self.infos = s['infos']
            self.infos['start_epoch'] = self.infos['epoch']
            return True
        logger.info('No checkpoint found! Training from the scratch')
        return False

    def _save_last(self, checked):
        """Exact-resume sidecar: weights, optimizer, infos, history, the
        resolved RL/CST start epochs and every rank's loader position and RNG
        streams (gathered, written by rank 0)."""
        opt = self.opt
        if not (opt.model_file and getattr(opt, 'save_last', 1)):
            return
        self.optimizer.consolidate(self.ctx)  # sharded update: full moments on every rank
        mine = {'loader': self.train_loader.state_dict(), 'rng': ckpt.rng_state()}
        if self.val_loader is not None:  # its caption draws continue too
            mine['val_loader'] = self.val_loader.state_dict()
        per_rank = self.ctx.all_gather_object(mine)
        if self.ctx.is_main:
            extra = {'history': self.history, 'checked': checked,
                     'use_rl_after': opt.use_rl_after,
                     'use_cst_after': getattr(opt, 'use_cst_after', 0)}
            ckpt.save_last(ckpt.last_path(opt.model_file), self.model, self.optimizer,
                           self.infos, opt, self.train_loader, per_rank=per_rank, extra=extra)
        self.ctx.barrier()

    def train(self):
        opt, infos = self.opt, None
        self._exact_resume = None
        checked = self.resume()
        infos = self.infos
        if opt.model_file and self.ctx.is_main and not os.path.exists(opt.model_file):
            logger.info('>>> No model file found. Write a base checkpoint.')
            ckpt.save_checkpoint(self.model, infos, opt, opt.model_file)
        self.ctx.barrier()
        if self._exact_resume is not None and 'use_rl_after' in self._exact_resume:
            # exact resume: keep the schedule origin of the interrupted run, so
            # MIXER / SCB annealing continues where it was
            opt.use_rl_after = self._exact_resume['use_rl_after']
            opt.use_cst_after = self._exact_resume['use_cst_after']
        elif opt.use_rl == 1 and opt.use_rl_after == 0:
            # train.py:95-98: RL starts at the (warm-start) resume epoch
            opt.use_rl_after = infos['epoch']
            opt.use_cst_after = infos['epoch']
            self.train_loader.set_current_epoch(infos['epoch'])
        while True:
            t0 = time.time()
            data = self.train_loader.get_batch()
            out = self.train_step(data, infos['epoch'])
            infos['mixer_from'] = out['mixer_from']
            infos['scb_captions'] = out['scb_captions']
            if opt.print_log_interval and infos['iter'] % opt.print_log_interval == 0:
                self._log(out, time.time() - t0)
            infos['iter'] += 1
            maybe_inject_fault(self.ctx.rank, infos['iter'])
            if infos['epoch'] < self.train_loader.get_current_epoch():
                infos['epoch'] = self.train_loader.get_current_epoch()
                checked = False
                lr = schedules.adjust_learning_rate(opt, self.optimizer,
                                                    infos['epoch'] - infos['start_epoch'])
                logger.info('===> Learning rate: %f: ', lr)
                self._save_last(checked=False)
            if (self.val_loader is not None and infos['epoch'] >= opt.save_checkpoint_from
                    and infos['epoch'] % opt.save_checkpoint_every == 0 and not checked):
                results = self.validate(self.val_loader)
                if self.ctx.is_main:
                    logger.info('Validation output: %s',
                                json.dumps(results['scores'], indent=4, sort_keys=True))
                infos.update(results['scores'])
                self.check_model()
                checked = True
                # re-save with the validated best score / epoch and history
                self._save_last(checked=True)
            if infos['epoch'] >= opt.max_epochs or \
                    infos['epoch'] - infos['best_epoch'] > opt.max_patience:
                logger.info('>>> Terminating...')
                break
        return infos

    def reduce_log_scalars(self, out):
        """C3: the logged scalars averaged over the ranks -- ONE small
        all-reduce, on log iterations only, before the host conversion.
        Returns ``[loss, reward mean, m, b]`` (the RL entries only in RL mode)
        as Python floats."""
        vals = [out['loss']]
        if self.rl_training:
            vals += [out['reward'].float().mean(), out['m'], out['b']]
        dev = self.ctx.comm_device if self.ctx.enabled else self.device
        t = torch.stack([torch.as_tensor(v).detach().to(dev, torch.float64).reshape(())
                         for v in vals])
        self.ctx.all_reduce_(t, average=True)
        return t.tolist()

    def check_device_errors(self):
        """Failed cross-workgroup hand-offs counted on the device (a bounded
        flag poll that ran out of polls, csrc/kernels/lstm.hip att_fuse_wait):
        the gradients of those steps are not trusted, so training stops."""
        if self.device.type != 'cuda':
            return 0
        from .. import _ext
        n = int(_ext.ops().device_errors(self.device.index or 0))
        if n:
            raise RuntimeError('%d cross-workgroup hand-off(s) timed out on the device; '
                               'the affected gradients are not trusted' % n)
        return n

    def _log(self, out, elapsed):
        opt, infos = self.opt, self.infos
        vals = self.reduce_log_scalars(out)
        loss = vals[0]
        infos['TrainLoss'] = loss
        items = [('Epoch', infos['epoch']), ('Iter', infos['iter']), ('Loss', loss)]
        if self.rl_training:
            items += [('Reward', vals[1]),
                      ('{} (m)'.format(opt.eval_metric), vals[2]),
                      ('{} (b)'.format(opt.eval_metric), vals[3])]
        if opt.use_ss == 1:
            items.append(('ss_prob', opt.ss_prob))
        if opt.use_mixer == 1:
            items.append(('mixer_from', out['mixer_from']))
        if opt.use_cst == 1:
            items.append(('scb_captions', out['scb_captions']))
        items.append(('Time', elapsed))
        # updates the NaN guard skipped so far (non-finite loss on any rank or
        # non-finite gradient norm; csrc/kernels/adam.hip)
        items.append(('Skipped', int(self.optimizer.skipped().item())))
        if self.engine is not None:  # exp-store rows recomputed (LSE jump > 60)
            items.append(('ExpFix', int(self.engine.exp_fix_rows.item())))
            self.check_device_errors()
        # throughput since the previous log line (the scalar reduction above
        # synchronised the device, so the wall clock covers finished work)
        now = time.perf_counter()
        last = getattr(self, '_last_log', None)
        self._last_log = (now, infos['iter'])
        if last is not None and infos['iter'] > last[1]:
            rows = self.train_loader.get_batch_size() * self.train_loader.get_seq_per_img()
            items.append(('Captions/s', round(rows * self.ctx.world_size * (infos['iter'] - last[1])
                                              / (now - last[0]), 1)))
        if self.device.type == 'cuda':
            items.append(('HBM_GB', round(torch.cuda.max_memory_allocated(self.device) / 2 ** 30,
                                          2)))
        ph = self.timer.summary()
        if ph:
            items.append(('phases_ms', ','.join('%s=%.2f' % kv for kv in ph.items())))
        if self.ctx.is_main:
            logger.info('%s', '\t'.join('{}: {}'.format(k, v) for k, v in items))

    # ----------------------------------------------------------- validate ---
    @torch.no_grad()
    def validate(self, loader):
        opt, m, ctx = self.opt, self.model, self.ctx
        m.eval()
        n_videos = loader.get_num_videos()
        bsz = loader.get_batch_size()
        n_iters = int(math.ceil(n_videos / bsz))
        S = loader.get_seq_per_img()
        m.set_seq_per_img(S)
        local = {'pred': [], 'loss': [], 'gt_avglogp': [], 'test_avglogp': []}
        for ii in range(ctx.rank, n_iters, ctx.world_size):  # C4: batches sharded over ranks
            data = loader.get_batch_at(ii)
            if loader.has_label:
                if self.engine is not None:
                    lp = self.engine.teacher_forced(m, data['feats'], data['labels'])
                    loss = self.xe_criterion(lp, data['labels'][:, 1:], data['masks'][:, 1:])
                    gt_seq, gt_lp = data['labels'][:, 1:lp.size(1) + 1], lp
                else:
                    pred, gt_seq, gt_lp = m(data['feats'], data['labels'])
                    loss = self.xe_criterion(pred, data['labels'][:, 1:], data['masks'][:, 1:])
                local['loss'].append((ii, float(loss)))
                if opt.output_logp == 1:
                    local['gt_avglogp'].append(
                        (ii, compute_avglogp(gt_seq.cpu().numpy(), gt_lp.cpu().numpy())))
            seq, logseq = m.sample(data['feats'], {'beam_size': opt.beam_size})
            seq, logseq = seq.cpu().numpy(), logseq.cpu().numpy()
            sents = decode_sequence(loader.get_vocab(), seq)
            avg = compute_avglogp(seq, logseq) if opt.output_logp == 1 else None
            for jj, sent in enumerate(sents):
                e = {'image_id': data['ids'][jj], 'caption': sent}
                if avg is not None:
                    e['avglogp'] = avg[jj]
                local['pred'].append((ii, jj, e))
                logger.debug('[%d] video %s: %s', jj, e['image_id'], sent)
        gathered = ctx.all_gather_object(local)
        preds = sorted((p for g in gathered for p in g['pred']), key=lambda x: (x[0], x[1]))
        predictions = [p[2] for p in preds]
        losses = [l for g in gathered for _, l in g['loss']]
        results = {'predictions': predictions}
        scores = {'Loss': -round(sum(losses) / n_iters, 3) if losses else 0.0}
        if ctx.is_main and opt.language_eval == 1 and loader.has_label:
            from ..eval import language_eval
            refs = loader.ds.refs()
            if refs:
                scores.update(language_eval(refs, predictions))
        if opt.output_logp == 1:
            ta = [p['avglogp'] for p in predictions]
            scores['avglogp'] = sum(ta) / len(ta)
            gl = sorted((x for g in gathered for x in g['gt_avglogp']), key=lambda x: x[0])
            gt = np.array([v for _, l in gl for v in l]).reshape(-1, S)
            if ctx.is_main and opt.model_file:
                # train.py:367-373: the (N, S) array pickled beside the model
                # (plus an .npy twin that loads without unpickling)
                import pickle
                path = opt.model_file.replace('.pth', '_gt_avglogps.pkl', 1)
                with open(path, 'wb') as f:
                    pickle.dump(gt, f, protocol=pickle.HIGHEST_PROTOCOL)
                np.save(path[:-4] + '.npy', gt)
                logger.info('Wrote GT logp to: %s', path)
        results['scores'] = ctx.broadcast_object(scores)
        m.train()
        return results

    def test(self, loader):
        results = self.validate(loader)
        if self.ctx.is_main:
            logger.info('Test output: %s', json.dumps(results['scores'], indent=4))
            if self.opt.result_file:
                with open(self.opt.result_file, 'w') as f:
                    json.dump(results, f)
                logger.info('Wrote output caption to: %s ', self.opt.result_file)
        return results

    def check_model(self):
        opt, infos = self.opt, self.infos
        if opt.eval_metric == 'MSRVTT':
            cur = infos['Bleu_4'] + infos['METEOR'] + infos['ROUGE_L'] + infos['CIDEr']
        else:
            cur = infos[opt.eval_metric]
        if cur >= infos['best_score']:
            infos['best_score'] = cur
            infos['best_iter'] = infos['iter']
            infos['best_epoch'] = infos['epoch']
            logger.info('>>> Found new best [%s] score: %f, at iter: %d, epoch %d',
                        opt.eval_metric, cur, infos['iter'], infos['epoch'])
            if self.ctx.is_main and opt.model_file:
                ckpt.save_checkpoint(self.model, infos, opt, opt.model_file)
        else:
            logger.info('>>> Current best [%s] score: %f, at iter %d, epoch %d',
                        opt.eval_metric, infos['best_score'], infos['best_iter'],
                        infos['best_epoch'])
        self.history[infos['epoch']] = dict(infos)
        if self.ctx.is_main:
            ckpt.write_history(getattr(opt, 'history_file', None), self.history)
        self.ctx.barrier()
