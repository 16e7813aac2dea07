"""Fused global-norm clip + Adam over one flat parameter buffer.

Replaces ``clip_grad_norm_(model.parameters(), grad_clip)`` +
``optim.Adam(lr)`` (``/root/reference/train.py:217-218,492``; default betas
(0.9, 0.999), eps 1e-8, no weight decay) with one pass over the flat
buffers of :class:`..parallel.FlatGradBucket`:

  * pass 1: sum of squares of the gradient (one block-reduction kernel);
  * pass 2: ``coef = min(1, clip / (norm + 1e-6))`` is computed ON DEVICE
    and applied inside the Adam update, which also refreshes the bf16
    shadow copies of the decoder weights used by the MFMA kernels
    (:meth:`set_shadows`).

No host synchronisation.  Learning rate and step count live in a device
tensor (``[lr, step, skipped, step after]``): the bias corrections follow
the device step, so a captured HIP graph replays correct updates, and
:meth:`sync_lr` (outside any capture) publishes an LR change made through
``param_groups``.  NaN guard: a device flag (non-finite loss on any rank) or
a non-finite gradient norm turns the update into a no-op that does not
advance the step; skips are counted on the device.  The math is PyTorch's Adam:
``denom = sqrt(v) / sqrt(1 - b2^t) + eps``,
``p -= lr / (1 - b1^t) * m / denom``.

Without the HIP extension (CPU) the same math runs as torch ops.
"""
import math

import torch

from .. import _ext


class FlatAdam:
    def __init__(self, bucket, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, grad_clip=0.25):
        self.bucket = bucket
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.grad_clip = grad_clip
        # the gradient buffer holds grad / grad_scale: a data-parallel SUM
        # all-reduce sets 1 / world_size here instead of dividing the buffer
        self.grad_scale = 1.0
        self.exp_avg = torch.zeros_like(bucket.data)
        self.exp_avg_sq = torch.zeros_like(bucket.data)
        self.param_groups = [{'lr': lr}]  # for adjust_learning_rate()
        self.last_norm = None
        self._use_hip = _ext.available() and bucket.data.is_cuda
        self.supports_shadows = self._use_hip
        self._shadow = (torch.empty(0, dtype=torch.int64), [])
        dev = bucket.data.device
        # [lr, step before the update, skipped updates, step after the update]
        # (csrc/kernels/adam.hip); the torch path uses the same layout
        self._hyper = torch.tensor([float(lr), 0.0, 0.0, 0.0], dtype=torch.float32, device=dev)
        if self._use_hip:
            # 1024 sum-of-squares partials + the sharded update's skip-flag slot
            self._partials = torch.zeros(1025, dtype=torch.float32, device=dev)
            self._scal = torch.empty(2, dtype=torch.float32, device=dev)
            self._no_skip = torch.zeros((), dtype=torch.bool, device=dev)
            self._lr_synced = float(lr)

    def set_shadows(self, meta, dsts):
        """bf16 shadow copies the update pass writes (see csrc/kernels/adam.hip)."""
        self._shadow = (meta, list(dsts))

    def sync_lr(self):
        """Publish ``param_groups[0]['lr']`` to the device (no-op if unchanged).
        Call outside graph capture."""
        lr = float(self.param_groups[0]['lr'])
        if self._use_hip and lr != self._lr_synced:
            self._hyper[0].fill_(lr)
            self._lr_synced = lr

    def zero_grad(self):
        self.bucket.zero_grad()

    def step(self, skip=None):
        """``skip``: optional 0-dim bool device tensor; when true the update
        is a no-op (NaN guard without a host sync).  A non-finite gradient
        norm skips the update too.  Skipped updates do not advance the step
        count (as in torch.optim.Adam) and are counted (:meth:`skipped`)."""
        self.lr = self.param_groups[0]['lr']
        b1, b2 = self.betas
        g, p = self.bucket.grad, self.bucket.data
        if self._use_hip:
            if not torch.cuda.is_current_stream_capturing():
                self.sync_lr()
            self.last_norm = _ext.ops().flat_adam_step(
                p, g, self.exp_avg, self.exp_avg_sq, self._partials, self._scal,
                skip if skip is not None else self._no_skip, self._hyper,
                float(b1), float(b2), float(self.eps), float(self.grad_clip),
                float(self.grad_scale), 0, *self._shadow)
            return self.last_norm
        h = self._hyper
        h[1].copy_(h[3])
        t = h[1].double() + 1
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        norm = torch.linalg.vector_norm(g) * self.grad_scale
        self.last_norm = norm
        bad = ~torch.isfinite(norm)
        if skip is not None:
            bad = bad | skip.reshape(())
        keep = ~bad
        coef = torch.clamp(self.grad_clip / (norm + 1e-6), max=1.0) * self.grad_scale
        gc = g * coef
        m_new = self.exp_avg * b1 + gc * (1 - b1)
        v_new = self.exp_avg_sq * b2 + gc * gc * (1 - b2)
        denom = v_new.sqrt() / bc2.sqrt().float() + self.eps
        upd = m_new / denom * (self.lr / bc1).float()
        # torch.where, not a 0/1 multiply: NaN * 0 is NaN
        self.exp_avg.copy_(torch.where(keep, m_new, self.exp_avg))
        self.exp_avg_sq.copy_(torch.where(keep, v_new, self.exp_avg_sq))
        p.copy_(torch.where(keep, p - upd, p))
        h[3].copy_(torch.where(keep, t.float(), h[1]))
        h[2].add_(bad.float())
        return norm

    def step_sharded(self, ctx, gshard, skip=None):
        """Data-parallel sharded update (``--dp_update sharded``): ``gshard``
        is this rank's shard of the gradient SUM (FlatGradBucket.reduce_scatter).
        The clip norm is global: the shard's sum-of-squares partials (and the
        rank's skip flag) are all-reduced before the update; Adam then runs on
        the shard only (moments of other shards stay untouched here) and the
        caller all-gathers the parameters.  Same arithmetic as :meth:`step` on
        the all-reduced buffer with ``grad_scale = 1 / N``."""
        import torch.distributed as dist
        b1, b2 = self.betas
        lo, hi = self.bucket.shard_range(ctx.rank)
        p, m, v = self.bucket.data[lo:hi], self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi]
        gscale = 1.0 / ctx.world_size
        flag = skip.reshape(1).float() if skip is not None else None
        if self._use_hip:
            if not torch.cuda.is_current_stream_capturing():
                self.sync_lr()
            ops = _ext.ops()
            args = (float(b1), float(b2), float(self.eps), float(self.grad_clip), gscale)
            ops.flat_adam_step(p, gshard, m, v, self._partials, self._scal, self._no_skip,
                               self._hyper, *args, 1, torch.empty(0, dtype=torch.int64), [])
            if flag is not None:
                self._partials[1024:1025].copy_(flag)
            else:
                self._partials[1024:1025].zero_()
            dist.all_reduce(self._partials, op=dist.ReduceOp.SUM)
            any_skip = self._partials[1024] > 0
            self.last_norm = ops.flat_adam_step(
                p, gshard, m, v, self._partials, self._scal, any_skip, self._hyper, *args, 2,
                torch.empty(0, dtype=torch.int64), [])
            return self.last_norm
        h = self._hyper
        h[1].copy_(h[3])
        t = h[1].double() + 1
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        red = torch.stack([gshard.double().pow(2).sum(),
                           flag.double().sum() if flag is not None else torch.zeros((), dtype=torch.float64)])
        dist.all_reduce(red, op=dist.ReduceOp.SUM)
        norm = red[0].sqrt().float() * gscale
        self.last_norm = norm
        bad = ~torch.isfinite(norm) | (red[1] > 0)
        keep = ~bad
        coef = torch.clamp(self.grad_clip / (norm + 1e-6), max=1.0) * gscale
        gc = gshard * coef
        m_new = m * b1 + gc * (1 - b1)
        v_new = v * b2 + gc * gc * (1 - b2)
        denom = v_new.sqrt() / bc2.sqrt().float() + self.eps
        upd = m_new / denom * (self.lr / bc1).float()
        m.copy_(torch.where(keep, m_new, m))
        v.copy_(torch.where(keep, v_new, v))
        p.copy_(torch.where(keep, p - upd, p))
        h[3].copy_(torch.where(keep, t.float(), h[1]))
        h[2].add_(bad.float())
        return norm

    def consolidate(self, ctx):
        """Sharded update: gather every rank's moment shards, so the full
        Adam state is on every rank (checkpoints).  Collective."""
        import torch.distributed as dist
        if not (self.bucket.sharded and ctx.enabled):
            return
        lo, hi = self.bucket.shard_range(ctx.rank)
        for buf in (self.exp_avg, self.exp_avg_sq):
            mine = buf[lo:hi].clone()
            dist.all_gather_into_tensor(buf, mine)

    @property
    def step_count(self):
        return self._steps()

    def skipped(self):
        """Updates the NaN guard skipped so far (0-dim device tensor: reading
        it synchronises, so the trainer converts it at log time only)."""
        return self._hyper[2]

    def _steps(self):
        # graph replays advance only the device counter
        return int(self._hyper[3].item())

    def state_dict(self):
        return {'step': self._steps(), 'exp_avg': self.exp_avg,
                'exp_avg_sq': self.exp_avg_sq, 'lr': self.param_groups[0]['lr'],
                'betas': self.betas, 'eps': self.eps,
                'skipped': int(self._hyper[2].item())}

    def load_state_dict(self, s):
        self.exp_avg.copy_(s['exp_avg'])
        self.exp_avg_sq.copy_(s['exp_avg_sq'])
        self.param_groups[0]['lr'] = s['lr']
        self._hyper[1].fill_(float(s['step']))
        self._hyper[3].fill_(float(s['step']))
        self._hyper[2].fill_(float(s.get('skipped', 0)))
        self._hyper[0].fill_(float(s['lr']))
        if self._use_hip:
            self._lr_synced = float(s['lr'])
