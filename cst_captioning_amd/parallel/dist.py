"""Data-parallel communication over ``torch.distributed`` (RCCL on ROCm).

The reference is single-GPU with no collectives.  This
layer adds DP for one node of MI355X GPUs, one process per GPU:

  C1  broadcast of parameters/buffers from rank 0 at start;
  C2  the whole gradient as ONE flat bucket, all-reduced in at most three
      large slices ordered by when the backward finalises them
      (:meth:`FlatGradBucket.all_reduce`): the vocabulary head (logit W, b:
      final after its dW GEMM, which runs under the reverse LSTM loop), the
      embedding (final after its GEMM in the post-loop tail), then the rest.
      The fused backward marks the first two with events (external
      event-record nodes inside a captured HIP graph); the comm stream (high
      priority: a hardware queue of its own) waits on the step-start event and
      on them -- never on the whole replay -- and their all-reduces run while
      the rest of the backward does -- eager RCCL, nothing captured.  Large slices are
      what a point-to-point xGMI ring moves at full per-link bandwidth
      (~20 M params = 84 MB fp32).  --dp_update sharded: reduce-scatter ->
      Adam on the rank's 1/N shard -> all-gather of the updated parameters.
      288 GB HBM makes the contiguous buffer free;
  C3  all-reduce of a small vector of log scalars;
  C4  all-gather of per-rank evaluation results;
  C5  broadcast of rank-0 decisions (best model / early stop);
  C6  barrier around rank-0 checkpoint IO.

CPU tests use the gloo backend with the same code.
"""
import datetime
import os

import torch
import torch.distributed as dist


class DistContext:
    def __init__(self, rank=0, world_size=1, local_rank=0, device=None, backend=None):
        self.rank = rank
        self.world_size = world_size
        self.local_rank = local_rank
        if device is None:
            device = (torch.device('cuda', torch.cuda.current_device())
                      if torch.cuda.is_available() else torch.device('cpu'))
        self.device = device
        self.backend = backend

    @property
    def enabled(self):
        return self.world_size > 1

    @property
    def is_main(self):
        return self.rank == 0

    # -- collectives ------------------------------------------------------------
    def barrier(self):
        if self.enabled:
            if self.backend == 'nccl':
                dist.barrier(device_ids=[self.local_rank])
            else:
                dist.barrier()

    def all_reduce_(self, t, average=False):
        if self.enabled:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            if average:
                t.div_(self.world_size)
        return t

    def broadcast_(self, t, src=0):
        if self.enabled:
            dist.broadcast(t, src)
        return t

    def broadcast_object(self, obj, src=0):
        if not self.enabled:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src)
        return box[0]

    def all_gather_object(self, obj):
        if not self.enabled:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj)
        return out

    def max_scalar(self, x):
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.comm_device)
        if self.enabled:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    @property
    def comm_device(self):
        return self.device if self.backend == 'nccl' else torch.device('cpu')

    def broadcast_module(self, module):
        """C1: every parameter and buffer from rank 0 (one flat message)."""
        if not self.enabled:
            return
        tensors = [t for t in list(module.parameters()) + list(module.buffers())
                   if t.dtype.is_floating_point]
        if not tensors:
            return
        flat = torch.cat([t.detach().reshape(-1).float() for t in tensors]).to(self.comm_device)
        dist.broadcast(flat, 0)
        off = 0
        with torch.no_grad():
            for t in tensors:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t).to(t.device, t.dtype))
                off += n

    def destroy(self):
        if self.enabled and dist.is_initialized():
            dist.destroy_process_group()


def init_distributed(device_type=None, timeout_s=600):
    """Initialise from the torchrun environment (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT).  Single process when WORLD_SIZE is unset."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if device_type is None:
        device_type = 'cuda' if torch.cuda.is_available() else 'cpu'
    if device_type == 'cuda':
        # one GPU per local rank; CSTCAP_SHARE_GPU=1 folds ranks onto the visible
        # devices (multi-rank tests on a one-GPU box, with the gloo backend)
        if os.environ.get('CSTCAP_SHARE_GPU') == '1':
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        device = torch.device('cuda', local)
    else:
        device = torch.device('cpu')
    backend = None
    if world > 1:
        backend = os.environ.get('CSTCAP_DIST_BACKEND') or ('nccl' if device_type == 'cuda'
                                                            else 'gloo')
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        kw = {}
        if backend == 'nccl':
            kw['device_id'] = device
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistContext(rank, world, local, device, backend)


class FlatGradBucket:
    """All trainable parameters re-homed into one contiguous fp32 buffer,
    with their ``.grad`` tensors viewing one contiguous gradient buffer.

    Autograd accumulates into the views in place, so after ``backward()`` the
    whole gradient is one tensor: one all-reduce (C2) and one fused
    clip + Adam kernel cover every parameter.
    """

    def __init__(self, params, first=(), world_size=1, wire='fp32', update='allreduce'):
        """``first``: parameters placed at the start of the buffer, in this
        order (the slices :meth:`set_groups` reduces ahead of the rest).  ``wire``:
        'fp32' (one all-reduce) or 'bf16' (see :meth:`all_reduce`); the buffer
        is padded so it splits into ``world_size`` equal chunks."""
        if wire not in ('fp32', 'bf16'):
            raise ValueError('wire must be fp32 or bf16')
        if update not in ('allreduce', 'sharded'):
            raise ValueError('update must be allreduce or sharded')
        if update == 'sharded' and wire != 'fp32':
            raise ValueError('the sharded update reduce-scatters an fp32 gradient')
        self.wire = wire
        self.update = update
        self.world_size = world_size
        params = [p for p in params if p.requires_grad]
        first = [p for p in first if p.requires_grad]
        first_ids = {id(p) for p in first}
        self.params = list(first) + [p for p in params if id(p) not in first_ids]
        self.groups = []  # streamed slices (set_groups)
        self.comm = None
        self._ev_start = None
        self._counts = None
        self.events_ok = False
        self.on_zero = None
        if not self.params:
            raise ValueError('no trainable parameters')
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        # one status slot after the parameters (padded to 64 elements): a
        # rank's "skip this step" flag rides the gradient all-reduce instead of
        # a collective of its own.  It is zero in every healthy step, so it adds
        # nothing to the gradient norm and Adam leaves its (zero) parameter
        # slot at zero.
        quantum = 64 * max(1, world_size)
        padded = (total + 1 + quantum - 1) // quantum * quantum
        self.data = torch.zeros(padded, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(padded, dtype=torch.float32, device=dev)
        self.flag = self.grad[total:total + 1]
        self.slices = []
        off = 0
        for p in self.params:
            n = p.numel()
            self.data[off:off + n].copy_(p.detach().reshape(-1))
            p.data = self.data[off:off + n].view_as(p)
            p.grad = self.grad[off:off + n].view_as(p)
            self.slices.append((off, n))
            off += n
        self.numel = total

    def set_flag(self, bad):
        """Store this rank's skip flag (0-dim bool device tensor) in the
        status slot before :meth:`all_reduce`."""
        self.flag.copy_(bad.reshape(1))

    def flag_any(self):
        """After :meth:`all_reduce`: true on every rank when any rank set its
        flag (0-dim bool device tensor, no host sync)."""
        return self.flag[0] > 0

    def zero_grad(self):
        self.grad.zero_()
        if self.on_zero is not None:  # e.g. re-arm the fused engine's direct slots
            self.on_zero()
        # autograd may have replaced a view (e.g. after set_to_none); re-point
        for p, (off, n) in zip(self.params, self.slices):
            if p.grad is None or p.grad.data_ptr() != self.grad[off:].data_ptr():
                p.grad = self.grad[off:off + n].view_as(p)

    def prefix_numel(self, params):
        """Elements of the leading slots holding exactly ``params``."""
        n = 0
        for p, want in zip(self.params, params):
            if p is not want:
                raise ValueError('parameters are not the leading slots of the bucket')
            n += p.numel()
        return n

    # -- sharded update (ZeRO-1 style, --dp_update sharded) ----------------------
    @property
    def sharded(self):
        return self.update == 'sharded' and self.world_size > 1

    def shard_range(self, rank):
        n = self.grad.numel() // self.world_size
        return rank * n, (rank + 1) * n

    def reduce_scatter(self, ctx):
        """Sum of every rank's gradient over this rank's 1/N shard (returned,
        a buffer of its own); the rest of the local buffer is left as is.
        Every rank's skip flag is carried separately (FlatAdam.step_sharded)."""
        lo, hi = self.shard_range(ctx.rank)
        if not hasattr(self, '_gshard') or self._gshard.numel() != hi - lo:
            self._gshard = torch.empty(hi - lo, dtype=self.grad.dtype, device=self.grad.device)
        if ctx.backend == 'gloo' and self.grad.is_cuda:
            # gloo has no reduce-scatter of device tensors (the shared-GPU
            # tests): the same sums through an all-reduce, then this shard
            dist.all_reduce(self.grad, op=dist.ReduceOp.SUM)
            self._gshard.copy_(self.grad[lo:hi])
        else:
            dist.reduce_scatter_tensor(self._gshard, self.grad, op=dist.ReduceOp.SUM)
        return self._gshard

    def all_gather_params(self, ctx):
        """Every rank's updated shard into the full parameter buffer."""
        lo, hi = self.shard_range(ctx.rank)
        mine = self.data[lo:hi].clone()  # (input and output must not alias)
        dist.all_gather_into_tensor(self.data, mine)

    def grad_scale(self, ctx):
        """Factor between the reduced buffer and the mean gradient: the fp32
        path SUMS over ranks and leaves the 1/N to the optimizer (FlatAdam's
        ``grad_scale``), so no separate pass over the buffer divides it."""
        return 1.0 / ctx.world_size if (ctx.enabled and self.wire == 'fp32') else 1.0

    def set_groups(self, groups, ctx, priority='normal'):
        """Leading slices reduced as soon as the backward marks them final:
        ``groups`` = [params of slice 0, params of slice 1(, slice 2)] (at
        most three; they must be the buffer's leading parameters, in order).
        The fused backward records the matching events (engine
        ``set_grad_events``): vocab head, embedding, and for the concat model
        W_ih + FeatPool (the video-gate backward done inside the engine).
        ``priority``: 'high' or 'normal' priority for the comm stream."""
        assert 1 <= len(groups) <= 3, 'one to three streamed slices'
        assert priority in ('high', 'normal'), 'comm priority: high or normal'

        self.groups = []
        off = 0
        want = [p for g in groups for p in g]
        self.prefix_numel(want)  # (checks the order)
        for g in groups:
            n = sum(p.numel() for p in g)
            self.groups.append((off, off + n))
            off += n
        if self.grad.is_cuda and self.comm is None:
            # Normal priority by default.  A HIGH-priority stream gets a
            # hardware queue of its own (the HIP runtime keeps one pool of
            # queues per priority), but measured with the trainer's replayed
            # step and 1-rank RCCL collectives on it, the high-priority queue
            # slowed the WHOLE step from 3.38 to 5.75 ms (the rollout most),
            # and a 32-workgroup stand-in for a ring kernel cost +160 us at
            # normal vs +290 us at high priority (scripts/dp_standin.py,
            # profiles/r6/dp_standin_rccl.json); the slices still start
            # inside the backward at normal priority.
            self.comm = torch.cuda.Stream(device=self.grad.device,
                                          priority=-1 if priority == 'high' else 0)
            self._ev_start = torch.cuda.Event()
        self._counts = None
        self.events_ok = False

    standin = None  # (workgroups, us): see all_reduce

    def _standin_buf(self):
        buf = getattr(self, '_standin_scratch', None)
        if buf is None:
            buf = self._standin_scratch = torch.empty(64 << 20, device=self.grad.device)
        return buf

    # -- streamed slices: ordering bookkeeping -------------------------------------
    @staticmethod
    def _event_counts():
        from .. import _ext
        return tuple(_ext.ops().grad_event_count(k) for k in range(3))

    def mark_start(self):
        """Record the step-start event on the current stream before a step's
        device work is enqueued (eager forward or graph replay): the lower
        bound of the comm stream (:meth:`all_reduce`)."""
        if self.groups and self.comm is not None:
            self._ev_start.record(torch.cuda.current_stream(self.grad.device))

    def begin_step(self, record_start=True):
        """Before a step's forward/backward is enqueued (``record_start``) or
        captured (False: no event inside a capture): :meth:`mark_start` and a
        snapshot of the engine's grad-event record counts, which
        :meth:`end_enqueue` compares."""
        if not self.groups or self.comm is None:
            return
        if record_start:
            self.mark_start()
        self._counts = self._event_counts()

    def end_enqueue(self):
        """After the step's backward was enqueued eagerly, or captured: True
        when the backward recorded (or captured a record node of) the event of
        every streamed slice.  Only then does :meth:`all_reduce` let the comm
        stream start a slice before the backward is done."""
        if not self.groups or self._counts is None:
            self.events_ok = False
            return False
        now = self._event_counts()
        self.events_ok = all(now[k] > self._counts[k] for k in range(len(self.groups)))
        self._counts = None
        return self.events_ok

    def all_reduce(self, ctx):
        """Reduce the gradient over ranks: fp32 wire -> the SUM (the mean is
        ``grad * grad_scale(ctx)``); bf16 wire -> the mean.

        wire 'fp32': RCCL ring all-reduces of the fp32 buffer -- with groups,
        each leading slice on the comm stream once ITS event fired (they run
        while the enqueued backward still computes the rest), then the rest
        on the current stream, which finally waits for the slices.  The comm
        stream is ordered only behind the step-start event (:meth:`begin_step`)
        and the slice events, never behind the whole backward.  Every rank
        issues the same collectives in the same order.  wire 'bf16': half the
        bytes on xGMI with fp32 accumulation -- every rank sends chunk j of
        its gradient as bf16 to rank j (all-to-all), sums the N received chunks
        in fp32, and the reduced chunks are all-gathered as bf16.  Per rank
        that moves (N-1)/N of the buffer in bf16 twice, half of the fp32
        ring's 2 (N-1)/N x 4 bytes; the applied gradient carries one bf16
        rounding of each input and of the sum (relative 2^-9), which Adam's
        normalised update tolerates.  The skip flag (0 / 1) is exact in bf16."""
        if ctx.enabled and self.wire == 'bf16':
            N = ctx.world_size
            chunk = self.grad.numel() // N
            send = self.grad.view(N, chunk).to(torch.bfloat16)
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send)
            mine = recv.float().sum(0).div_(N).to(torch.bfloat16)
            out = torch.empty(N * chunk, dtype=torch.bfloat16, device=self.grad.device)
            dist.all_gather_into_tensor(out, mine)
            self.grad.copy_(out)
            return
        if not ctx.enabled:
            return
        if not self.groups or self.comm is None:
            dist.all_reduce(self.grad, op=dist.ReduceOp.SUM)
            return
        from .. import _ext
        from ..utils import stamps
        main = torch.cuda.current_stream(self.grad.device)
        events_ok, self.events_ok = self.events_ok, False  # (one step's verdict)
        if events_ok:
            self.comm.wait_event(self._ev_start)
        else:  # this step recorded no slice events: order behind the whole step
            self.comm.wait_stream(main)
        # nccl (RCCL): a synchronous collective is enqueued on the CURRENT
        # stream (the comm stream here) and returns without blocking the host;
        # gloo (shared-GPU tests): asynchronous work joined below
        sync_on_stream = ctx.backend == 'nccl'
        works = []
        with torch.cuda.stream(self.comm):
            for k, (lo, hi) in enumerate(self.groups):
                if events_ok:
                    _ext.ops().grad_event_wait(k, self.comm.cuda_stream)
                stamps.mark('comm%d' % k)
                if k == 0 and self.standin is not None:
                    # measurement hook (tests / scripts): a collective-shaped
                    # stand-in kernel where the vocab-head slice's ring runs
                    blocks, us = self.standin
                    _ext.ops().busy_copy(self._standin_buf(), blocks, us, self.comm.cuda_stream)
                w = dist.all_reduce(self.grad[lo:hi], op=dist.ReduceOp.SUM,
                                    async_op=not sync_on_stream)
                if w is not None:
                    works.append(w)
        dist.all_reduce(self.grad[self.groups[-1][1]:], op=dist.ReduceOp.SUM)
        for w in works:
            w.wait()
        main.wait_stream(self.comm)
