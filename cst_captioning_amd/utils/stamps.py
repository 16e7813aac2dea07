"""Device timeline stamps (SURVEY.md 5.1 tracing).

A one-thread kernel (``csrc/kernels/stamp.hip``) writes the GPU wall clock
(100 MHz) into a slot of a device buffer on the stream that runs a phase.
The stamps are enqueued like any other kernel, so inside a captured HIP graph
they become graph nodes on the branch they were captured on and show the
replayed step's real concurrency (rocprofv3 serialises a replayed graph onto
one queue, so its timelines cannot): when the greedy branch starts and ends,
how long the reverse loop waits for the vocab head's first dHd chunk, which
stream ends last before Adam.

Enabled only through :func:`enable` (``bench.py --stamps``); disabled, no
stamp kernel is enqueued and captured graphs carry no stamp nodes.  Each
stamp costs one tiny launch (~2 us on its stream), so a stamped step runs a
little slower than the headline one.
"""
import torch

# trainer phases (slot), then the executor's slot bases (csrc/launchers.h
# StampSlot: forward 0..2, backward 0..10)
TRAINER = ['step', 'rollout_enq', 'greedy_begin', 'greedy_end', 'sample_scores', 'loss',
           'bwd_end', 'adam_begin', 'adam_end', 'ptab_end', 'x_end', 'gathered', 'prev_end',
           'comm0', 'comm1', 'comm2']
# executor slots 0..2 (csrc), 3: the decode's prologue (video gates) done (Python)
FWD = ['begin', 'step0', 'end', 'vgate']
BWD = ['begin', 'onehot', 'dhd0', 'dhd', 'loop0', 'loop', 'dw', 'side', 'toksum', 'tokgemm',
       'end']
BASE = {'trainer': 0, 'fwd_sample': 16, 'fwd_greedy': 20, 'bwd': 32}
NSLOTS = 64

_buf = None
_base = None


def names():
    out = {}
    for i, n in enumerate(TRAINER):
        out[BASE['trainer'] + i] = n
    for i, n in enumerate(FWD):
        out[BASE['fwd_sample'] + i] = 'sample.' + n
        out[BASE['fwd_greedy'] + i] = 'greedy.' + n
    for i, n in enumerate(BWD):
        out[BASE['bwd'] + i] = 'bwd.' + n
    return out


def enabled():
    return _buf is not None


def enable(device):
    """Register a stamp buffer on ``device`` (before any graph capture)."""
    global _buf
    from .. import _ext
    _buf = torch.zeros(NSLOTS, dtype=torch.int64, device=device)
    _ext.ops().stamp_buffer(_buf)
    return _buf


def disable():
    global _buf
    if _buf is None:
        return
    from .. import _ext
    _ext.ops().stamp_buffer(torch.empty(0, dtype=torch.int64))
    _ext.ops().set_stamp_base(-1)
    _buf = None


def mark(name):
    """Stamp trainer phase ``name`` on the current stream (no-op if disabled)."""
    if _buf is None:
        return
    from .. import _ext
    if name == 'step':  # the previous step's last stamp, before this step's first
        _buf[TRAINER.index('prev_end')].copy_(_buf[TRAINER.index('ptab_end')])
    _ext.ops().stamp_now(BASE['trainer'] + TRAINER.index(name))


def base(which):
    """Slot base of the next executor call ('fwd_sample', 'fwd_greedy',
    'bwd'; None = no executor stamps)."""
    global _base
    if _buf is None:
        return
    from .. import _ext
    _base = which
    _ext.ops().set_stamp_base(-1 if which is None else BASE[which])


def mark_fwd(name):
    """Stamp decode phase ``name`` (FWD) of the current executor base on the
    current stream (no-op if disabled or no forward base is set)."""
    if _buf is None or _base not in ('fwd_sample', 'fwd_greedy'):
        return
    from .. import _ext
    _ext.ops().stamp_now(BASE[_base] + FWD.index(name))


def read(clear=True):
    """{phase: microseconds after the step stamp} of the last stamped step,
    phases that were not stamped left out (ordered by time)."""
    if _buf is None:
        return {}
    torch.cuda.synchronize(_buf.device)
    v = _buf.cpu().tolist()
    if clear:
        _buf.zero_()
    t0 = v[BASE['trainer']]
    if t0 == 0:
        return {}
    from .. import _ext
    per_us = (_ext.ops().wall_clock_khz() or 100000) / 1000.0  # ticks per microsecond
    out = {nm: (v[i] - t0) / per_us for i, nm in names().items() if v[i] != 0}
    return dict(sorted(out.items(), key=lambda kv: kv[1]))
