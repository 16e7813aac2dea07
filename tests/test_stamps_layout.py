"""Slot layout of the device timeline stamps (utils/stamps.py): the trainer
phases and the executor's forward / backward slots (csrc/launchers.h
StampSlot) never overlap and fit the buffer; disabled, the helpers do
nothing (no extension call, no GPU)."""
from cst_captioning_amd.utils import stamps


def test_slots_are_disjoint_and_fit():
    names = stamps.names()
    assert len(names) == len(set(names.values()))
    assert max(names) < stamps.NSLOTS
    tr = [stamps.BASE['trainer'] + i for i in range(len(stamps.TRAINER))]
    fs = [stamps.BASE['fwd_sample'] + i for i in range(len(stamps.FWD))]
    fg = [stamps.BASE['fwd_greedy'] + i for i in range(len(stamps.FWD))]
    bw = [stamps.BASE['bwd'] + i for i in range(len(stamps.BWD))]
    allslots = tr + fs + fg + bw
    assert len(allslots) == len(set(allslots))
    # the executor's backward uses 11 slots (STAMP_BWD_BEGIN .. STAMP_BWD_END),
    # its forward 3 (STAMP_FWD_*) plus the decode prologue's Python stamp
    assert len(stamps.BWD) == 11 and len(stamps.FWD) == 4
    assert stamps.FWD[:3] == ['begin', 'step0', 'end']
    # each forward base has room for its 4 slots before the next base
    assert stamps.BASE['fwd_greedy'] - stamps.BASE['fwd_sample'] >= len(stamps.FWD)
    assert stamps.BASE['bwd'] - stamps.BASE['fwd_greedy'] >= len(stamps.FWD)
    assert stamps.BASE['fwd_sample'] >= len(stamps.TRAINER)


def test_disabled_helpers_are_no_ops():
    assert not stamps.enabled()
    stamps.mark('step')
    stamps.mark_fwd('vgate')
    stamps.base('bwd')
    stamps.base(None)
    assert stamps.read() == {}
    stamps.disable()
