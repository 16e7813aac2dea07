"""Device timeline stamps (utils/stamps.py, csrc/kernels/stamp.hip) inside
the captured SCST step: every phase is stamped, the stream-ordered phases
come out in order, and disabling them leaves a graph without stamp nodes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_stamps_in_graph_step_are_ordered():
    from cst_captioning_amd.utils import stamps
    from test_gpu_graph import _setup
    stamps.enable(torch.device('cuda'))
    try:
        tr, loader = _setup(rl=True, graph=1)
        for _ in range(3):  # eager once, capture, replay
            tr.train_step(loader.get_batch(), 0)
        assert tr._graph is not None
        stamps.read()  # clear the capture step's values
        tr.train_step(loader.get_batch(), 0)
        t = stamps.read()
    finally:
        stamps.disable()
    for k in ('sample.begin', 'sample.end', 'greedy.begin', 'greedy.end', 'greedy_begin',
              'greedy_end', 'loss', 'bwd.begin', 'bwd.loop', 'bwd.end', 'bwd_end',
              'adam_begin', 'adam_end'):
        assert k in t, (k, t)
    order = ['sample.begin', 'sample.step0', 'sample.end', 'sample_scores', 'loss',
             'bwd.begin', 'bwd.loop0', 'bwd.loop', 'bwd.toksum', 'bwd.end', 'bwd_end',
             'adam_begin', 'adam_end']
    vals = [t[k] for k in order]
    assert vals == sorted(vals), t
    assert t['greedy.begin'] <= t['greedy.end'] <= t['loss']
    assert t['bwd.dhd0'] <= t['bwd.loop0'] and t['bwd.dw'] <= t['bwd_end']
    assert 0 < t['adam_end'] < 1e6  # microseconds, one step


def test_stamps_disabled_enqueue_nothing():
    from cst_captioning_amd import _ext
    from cst_captioning_amd.utils import stamps
    assert not stamps.enabled()
    buf = torch.zeros(4, dtype=torch.int64, device='cuda')
    _ext.ops().stamp_now(0)  # no buffer registered: no launch, nothing written
    torch.cuda.synchronize()
    assert int(buf.sum()) == 0
    stamps.enable(torch.device('cuda'))
    try:
        stamps.mark('step')
        stamps.mark('loss')
        torch.cuda.synchronize()
        v = stamps._buf.cpu()
        assert v[0] > 0 and v[stamps.TRAINER.index('loss')] >= v[0]
    finally:
        stamps.disable()
