"""The event mechanism of the overlapped data-parallel all-reduce
(parallel/dist.py FlatGradBucket.all_reduce, csrc/engine.cpp set_grad_events):
an event recorded INSIDE a captured HIP graph (external event-record node)
orders work that another stream enqueues after the replay behind the node's
position in the graph -- not behind the whole graph, and never before it."""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_external_event_in_replayed_graph_orders_other_stream():
    from cst_captioning_amd import _ext
    ops = _ext.ops()
    dev = torch.device('cuda', 0)
    x = torch.zeros(1 << 20, device=dev)
    y = torch.zeros_like(x)
    a = torch.randn(4096, 4096, device=dev)
    b = torch.empty_like(a)
    side = torch.cuda.Stream(device=dev)
    torch.mm(a, a, out=b)  # (BLAS handle / workspace set up outside the capture)
    x.fill_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        x.fill_(1.0)
        ops.grad_event_record(0, torch.cuda.current_stream().cuda_stream)
        for _ in range(40):  # a few ms of GEMMs after the event
            torch.mm(a, a, out=b)
        x.fill_(2.0)
    seen = []
    for _ in range(4):
        x.zero_()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        g.replay()
        ops.grad_event_wait(0, side.cuda_stream)
        with torch.cuda.stream(side):
            y.copy_(x)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(side)
        ev2 = torch.cuda.Event(enable_timing=True)
        ev2.record()
        torch.cuda.synchronize()
        v = float(y[0])
        assert v in (1.0, 2.0), 'the other stream ran before the event position (%s)' % v
        assert bool((y == v).all())
        seen.append((v, ev0.elapsed_time(ev1), ev0.elapsed_time(ev2)))
    print('value, ms to the copy, ms to the graph end:', seen)
    # after the first replay the copy runs at the event, ahead of the GEMMs
    assert any(v == 1.0 and t1 < t2 for v, t1, t2 in seen[1:]), seen
