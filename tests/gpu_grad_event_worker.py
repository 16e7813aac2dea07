"""Worker of tests/test_gpu_grad_events.py, run in a fresh process: a
long-lived test process has created many streams, which the HIP runtime
multiplexes over its few hardware queues -- a side stream sharing the graph's
queue then runs behind the whole replay whatever the event says."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
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
    print('grad-event ok')


if __name__ == '__main__':
    main()
