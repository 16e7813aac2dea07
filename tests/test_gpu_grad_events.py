"""The event mechanism of the overlapped data-parallel all-reduce
(parallel/dist.py FlatGradBucket.all_reduce, csrc/engine.cpp set_grad_events):
an event recorded INSIDE a captured HIP graph (external event-record node)
orders work that another stream enqueues after the replay behind the node's
position in the graph -- not behind the whole graph, and never before it.
(Run in a fresh process: see gpu_grad_event_worker.py.)"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_external_event_in_replayed_graph_orders_other_stream():
    res = subprocess.run([sys.executable, os.path.join(HERE, 'gpu_grad_event_worker.py')],
                         capture_output=True, text=True, timeout=110)
    print(res.stdout)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    assert 'grad-event ok' in res.stdout
