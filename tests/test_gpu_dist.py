"""Data parallelism with the fused HIP engine on the GPU: two ranks share the
one GPU of the test box (``CSTCAP_SHARE_GPU=1``, gloo backend on CUDA
tensors -- RCCL needs one GPU per rank).  The all-reduced gradient of the
engine's backward equals the gradient of the mean of the per-shard losses
computed in one process, parameters stay identical across ranks after
optimizer steps, and sharded validation matches a single rank.  The RCCL path
is the same code with the ``nccl`` backend (bench.py under torchrun)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, out, graph, wire='fp32', update='allreduce', mode='xe', worker='dist_worker.py'):
    env = dict(os.environ, CSTCAP_TEST_GRAPH=str(graph), CSTCAP_TEST_WIRE=wire,
               CSTCAP_TEST_DPUPDATE=update, CSTCAP_TEST_MODE=mode)
    env.update(PYTHONPATH=ROOT + os.pathsep + env.get('PYTHONPATH', ''), CSTCAP_SHARE_GPU='1',
               CSTCAP_DIST_BACKEND='gloo', CSTCAP_TEST_IMPL='hip', OMP_NUM_THREADS='4',
               PYTHONFAULTHANDLER='1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node',
           str(world), '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(HERE, worker), out]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return torch.load(out, weights_only=False)


@pytest.mark.parametrize('graph,wire', [(1, 'fp32'), (0, 'fp32'), (1, 'bf16')],
                         ids=['hip_graph_streamed', 'eager_streamed', 'hip_graph_bf16_wire'])
def test_engine_dp_allreduce_matches_single_process(tmp_path, graph, wire):
    """graph=1: steps replayed as HIP graphs, the vocab-head and embedding
    slices all-reduced on the comm stream once the replayed backward's
    external events fire, the rest after the replay; graph=0: the same
    streamed slices behind the eager backward's events; bf16 wire:
    all-to-all + fp32 sum + all-gather of bf16 chunks."""
    os.environ['CSTCAP_TEST_IMPL'] = 'hip'
    r2 = _run(2, str(tmp_path / 'w2.pt'), graph, wire)
    r1 = _run(1, str(tmp_path / 'w1.pt'), graph, wire)
    sys.path.insert(0, HERE)
    import dist_worker as W
    from cst_captioning_amd.parallel import DistContext
    from cst_captioning_amd.train.trainer import Trainer
    dev = torch.device('cuda', 0)
    opt, model, engine, _, _ = W.build(0, 2, dev)
    assert engine is not None, 'the fused engine must be active in this test'
    grads = mags = None
    for k in range(2):
        _, _, _, loader, _ = W.build(k, 2, dev)
        tr = Trainer(opt, model, loader, None, DistContext(device=dev), engine)
        tr.optimizer.zero_grad()
        loss, _ = tr.xe_loss(loader.get_batch())
        loss.backward()
        g = tr.bucket.grad.detach().clone() / 2
        grads = g if grads is None else grads + g
        mags = g.abs() if mags is None else mags + g.abs()
    n = min(grads.numel(), r2['grad'].numel())  # (padding depends on the world size)
    got, ref = r2['grad'][:n], grads[:n].cpu()
    if wire == 'fp32':
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-6)
    else:  # one bf16 rounding of each rank's input and of the sum (+ fp32 noise)
        bound = 2 ** -8 * (mags[:n].cpu() + ref.abs()) + 1e-4 * ref.abs() + 1e-6
        assert ((got - ref).abs() <= bound).all()
    assert r2['same_after_steps']
    assert r1['predictions'] == r2['predictions']


def test_engine_dp_sharded_update_matches_allreduce(tmp_path):
    """--dp_update sharded on the GPU (HIP-graph steps, fused engine): the
    reduce-scattered gradient, the Adam update of each rank's 1/N shard with
    the global clip norm and the all-gather give the parameters and moments of
    the all-reduce path, keep the ranks identical and skip everywhere on one
    rank's NaN loss."""
    os.environ['CSTCAP_TEST_IMPL'] = 'hip'
    a = _run(2, str(tmp_path / 'ar.pt'), 1)
    b = _run(2, str(tmp_path / 'sh.pt'), 1, update='sharded')
    torch.testing.assert_close(b['params_after'], a['params_after'], rtol=1e-5, atol=1e-6)
    for x, y in zip(b['moments'], a['moments']):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-10)
    assert b['same_after_steps'] and b['nan_skip_all']
    assert b['steps_done'] == a['steps_done'] and b['skipped'] == a['skipped'] == 1


def test_engine_dp_scst_step_matches_per_shard_mean(tmp_path):
    """The shipped headline step under data parallelism, on the GPU: fused
    engine, SCST with rank-local rollouts, greedy baselines (side stream) and
    on-GPU CIDEr-D rewards, the step captured and replayed as HIP graphs
    around the eager bucket all-reduce.  The reduced gradient of the replayed
    step equals the mean of the per-shard SCST gradients computed eagerly in
    one process with each rank's sampling seeds (1e-4 relative), and the
    ranks stay identical."""
    os.environ['CSTCAP_TEST_IMPL'] = 'hip'
    r = _run(2, str(tmp_path / 'scst.pt'), 1, mode='scst')
    assert r['graphed'], 'the second step must be a replayed graph'
    sys.path.insert(0, HERE)
    from test_dist import reference_scst_grad
    ref = reference_scst_grad(2, r['p1'], torch.device('cuda', 0)).cpu()
    n = ref.numel()
    err = ((r['grad'][:n] - ref).norm() / ref.norm()).item()
    assert err < 1e-4, err
    assert r['same_after_steps']
    assert not torch.equal(r['rewards'][0], r['rewards'][1])


def test_dp_slice_allreduce_starts_inside_the_backward(tmp_path):
    """The shipped DP path overlaps communication with the backward: in the
    trainer's replayed SCST step (data-parallel code path, the collectives
    of a 1-rank gloo group), the comm stream passes the vocab-head slice's
    event -- where that slice's all-reduce starts -- while the replayed
    backward is still running: the ``comm0`` stamp (enqueued eagerly on the
    comm stream after the event wait) lands before the graph's own
    ``bwd_end`` stamp.  Before round 5 the comm stream first waited for the
    whole replay, which this catches."""
    out = str(tmp_path / 'ov.pt')
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get('PYTHONPATH', ''),
               CSTCAP_TEST_IMPL='hip', PYTHONFAULTHANDLER='1')
    r = subprocess.run([sys.executable, os.path.join(HERE, 'gpu_overlap_worker.py'), out,
                        str(_free_port())], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = torch.load(out, weights_only=False)
    assert r['graphed'], 'the steps must be replayed graphs'
    assert all(r['events_ok'][1:]), r['events_ok']  # captured record nodes of both slices
    assert r['comm_priority'] == 0  # normal priority (the measured default, dist.py)
    for st in r['stamps']:
        assert 'comm0' in st and 'bwd_end' in st, sorted(st.items(), key=lambda kv: kv[1])
        # the vocab head is final under the reverse loop, long before the tail
        assert st['comm0'] < st['bwd_end'] - 50.0, sorted(st.items(), key=lambda kv: kv[1])
        assert st['comm0'] > st.get('bwd.begin', 0.0), sorted(st.items(), key=lambda kv: kv[1])
        # the third slice (W_ih + FeatPool: the video-gate backward runs in
        # the engine on a side stream right after the loop) starts after the
        # loop and before the remainder is reduced (behind adam_begin).  At
        # this small width it lands within ~10 us of bwd_end either side; at
        # the headline width ~290 us before it (scripts/dp_overlap_stamps.py,
        # profiles/r5/dp_model_n8.md)
        assert 'comm2' in st and st['bwd.loop'] < st['comm2'] < st['adam_begin'], \
            sorted(st.items(), key=lambda kv: kv[1])
        assert r['n_groups'] == 3


def test_dp_step_over_rccl_one_rank(tmp_path):
    """The same replayed DP step with the collectives on RCCL (backend
    ``nccl``, a 1-rank communicator -- a one-GPU box cannot hold two RCCL
    ranks): the streamed slice all-reduces are real RCCL launches on the
    high-priority comm stream, issued around the replayed graphs; the steps
    complete, the weights stay finite and the slice order holds as under
    gloo."""
    out = str(tmp_path / 'ov_rccl.pt')
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get('PYTHONPATH', ''),
               CSTCAP_TEST_IMPL='hip', PYTHONFAULTHANDLER='1')
    r = subprocess.run([sys.executable, os.path.join(HERE, 'gpu_overlap_worker.py'), out,
                        str(_free_port()), 'nccl'], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = torch.load(out, weights_only=False)
    assert r['backend'] == 'nccl' and r['graphed'] and r['finite']
    assert all(r['events_ok'][1:]), r['events_ok']
    for st in r['stamps']:
        # at this small width the vocab head's weight gradients (after the
        # persistent reverse loop) end just before the backward does; the
        # slice's all-reduce starts right after them, not after the replay's
        # remainder (normal-priority comm stream)
        assert st['bwd.dw'] <= st['comm0'] < st['bwd_end'] + 100.0, \
            sorted(st.items(), key=lambda kv: kv[1])


def test_dp_ring_standin_overlaps_backward_at_default_priority(tmp_path):
    """A collective-shaped stand-in (32 copying workgroups for 300 us, the
    engine's busy_copy kernel) where the vocab-head slice's RCCL ring runs,
    on the comm stream at the default (normal) priority: it starts right after
    the vocab head's gradients are final, not behind the replay's remainder
    (bwd.dw <= comm0 < bwd_end + 100 us) on every stamped step, and the steps
    complete with finite weights.  The priority default itself comes
    from scripts/dp_standin.py at the headline shape (high priority slowed
    the whole step 1.7x, profiles/r6/dp_standin_rccl.json)."""
    out = str(tmp_path / 'ov_standin.pt')
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get('PYTHONPATH', ''),
               CSTCAP_TEST_IMPL='hip', PYTHONFAULTHANDLER='1', CSTCAP_TEST_STANDIN='32,300')
    r = subprocess.run([sys.executable, os.path.join(HERE, 'gpu_overlap_worker.py'), out,
                        str(_free_port()), 'nccl'], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = torch.load(out, weights_only=False)
    assert r['graphed'] and r['finite'] and r['comm_priority'] == 0
    assert all(r['events_ok'][1:]), r['events_ok']
    for st in r['stamps']:
        assert st['bwd.dw'] <= st['comm0'] < st['bwd_end'] + 100.0, \
            sorted(st.items(), key=lambda kv: kv[1])
