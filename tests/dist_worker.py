"""Worker for tests/test_dist.py, launched by torchrun (gloo on CPU, or RCCL
on GPUs): one XE gradient all-reduce, two optimizer steps, and a sharded
validation.  Writes rank 0's results to ``argv[1]`` (torch.save)."""
import os
import sys

import torch

from cst_captioning_amd.cli import build_model, load_splits
from cst_captioning_amd.config import parse_opts
from cst_captioning_amd.data import CaptionLoader
from cst_captioning_amd.parallel import init_distributed
from cst_captioning_amd.train.trainer import Trainer

ARGS = ['--synthetic', 'msvd', '--synthetic_videos', '24', '--synthetic_vocab', '40',
        '--seq_length', '10', '--rnn_size', '64', '--input_encoding_size', '64',
        '--feat_dims', '16', '8', '--batch_size', '4', '--train_seq_per_img', '3',
        '--test_batch_size', '3', '--test_seq_per_img', '3', '--beam_size', '2',
        '--impl', os.environ.get('CSTCAP_TEST_IMPL', 'torch'), '--loglevel', 'WARNING',
        '--drop_prob_lm', '0', '--cuda_graph', os.environ.get('CSTCAP_TEST_GRAPH', '1'),
        '--learning_rate', '1e-3', '--language_eval', '0',
        '--grad_wire', os.environ.get('CSTCAP_TEST_WIRE', 'fp32'),
        '--dp_update', os.environ.get('CSTCAP_TEST_DPUPDATE', 'allreduce')]


def build(rank, world, device):
    opt = parse_opts(ARGS)
    torch.manual_seed(1234 + rank)  # different init per rank: broadcast must fix it
    tr, va, _ = load_splits(opt)
    loader = CaptionLoader(tr, opt.batch_size, opt.train_seq_per_img, 'train', device,
                           rank, world, opt.seed)
    opt.vocab, opt.vocab_size = loader.get_vocab(), loader.get_vocab_size()
    opt.seq_length, opt.feat_dims = loader.get_seq_length(), loader.get_feat_dims()
    model, engine = build_model(opt, device)
    val = CaptionLoader(va, opt.test_batch_size, opt.test_seq_per_img, 'test', device)
    return opt, model, engine, loader, val


def fix_seeds(tr, rank, dev):
    """Rank-dependent but reproducible sampling: the fused engine reads its
    (dropout, sampling) seeds and FeatPool's from fixed device tensors; the
    PyTorch path draws from the global generator, seeded per step by the
    caller."""
    from cst_captioning_amd.ops import featpool as fp
    fixed = torch.tensor([4242 + 17 * rank, 777 + 31 * rank], dtype=torch.int32, device=dev)
    if tr.engine is not None:
        tr.engine._rng = lambda d: fixed
    fp.SEED_SOURCE = lambda d: fixed
    return fixed


def main_scst(out):
    """SCST data parallelism (CSTCAP_TEST_MODE=scst): rank-local rollouts,
    greedy baselines and CIDEr-D rewards.  Step 1 (eager: the warm-up of the
    schedule key), then step 2 (with --cuda_graph 1 on the GPU: captured and
    replayed).  Saves the parameters before step 2 and the all-reduced mean
    gradient of step 2, which tests/test_dist.py compares with the mean of
    the per-shard SCST gradients computed in one process."""
    ctx = init_distributed()
    opt, model, engine, loader, val = build(ctx.rank, ctx.world_size, ctx.device)
    tr = Trainer(opt, model, loader, val, ctx, engine)
    tr.rl_training = True
    fix_seeds(tr, ctx.rank, ctx.device)
    torch.manual_seed(555 + ctx.rank)
    tr.train_step(loader.get_batch(), 0)
    p1 = tr.bucket.data.detach().cpu().clone()
    torch.manual_seed(999 + ctx.rank)
    out_step = tr.train_step(loader.get_batch(), 0)
    grad = (tr.bucket.grad * tr.optimizer.grad_scale).detach().cpu().clone()
    flat = tr.bucket.data.detach().cpu().clone()
    allp = ctx.all_gather_object(flat)
    same = all(torch.equal(allp[0], q) for q in allp)
    rewards = ctx.all_gather_object(out_step['reward'].detach().cpu().clone())
    graphed = tr._graph is not None
    if ctx.is_main:
        torch.save({'p1': p1, 'grad': grad, 'same_after_steps': same, 'rewards': rewards,
                    'graphed': graphed, 'world': ctx.world_size}, out)
    ctx.destroy()


def main(out):
    if os.environ.get('CSTCAP_TEST_MODE') == 'scst':
        return main_scst(out)
    ctx = init_distributed()
    opt, model, engine, loader, val = build(ctx.rank, ctx.world_size, ctx.device)
    tr = Trainer(opt, model, loader, val, ctx, engine)  # C1 broadcast happens here
    init = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
    res = tr.validate(val)  # C4, on the broadcast initial weights
    # one all-reduced XE gradient
    data = loader.get_batch()
    tr.optimizer.zero_grad()
    loss, _ = tr.xe_loss(data)
    loss.backward()
    # drop the autograd graph: a graph kept alive across the HIP-graph capture
    # of the next train_step pins AccumulateGrad nodes to the default stream
    del loss
    tr.bucket.all_reduce(ctx)
    # (the fp32 path sums; the optimizer applies the 1/N)
    grad = (tr.bucket.grad * tr.optimizer.grad_scale).detach().cpu().clone()
    # two full steps: parameters must stay identical on every rank
    for _ in range(2):
        tr.train_step(loader.get_batch(), 0)
    flat = tr.bucket.data.detach().cpu().clone()
    allp = ctx.all_gather_object(flat)
    same = all(torch.equal(allp[0], p) for p in allp)
    tr.optimizer.consolidate(ctx)  # (sharded update: gather the moment shards)
    moments = (tr.optimizer.exp_avg.detach().cpu().clone(),
               tr.optimizer.exp_avg_sq.detach().cpu().clone())
    steps_done = tr.optimizer.step_count
    # NaN guard: only the last rank's loss is NaN; its skip flag rides the
    # gradient all-reduce, so every rank must skip the update
    data = loader.get_batch()
    if ctx.rank == ctx.world_size - 1:
        data['masks'] = data['masks'] * float('nan')
    tr.train_step(data, 0)
    after = tr.bucket.data.detach().cpu().clone()
    nan_skip = all(ctx.all_gather_object(torch.equal(after, flat)))
    # C3: logged scalars are the mean over ranks (rank r logs loss r + 1,
    # reward row means r, m = 2r, b = -r)
    r = float(ctx.rank)
    tr.rl_training = True
    logged = tr.reduce_log_scalars({'loss': torch.tensor(r + 1.0),
                                    'reward': torch.full((6,), r), 'm': 2 * r, 'b': -r})
    step_out = tr.train_step(loader.get_batch(), 0)
    tr.rl_training = False
    xe_logged = tr.reduce_log_scalars(step_out)
    xe_losses = ctx.all_gather_object(float(step_out['loss']))
    if ctx.is_main:
        torch.save({'init': init, 'grad': grad, 'same_after_steps': same, 'nan_skip_all': nan_skip,
                    'predictions': res['predictions'], 'loss': res['scores']['Loss'],
                    'world': ctx.world_size, 'logged': logged, 'xe_logged': xe_logged,
                    'xe_losses': xe_losses, 'params_after': flat, 'moments': moments,
                    'steps_done': steps_done, 'skipped': int(tr.optimizer.skipped())}, out)
    ctx.destroy()


if __name__ == '__main__':
    main(sys.argv[1])
