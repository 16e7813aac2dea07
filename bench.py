#!/usr/bin/env python3
"""Headline benchmark: SCST training captions/sec (whole job).

Workload (BASELINE.json / BASELINE.md): MSR-VTT-shaped CaptionModel
(``concat``, 4 modalities resnet 2048 / c3d 4096 / mfcc 1024 / category 300,
LSTM 512, embedding 512, vocab 10,509, max length 30, dropout 0.5),
B = 64 videos x 20 captions = 1,280 caption rows per GPU per step (weak
scaling), SCST recipe of the reference README (``USE_RL=1 USE_CST=0
USE_MIXER=1 MIXER_FROM=1 USE_EOS=1``): multinomial rollout from t=1, greedy
baseline, CIDEr-D reward, REINFORCE loss, backward, gradient all-reduce,
clip 0.25, Adam.  Synthetic data (6,513 videos x 20 captions, Zipf
captions) and random-init weights: there is no network for datasets or
checkpoints.

Every step inside the timed region does ALL of the above (nothing cached,
no layers skipped).  Timed region: barrier + synchronize, K steps, barrier +
synchronize; the MAX over ranks is reported.

BASELINE.json's metric names the LSTM-attn decoder while the headline config
(the reference default ``--num_chunks 1``) mean-pools the features, so an SCST
run also times the 8-frame temporal-attention config of the same job (same K
and W, after the headline run's buffers are freed) and reports it as the
``att8`` field ({value, ms_per_step, ...}); ``--att8 0`` skips it.  After the
timed steps the headline run also times the beam-5 evaluation decode of one
batch (BASELINE config 5) on the weights it trained: the ``beam5`` field
({videos_per_s (whole job), ms_per_batch, ...}); ``--beam5 0`` skips it.

Modes:
  --impl hip   (default) fused HIP engine + on-GPU CIDEr-D, bf16 MFMA
  --impl torch --reward cpu --precision fp32 --dedupe_greedy 0
               reference semantics (PyTorch ops, CPU CIDEr-D in Python):
               the baseline BASELINE.md asks to beat.
  --impl torch --precision bf16
               same-precision PyTorch baseline: PyTorch decoder ops under bf16
               autocast with the on-GPU CIDEr-D reward, so the kernels'
               speed-up is separated from the precision change.

Launch: ``python bench.py`` (1 GPU), ``python bench.py --gpus N`` (starts
the PyTorch launcher with N ranks as a child process), or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1
--master-port P bench.py --gpus N``.  Every rank checks that the job's world
size equals ``--gpus`` and exits non-zero otherwise.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# BASELINE.md publishes no number for the metric (BASELINE.json "published":
# {}), so vs_baseline is null; the self-measured reference-semantics run is
# reported as a separate ratio
BASELINE_FILE = os.path.join(REPO, 'profiles', 'reference_semantics_baseline.json')
BCMR_FILE = os.path.join(REPO, 'profiles', 'bench_bcmr_msrvtt_seed123.npz')


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--impl', default='hip', choices=['hip', 'torch'])
    p.add_argument('--reward', default='gpu', choices=['gpu', 'cpu'])
    p.add_argument('--precision', default='bf16', choices=['bf16', 'fp32'])
    p.add_argument('--mode', default='scst', choices=['scst', 'cst', 'xe', 'beam'],
                   help='beam: evaluation decode throughput (beam search, --beam_size) '
                        'instead of a training step')
    p.add_argument('--beam_size', type=int, default=5)
    p.add_argument('--dedupe_greedy', type=int, default=1)
    p.add_argument('--batch_size', type=int, default=64)
    p.add_argument('--videos', type=int, default=6513)
    p.add_argument('--vocab', type=int, default=10509)
    p.add_argument('--seed', type=int, default=123)
    p.add_argument('--num_chunks', type=int, default=1,
                   help='frames per video; > 1 enables temporal attention (the reference '
                        'default, and the headline config, is 1: mean-pooled features)')
    p.add_argument('--cuda_graph', type=int, default=1,
                   help='replay the training step as a captured HIP graph (fused engine)')
    p.add_argument('--rnn_type', default='lstm', choices=['lstm', 'gru', 'rnn'],
                   help='decoder cell (headline: lstm)')
    p.add_argument('--model_type', default='concat', choices=['concat', 'standard', 'manet'],
                   help="headline: concat; 'standard' uses input_encoding_size = F * 512")
    p.add_argument('--num_layers', type=int, default=1)
    p.add_argument('--grad_wire', default='fp32', choices=['fp32', 'bf16'],
                   help='DP gradient reduction: fp32 all-reduce or bf16 wire / fp32 accumulation')
    p.add_argument('--att8', type=int, default=1,
                   help='scst with --num_chunks 1: also time the 8-frame temporal-attention '
                        'config in the same invocation and report it as the "att8" field')
    p.add_argument('--beam5', type=int, default=1,
                   help='scst, headline config: also time the beam-5 evaluation decode of one '
                        'batch (BASELINE config 5) on the trained weights and report it as the '
                        '"beam5" field')
    p.add_argument('--cst', type=int, default=1,
                   help='scst, headline config: also time the CST recipe (README "CST_MS_SCB": '
                        'consensus baseline from the GT captions, --scb_baseline) in the same '
                        'invocation and report it as the "cst" field')
    p.add_argument('--xe', type=int, default=1,
                   help='scst, headline config: also time the XE recipe (BASELINE config 2, the '
                        'reference\'s cross-entropy warm-up stage: teacher forcing, same '
                        'model / batch) in the same invocation and report it as the "xe" field')
    p.add_argument('--comm_priority', default='normal', choices=['high', 'normal'],
                   help='data parallelism: priority of the gradient all-reduce stream (high '
                        'measured 1.7x slower per step, profiles/r6/dp_standin_rccl.json)')
    p.add_argument('--scb_baseline', type=int, default=1, choices=[1, 2],
                   help='CST baseline: 1 = GT consensus scores (CST_MS_SCB), 2 = the samples\' own '
                        'scores (CST_MS_SCB(*))')
    p.add_argument('--json_out', default='')
    p.add_argument('--profile_phases', type=int, default=0,
                   help='print the mean per-phase GPU time (HIP events) of the timed steps')
    p.add_argument('--stamps', type=int, default=0,
                   help='N > 0: device timeline stamps (utils/stamps.py) captured into the '
                        'graph; after the timed steps, N more steps are stamped and the mean '
                        'phase times (us after the step start) are printed to stderr and '
                        'stored as "stamps_us" (diagnostic: stamps add ~2 us per phase)')
    p.add_argument('--sync_each', type=int, default=0,
                   help='diagnostic: synchronise after every timed step (isolated steps; '
                        'not the headline measurement)')
    p.add_argument('--sync_debug', type=int, default=0,
                   help='after warmup: report host-synchronising calls and host enqueue time of one step')
    return p.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def relaunch_if_needed(a):
    """``python bench.py --gpus N`` with no torchrun environment: start the
    PyTorch launcher with N ranks as a CHILD process and exit with its code.
    This runs before torch is imported, so the parent never touches the GPU
    (no exec from a process that initialised HIP)."""
    if a.gpus <= 1 or 'WORLD_SIZE' in os.environ:
        return
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(a.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def run_config(a, ctx, num_chunks, sync, sync_debug=0, mode=None):
    """Build the dataset, model, engine and trainer for ``num_chunks`` frames
    per video, run ``a.warmup`` untimed and ``a.steps`` timed steps (barrier +
    synchronize on both sides, MAX over ranks) and free the GPU buffers.
    ``mode`` overrides ``a.mode`` (the extra CST run of an SCST bench)."""
    mode = mode or a.mode
    import gc
    import torch
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import CaptionLoader, make_synthetic
    from cst_captioning_amd.cli import build_model, seed_everything
    from cst_captioning_amd.train.trainer import Trainer

    seed_everything(a.seed, ctx.rank)
    t_gen = time.time()
    ds = make_synthetic('msrvtt', num_videos=a.videos, vocab_size=a.vocab, seed=a.seed,
                        num_chunks=num_chunks)
    bcmr_src = None
    if mode == 'cst' and a.scb_baseline == 1:
        # GT consensus scores of CST_MS_SCB: prepro/evalscores.py's coco CIDEr
        # of each GT caption against the video's other captions, cached for
        # the bench dataset (scripts/make_bench_bcmr.py; the reference reads
        # them from a file as well, dataloader.py:62-71)
        import numpy as np
        z = np.load(BCMR_FILE, allow_pickle=False) if os.path.exists(BCMR_FILE) else None
        if (z is not None and int(z['seed']) == a.seed and int(z['videos']) == a.videos
                and int(z['vocab']) == a.vocab):
            ds.bcmrscores = np.asarray(z['CIDEr'], dtype=np.float64)
            bcmr_src = 'prepro/evalscores.py (cached: %s)' % os.path.relpath(BCMR_FILE, REPO)
        else:
            from cst_captioning_amd.prepro.evalscores import compute_consensus_scores
            ds.bcmrscores = compute_consensus_scores(ds.gt_refs, 20, True, tokenize=False,
                                                     metrics=('CIDEr',))['CIDEr']
            bcmr_src = 'prepro/evalscores.py'
    t_gen = time.time() - t_gen
    S = 20
    opt = default_opts(
        batch_size=a.batch_size, train_seq_per_img=S, test_seq_per_img=S, rnn_size=512,
        input_encoding_size=512 * len(ds.feat_dims) if a.model_type == 'standard' else 512,
        drop_prob_lm=0.5, rnn_type=a.rnn_type, num_layers=a.num_layers, learning_rate=1e-4,
        grad_clip=0.25, model_type=a.model_type, num_chunks=num_chunks, eval_metric='CIDEr',
        max_epochs=10 ** 9, print_log_interval=0,
        use_rl=1 if mode != 'xe' else 0, use_rl_after=0, use_cst=1 if mode == 'cst' else 0,
        use_mixer=1, mixer_from=1, use_eos=1, expand_feat=1, scb_baseline=a.scb_baseline,
        scb_captions=S,
        impl=a.impl, precision=a.precision, reward_device=a.reward,
        dedupe_greedy=a.dedupe_greedy, seed=a.seed, loglevel='WARNING', save_last=0,
        profile_phases=a.profile_phases, cuda_graph=a.cuda_graph, grad_wire=a.grad_wire,
        comm_priority=a.comm_priority)
    opt.vocab = {i: w for i, w in enumerate(ds.vocab)}
    opt.vocab_size = ds.vocab_size
    opt.seq_length = ds.seq_length
    opt.feat_dims = ds.feat_dims
    dev = ctx.device
    loader = CaptionLoader(ds, a.batch_size, S, 'train', dev, ctx.rank, ctx.world_size, a.seed)
    model, engine = build_model(opt, dev, a.impl)
    trainer = Trainer(opt, model, loader, None, ctx, engine)
    trainer.rl_training = mode != 'xe'
    n_params = sum(p.numel() for p in model.parameters())

    def step():
        data = loader.get_batch()
        if mode == 'beam':  # BASELINE config 5: beam-5 evaluation decode
            model.eval()
            with torch.no_grad():
                seq, _ = model.sample(data['feats'], {'beam_size': a.beam_size})
            return {'loss': seq.float().mean()}
        return trainer.train_step(data, 0)

    if a.stamps and dev.type == 'cuda':
        from cst_captioning_amd.utils import stamps as stamps_mod
        stamps_mod.enable(dev)  # before the first step: the captured graph carries them
    for _ in range(a.warmup):
        out = step()
    sync()
    if sync_debug and dev.type == 'cuda':
        import warnings
        warnings.simplefilter('always')
        torch.cuda.set_sync_debug_mode('warn')
        th = time.perf_counter()
        step()
        th = time.perf_counter() - th
        torch.cuda.set_sync_debug_mode(0)
        sync()
        tg = time.perf_counter()
        step()
        sync()
        tg = time.perf_counter() - tg
        print('sync_debug: host enqueue %.3f ms, synced step %.3f ms' % (th * 1e3, tg * 1e3),
              file=sys.stderr, flush=True)
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    phases = {}
    for _ in range(a.steps):
        out = step()
        if a.sync_each:
            sync()
        if a.profile_phases:  # reads the events: synchronises, diagnostic only
            for k, v in trainer.timer.summary().items():
                phases[k] = phases.get(k, 0.0) + v / a.steps
    sync()
    ctx.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt = ctx.max_scalar(dt)
    stamp_mean = {}
    if a.stamps and dev.type == 'cuda':
        for _ in range(a.stamps):
            # two back-to-back steps per read: the second one's 'prev_end' is
            # the first one's last stamp (> 0: the two steps overlapped)
            step()
            step()
            for k, v in stamps_mod.read().items():
                stamp_mean[k] = stamp_mean.get(k, 0.0) + v / a.stamps
        stamps_mod.disable()
        stamp_mean = {k: round(v, 1) for k, v in sorted(stamp_mean.items(), key=lambda kv: kv[1])}
        print('stamps (us after the step stamp, mean of %d steps, %d frames):' % (a.stamps, num_chunks),
              file=sys.stderr)
        for k, v in stamp_mean.items():
            print('  %9.1f  %s' % (v, k), file=sys.stderr)
        sys.stderr.flush()
    beam = None
    if (a.beam5 and mode == 'scst' and num_chunks == 1 and engine is not None
            and dev.type == 'cuda'):
        # BASELINE config 5: beam-5 evaluation decode of one batch (64 videos
        # per rank) with the weights the timed steps trained
        model.eval()
        bdata = loader.get_batch()
        nb = max(a.steps, 5)
        with torch.no_grad():
            for _ in range(3):
                model.sample(bdata['feats'], {'beam_size': 5})
            sync()
            ctx.barrier()
            sync()
            tb = time.perf_counter()
            for _ in range(nb):
                model.sample(bdata['feats'], {'beam_size': 5})
            sync()
            ctx.barrier()
            sync()
        tb = ctx.max_scalar(time.perf_counter() - tb)
        beam = {'videos_per_s': round(a.batch_size * ctx.world_size * nb / tb, 1),
                'ms_per_batch': round(tb / nb * 1e3, 3), 'videos_per_batch_per_gpu': a.batch_size,
                'beam_size': 5, 'decodes': nb}
        model.train()
    dev_err = None
    if engine is not None and dev.type == 'cuda':
        # failed cross-workgroup hand-offs counted on the device over every
        # step of this run (csrc/engine.cpp device_errors); 0 = none
        from cst_captioning_amd import _ext
        dev_err = int(_ext.ops().device_errors(dev.index or 0))
    res = {'dt': dt, 'ms': dt / a.steps * 1e3, 'loss': float(out['loss']),
           'device_errors': dev_err,
           'caps': a.batch_size * S * ctx.world_size * a.steps / dt,
           'vids': a.batch_size * ctx.world_size * a.steps / dt, 'phases': phases,
           'skipped': int(trainer.optimizer.skipped().item()),
           'exp_fix': int(engine.exp_fix_rows.item()) if engine is not None else None,
           'graph': int(trainer._graph is not None), 'n_params': n_params, 't_gen': t_gen,
           'bf16': engine is not None or trainer.autocast_bf16, 'stamps': stamp_mean,
           'beam5': beam, 'bcmr': bcmr_src, 'blaslt': _blaslt_choices(engine)}
    del trainer, model, engine, loader, ds, step, out
    gc.collect()
    if dev.type == 'cuda':
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return res


def _blaslt_choices(engine):
    """The hipBLASLt algorithm the X = E W plan chose per shape (candidate
    index in the heuristic's list, its measured us): recorded so a run's
    numerics can be reproduced with CSTCAP_BLASLT_ALGO=<index>."""
    if engine is None:
        return None
    from cst_captioning_amd import _ext
    try:
        return [{'m': int(c[0]), 'n': int(c[1]), 'k': int(c[2]), 'candidate': int(c[3]),
                 'us': round(c[4], 1), 'batch': int(c[5])}
                for c in _ext.ops().gemm_tuned_choices()]
    except Exception:
        return None


def main():
    a = parse()
    relaunch_if_needed(a)
    import torch
    from cst_captioning_amd.parallel import init_distributed

    ctx = init_distributed()
    if ctx.world_size != a.gpus:
        print('bench.py: --gpus %d but the job has %d rank(s) (WORLD_SIZE=%s)'
              % (a.gpus, ctx.world_size, os.environ.get('WORLD_SIZE')), file=sys.stderr)
        ctx.destroy()
        sys.exit(3)
    if a.impl == 'torch':
        os.environ['CSTCAP_ALLOW_TORCH_FALLBACK'] = '1'
    sync = torch.cuda.synchronize if ctx.device.type == 'cuda' else (lambda: None)
    main_run = run_config(a, ctx, a.num_chunks, sync, sync_debug=a.sync_debug)
    att8 = None
    if a.att8 and a.mode == 'scst' and a.num_chunks == 1:
        # the temporal-attention variant of the same job (8 frames per video),
        # same steps / warmup, measured after the headline run's buffers are freed
        r = run_config(a, ctx, 8, sync)
        att8 = {'value': round(r['caps'], 2), 'ms_per_step': round(r['ms'], 3),
                'temporal_attention_frames': 8, 'final_loss': r['loss'],
                'skipped_steps': r['skipped'], 'device_errors': r['device_errors']}
        if r['stamps']:
            att8['stamps_us'] = r['stamps']
    cst = None
    if a.cst and a.mode == 'scst' and a.num_chunks == 1:
        # the CST recipe of the same job (the reference's namesake), same steps
        # / warmup, after the previous runs' buffers are freed
        r = run_config(a, ctx, 1, sync, mode='cst')
        cst = {'value': round(r['caps'], 2), 'ms_per_step': round(r['ms'], 3),
               'recipe': 'CST_MS_SCB' if a.scb_baseline == 1 else 'CST_MS_SCB(*)',
               'scb_baseline': a.scb_baseline, 'scb_captions': 20, 'bcmr': r['bcmr'],
               'final_loss': r['loss'], 'skipped_steps': r['skipped']}
    xe = None
    if a.xe and a.mode == 'scst' and a.num_chunks == 1:
        # BASELINE config 2: the XE (teacher-forced cross-entropy) stage of the
        # same job on the same fused path (graph replay, X after the forward)
        r = run_config(a, ctx, 1, sync, mode='xe')
        xe = {'value': round(r['caps'], 2), 'ms_per_step': round(r['ms'], 3),
              'recipe': 'XE (teacher forcing)', 'final_loss': r['loss'],
              'skipped_steps': r['skipped'], 'cuda_graph': r['graph'],
              'device_errors': r['device_errors']}
    dt, ms, caps, vids = main_run['dt'], main_run['ms'], main_run['caps'], main_run['vids']
    loss, n_params, t_gen = main_run['loss'], main_run['n_params'], main_run['t_gen']
    S = 20
    def _value(path):
        if not os.path.exists(path):
            return None
        with open(path) as f:
            return json.load(f).get('value')
    ref_sem = _value(BASELINE_FILE)
    if a.mode == 'beam':
        metric, value, unit = 'beam-%d evaluation decode videos/sec (whole job)' % a.beam_size, \
            vids, 'videos/s'
    elif a.mode == 'scst':
        metric, value, unit = ('SCST training captions/sec (whole node), MSR-VTT LSTM-attn at '
                               '1/2/4/8 MI355X', caps, 'captions/s')
    else:
        metric, value, unit = '%s training captions/sec (whole job)' % a.mode.upper(), caps, \
            'captions/s'
    rec = {
        'metric': metric,
        'value': round(value, 2), 'unit': unit, 'n_gpus': ctx.world_size,
        'steps': a.steps, 'warmup': a.warmup, 'ms_per_step': round(ms, 3),
        'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': None,  # no published number
        # self-measured, same job on one MI355X, NOT a published baseline:
        # reference semantics (PyTorch ops, fp32, CPU CIDEr-D in Python;
        # profiles/reference_semantics_baseline.json)
        'vs_reference_semantics_1gpu': (round(caps / ctx.world_size / ref_sem, 2)
                                        if (ref_sem and a.mode == 'scst') else None),
        # effective compute dtype: the fused engine is bf16; the PyTorch path is
        # bf16 under autocast with --precision bf16 on a GPU, else fp32
        'dtype': 'bf16' if main_run['bf16'] else 'fp32',
        'data': 'synthetic (MSR-VTT-shaped, random-init weights)',
        'config': {'model': 'CaptionModel %s %s%s-512 (resnet+c3d+mfcc+category, '
                            'V=%d, L=30)' % (a.model_type, a.rnn_type.upper(),
                                             'x%d' % a.num_layers if a.num_layers > 1 else '',
                                             a.vocab),
                   'global_batch': a.batch_size * (1 if a.mode == 'beam' else S) * ctx.world_size,
                   'videos_per_gpu': a.batch_size, 'seq_per_img': S, 'seq_len': 30,
                   'parallelism': 'dp%d' % ctx.world_size, 'impl': a.impl,
                   'reward': a.reward, 'mode': a.mode, 'params': n_params,
                   'dedupe_greedy': a.dedupe_greedy,
                   'cuda_graph': main_run['graph'],
                   'grad_wire': a.grad_wire,
                   'temporal_attention_frames': a.num_chunks if a.num_chunks > 1 else None},
        'final_loss': loss, 'datagen_s': round(t_gen, 1),
        # optimizer updates the NaN guard skipped (non-finite loss or gradient
        # norm) over warmup + timed steps, all ranks agree (adam.hip)
        'skipped_steps': main_run['skipped'],
        # exp-store rows the backward recomputed (LSE jump > 60 between steps)
        'exp_fix_rows': main_run['exp_fix'],
        'world_size_seen': ctx.world_size, 'backend': ctx.backend or 'none',
        'comm_priority': a.comm_priority,
        # failed cross-workgroup hand-offs counted on the device (bounded flag
        # polls that gave up) over the headline run; must be 0
        'device_errors': main_run['device_errors'],
    }
    if att8 is not None:
        # BASELINE.json's metric names the LSTM-attn decoder: its temporal-
        # attention config (C = 8 frames, MFMA attention) on the same job
        rec['att8'] = att8
    if cst is not None:
        # the CST recipe (README CST_MS_SCB), fused consensus-baseline loss
        rec['cst'] = cst
    if xe is not None:
        rec['xe'] = xe
    if main_run.get('blaslt'):
        rec['blaslt_x_choice'] = main_run['blaslt']
    if main_run.get('beam5'):
        # BASELINE config 5: beam-5 evaluation decode (graph-replayed), whole job
        rec['beam5'] = main_run['beam5']
    if main_run['stamps']:
        rec['stamps_us'] = main_run['stamps']
    if main_run['phases']:
        rec['phases_ms'] = {k: round(v, 3) for k, v in main_run['phases'].items()}
    if ctx.is_main:
        line = json.dumps(rec)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, 'w') as f:
                f.write(line + '\n')
    ctx.destroy()


if __name__ == '__main__':
    main()
