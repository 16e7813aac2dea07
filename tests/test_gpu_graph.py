"""The HIP-graph training step and the pieces that make its replay correct
(``Trainer._graph_step``): device-side RNG seeds, device-side Adam lr/step,
bf16 weight shadows written by the Adam pass, and the counting sort of the
backward's input tokens."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _setup(rl, seed=0, V=500, H=128, drop=0.0, graph=1):
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.cli import build_model
    from cst_captioning_amd.parallel import DistContext
    from cst_captioning_amd.train.trainer import Trainer
    ds = make_synthetic('msrvtt', num_videos=48, vocab_size=V, seq_length=12,
                        feat_dims=[64, 32], seed=seed)
    opt = default_opts(vocab_size=V, seq_length=12, feat_dims=[64, 32], train_seq_per_img=5,
                       batch_size=8, rnn_size=H, input_encoding_size=H, drop_prob_lm=drop,
                       use_rl=int(rl), use_rl_after=0, use_cst=0, use_mixer=1, mixer_from=1,
                       use_eos=1, impl='hip', cuda_graph=graph, learning_rate=1e-3)
    opt.vocab = {i: w for i, w in enumerate(ds.vocab)}
    torch.manual_seed(seed)
    dev = torch.device(DEV)
    model, engine = build_model(opt, dev, 'hip')
    assert engine is not None
    loader = CaptionLoader(ds, 8, 5, 'train', dev, seed=seed)
    tr = Trainer(opt, model, loader, None, DistContext(device=dev), engine)
    tr.rl_training = bool(rl)
    return tr, loader


def _flat(model):
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


def test_graph_xe_steps_match_eager():
    """XE without dropout is deterministic up to summation order: 6 steps
    through the captured graph equal 6 eager steps on the same batches."""
    a, la = _setup(rl=False, graph=0)
    b, lb = _setup(rl=False, graph=1)
    torch.testing.assert_close(_flat(a.model), _flat(b.model), rtol=0, atol=0)
    for _ in range(6):
        da, db = la.get_batch(), lb.get_batch()
        oa = a.train_step(da, 0)
        ob = b.train_step(db, 0)
        torch.testing.assert_close(float(oa['loss']), float(ob['loss']), rtol=1e-4, atol=1e-5)
    assert b._graph is not None, 'the graph path was never captured'
    pa, pb = _flat(a.model), _flat(b.model)
    assert ((pa - pb).norm() / pa.norm()).item() < 1e-4
    # the optimizer's device step counter advanced on every replay
    assert b.optimizer.state_dict()['step'] == 6


@pytest.mark.parametrize('H', [128, 512])
def test_graph_scst_step_matches_eager_with_fixed_seeds(H):
    """The step that ships -- one captured HIP graph: FeatPool + video gate,
    MIXER rollout, the greedy baseline decoded concurrently on a side stream,
    on-GPU CIDEr-D of both, the fused SCST reward / mask / REINFORCE loss,
    the backward, clip + Adam + bf16 weight shadows -- against the same step
    enqueued eagerly (reference step: /root/reference/train.py:167-218), with
    dropout 0.5 and the dropout / sampling seeds pinned on the device: the
    same sampled tokens, rewards and loss every step, and the same weights
    after 5 updates."""
    from cst_captioning_amd.ops import featpool as fp
    fixed = torch.tensor([12345, 67890], dtype=torch.int32, device=DEV)
    a, la = _setup(rl=True, drop=0.5, graph=0, H=H)
    b, lb = _setup(rl=True, drop=0.5, graph=1, H=H)
    torch.testing.assert_close(_flat(a.model), _flat(b.model), rtol=0, atol=0)
    for tr in (a, b):
        tr.engine._rng = lambda dev: fixed
    old = fp.SEED_SOURCE
    fp.SEED_SOURCE = lambda dev: fixed
    try:
        for _ in range(5):
            oa = a.train_step(la.get_batch(), 0)
            ob = b.train_step(lb.get_batch(), 0)
            torch.cuda.synchronize()
            assert torch.equal(oa['seq'], ob['seq'])
            torch.testing.assert_close(oa['reward'], ob['reward'], rtol=1e-5, atol=1e-6)
            for k in ('loss', 'm', 'b'):
                torch.testing.assert_close(torch.as_tensor(oa[k]).float(),
                                           torch.as_tensor(ob[k]).float(), rtol=1e-5, atol=1e-6)
    finally:
        fp.SEED_SOURCE = old
    assert b._graph is not None and a._graph is None
    pa, pb = _flat(a.model), _flat(b.model)
    assert ((pa - pb).norm() / pa.norm()).item() < 1e-4
    assert a.optimizer.step_count == b.optimizer.step_count == 5


@pytest.mark.parametrize('H', [128, 512])
def test_x_after_rollout_matches_folded_path(H):
    """X = E W launched after the rollout on the engine's stream
    (engine.launch_x; the loop adds alpha X + the one-hot rows) against the
    backward's own E' W GEMM (one-hot terms folded into E): same seeds, same
    batch, one eager step and one captured step each: identical rollouts and
    rewards, updates equal within the bf16 rounding of the fold (later steps
    may flip near-tied greedy tokens, so only the first update of each mode
    is compared)."""
    from cst_captioning_amd.ops import featpool as fp
    fixed = torch.tensor([4242, 777], dtype=torch.int32, device=DEV)
    old = fp.SEED_SOURCE
    fp.SEED_SOURCE = lambda dev: fixed
    try:
        for graph in (0, 1):
            runs = []
            for x_after in (True, False):
                tr, ld = _setup(rl=True, drop=0.5, graph=graph, H=H)
                tr.engine._rng = lambda dev: fixed
                if graph:  # eager warm-up step of the key (same path), then the capture
                    tr.use_x_after_rollout = False
                    tr.train_step(ld.get_batch(), 0)
                tr.use_x_after_rollout = x_after
                p0 = _flat(tr.model)
                out = tr.train_step(ld.get_batch(), 0)
                torch.cuda.synchronize()
                assert (tr._graph is not None) == bool(graph)
                runs.append((out['seq'].clone(), out['reward'].clone(), p0, _flat(tr.model)))
            (sa, ra, p0a, pa), (sb, rb, p0b, pb) = runs
            assert torch.equal(sa, sb)
            torch.testing.assert_close(ra, rb, rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(p0a, p0b, rtol=0, atol=0)
            da, db = pa - p0a, pb - p0b
            err = ((da - db).norm() / db.norm()).item()
            assert err < 2e-2, (graph, err)
    finally:
        fp.SEED_SOURCE = old


def test_graph_replays_draw_fresh_samples():
    """The same batch replayed twice gives different rollouts (seeds are
    drawn on the device inside the graph), and the weights keep training."""
    tr, loader = _setup(rl=True, drop=0.5)
    seqs = []
    for _ in range(4):
        before = _flat(tr.model).clone()
        out = tr.train_step(loader.get_batch_at(0), 0)  # the same videos every step
        torch.cuda.synchronize()
        assert torch.isfinite(out['loss']).item()
        assert not torch.equal(before, _flat(tr.model))
        seqs.append(out['seq'].clone() if tr._graph is not None else None)
    assert tr._graph is not None
    assert seqs[-1] is not None and seqs[-2] is not None
    assert not torch.equal(seqs[-1], seqs[-2])


def test_adam_pass_writes_the_bf16_shadows():
    """After training steps the engine's shadow buffers (written by the fused
    Adam pass) equal a from-scratch refresh of the fp32 parameters."""
    tr, loader = _setup(rl=True, drop=0.5)
    for _ in range(4):
        tr.train_step(loader.get_batch(), 0)
    eng = tr.engine
    got = [t.clone() for t in (eng.wx, eng.whh_q, eng.emb, eng.wlog, eng.current_ptab())]
    assert eng.wiv is not None  # concat model: W_ih's video columns, packed
    wiv = eng.wiv.clone()
    eng.refresh_weights()
    for g, r in zip(got, (eng.wx, eng.whh_q, eng.emb, eng.wlog)):
        assert torch.equal(g, r)
    assert torch.equal(wiv, eng.wiv)
    torch.testing.assert_close(got[4], eng.ptab, rtol=1e-5, atol=1e-5)


def test_gate_table_tracks_replayed_updates():
    """The gate table P = emb W_ie^T is refreshed lazily (decoder_engine.py
    prefetch_ptab / ensure_ptab).  An eval between replays refreshes it; the
    replays after it change the weights on the device only, so the next
    user must see P stale again (a replay did not bump the
    version).  And a graph captured while P is marked fresh must still hold
    its refresh: every replay then trains with the current P."""
    tr, loader = _setup(rl=True, drop=0.5)
    eng = tr.engine
    for _ in range(3):  # eager warm-up, capture + replay
        tr.train_step(loader.get_batch(), 0)
    eng.current_ptab()  # an eval: P marked fresh
    for _ in range(2):
        tr.train_step(loader.get_batch(), 0)
    got = eng.current_ptab().clone()
    eng.refresh_weights()
    torch.testing.assert_close(got, eng.ptab, rtol=1e-5, atol=1e-5)
    # recapture while P is fresh (a new schedule key after an eval)
    tr._graph_key = None
    tr._graph_warm = {k: 1 for k in tr._graph_warm}
    eng.current_ptab()
    before = eng.ptab.clone()
    tr.train_step(loader.get_batch(), 0)  # capture + replay
    tr.train_step(loader.get_batch(), 0)  # replay: trains with the refreshed P
    torch.cuda.synchronize()
    assert not torch.equal(before, eng.ptab), 'the captured step never refreshed P'
    got = eng.current_ptab().clone()
    eng.refresh_weights()
    torch.testing.assert_close(got, eng.ptab, rtol=1e-5, atol=1e-5)


def test_token_counting_sort():
    from cst_captioning_amd import _ext
    V = 10509
    toks = torch.randint(0, V, (28 * 1280,), device=DEV)
    toks[:5000] = 0  # a heavy bucket (EOS)
    stok, srow = _ext.ops().token_sort(toks, V)
    st, sr = stok.cpu().numpy(), srow.cpu().numpy()
    t = toks.cpu().numpy()
    assert (np.diff(st) >= 0).all()                  # grouped by token
    assert np.array_equal(np.sort(sr), np.arange(t.size))  # a permutation of the rows
    assert np.array_equal(t[sr], st)                 # each row under its own token


@pytest.mark.parametrize('C', [2048, 4096])
def test_token_group_sums(C):
    """Per-token row sums (embedding / input-weight gradient operand): short
    groups summed by their owning block, long groups (the BOS / EOS buckets,
    groups of 200-300 entries around the 192-entry split) through the fp32
    scratch, and tokens without rows zero-filled -- against an fp32
    index_add."""
    from cst_captioning_amd import _ext
    V, N = 10509, 28 * 1280
    g = torch.Generator(device='cpu').manual_seed(3)
    toks = torch.randint(1, V - 50, (N,), generator=g)
    toks[:1280] = 0                     # step 0: BOS for every row
    toks[5000:5250] = 7                 # long groups just above / below the split
    toks[9000:9193] = 8
    toks[12000:12192] = 9
    toks = toks[torch.randperm(N, generator=g)].to(DEV)
    x = torch.randn(N, C, generator=g).to(DEV, torch.bfloat16)
    S = _ext.ops().token_group_sum(x, toks, V)
    ref = torch.zeros(V, C, device=DEV).index_add_(0, toks, x.float())
    assert S.dtype == torch.bfloat16 and S.shape == (V, C)
    assert torch.all(S[V - 50:] == 0)   # tokens without rows
    err = (S.float() - ref).norm() / ref.norm()
    assert err < 4e-3, err


def test_lr_change_reaches_the_graph():
    """An LR decay between replays (adjust_learning_rate) takes effect
    without a re-capture: with lr = 0 the weights stop moving."""
    tr, loader = _setup(rl=False)
    for _ in range(3):
        tr.train_step(loader.get_batch(), 0)
    assert tr._graph is not None
    tr.optimizer.param_groups[0]['lr'] = 0.0
    before = _flat(tr.model).clone()
    tr.train_step(loader.get_batch(), 0)
    torch.testing.assert_close(_flat(tr.model), before, rtol=0, atol=0)
