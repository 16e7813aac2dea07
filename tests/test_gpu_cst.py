"""The CST recipe (the reference's namesake, ``/root/reference/utils.py:229-324``,
``train.py:182-194``, README "CST_MS_SCB" / "CST_MS_SCB(*)") on the fused
path: the consensus baseline, reward, mask and REINFORCE loss in one launch
(``csrc/kernels/loss.hip`` CST mode, ``ops/scst_loss.py:cst_loss``), checked
against ``cst_from_scores`` + ``RewardCriterion`` in fp32, and inside the
replayed HIP-graph training step."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.mark.parametrize('scb_baseline,scb_captions', [(1, 20), (2, 20), (1, 5), (2, 7), (2, 0)])
def test_fused_cst_loss_matches_torch(scb_baseline, scb_captions):
    """Loss, reward, logged means and the log-prob gradient of the fused CST
    loss against the reference arithmetic in fp32 (ties included: scores are
    drawn from a coarse grid so the k-lowest selection meets equal values)."""
    from cst_captioning_amd.models import RewardCriterion
    from cst_captioning_amd.ops.scst_loss import cst_loss
    from cst_captioning_amd.reward.rewards import cst_from_scores
    torch.manual_seed(scb_captions + 10 * scb_baseline)
    B, S, T = 64, 20, 28
    R = B * S
    seq = torch.randint(0, 50, (R, T), device=DEV)
    seq[torch.rand(R, T, device=DEV) < 0.1] = 0
    lp = (-torch.rand(R, T, device=DEV) * 5).requires_grad_(True)
    scores = torch.randint(0, 12, (B, S), device=DEV).float() / 8.0
    bcmr = torch.randint(0, 12, (B, S), device=DEV).float() / 7.0
    loss, reward, m, b = cst_loss(seq, lp, scores, bcmr, scb_captions, scb_baseline)
    rref, mref, bref = cst_from_scores(scores, bcmr, scb_captions, scb_baseline)
    lp2 = lp.detach().clone().requires_grad_(True)
    ref = RewardCriterion()(seq, lp2, rref)
    torch.testing.assert_close(reward, rref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m, torch.as_tensor(mref, device=DEV).float(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(b, torch.as_tensor(bref, device=DEV).float(), rtol=1e-6, atol=1e-6)
    (2.0 * loss).backward()
    (2.0 * ref).backward()
    torch.testing.assert_close(lp.grad, lp2.grad, rtol=1e-5, atol=1e-8)


def _setup(scb_baseline, graph, seed=0, V=500, H=128):
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.cli import build_model
    from cst_captioning_amd.parallel import DistContext
    from cst_captioning_amd.train.trainer import Trainer
    S = 5
    ds = make_synthetic('msrvtt', num_videos=48, vocab_size=V, seq_length=12,
                        feat_dims=[64, 32], seed=seed, with_consensus=True, consensus_cols=S)
    opt = default_opts(vocab_size=V, seq_length=12, feat_dims=[64, 32], train_seq_per_img=S,
                       batch_size=8, rnn_size=H, input_encoding_size=H, drop_prob_lm=0.5,
                       use_rl=1, use_rl_after=0, use_cst=1, use_mixer=1, mixer_from=1,
                       scb_baseline=scb_baseline, scb_captions=S, use_eos=1, impl='hip',
                       cuda_graph=graph, learning_rate=1e-3)
    opt.vocab = {i: w for i, w in enumerate(ds.vocab)}
    torch.manual_seed(seed)
    dev = torch.device(DEV)
    model, engine = build_model(opt, dev, 'hip')
    assert engine is not None
    loader = CaptionLoader(ds, 8, S, 'train', dev, seed=seed)
    tr = Trainer(opt, model, loader, None, DistContext(device=dev), engine)
    tr.rl_training = True
    return tr, loader


@pytest.mark.parametrize('scb_baseline', [1, 2])
def test_cst_step_fused_and_graphed(scb_baseline):
    """CST_MS_SCB (GT consensus baseline) and CST_MS_SCB(*) (baseline from the
    samples' own scores) through the trainer: (a) the eager fused step's
    reward equals cst_from_scores of the on-GPU CIDEr-D scores of the tokens
    it sampled; (b) the captured, replayed step gives the eager step's
    samples, rewards, loss and logged means with the seeds pinned, and the
    same weights after 4 updates."""
    from cst_captioning_amd.ops import featpool as fp
    from cst_captioning_amd.reward.rewards import cst_from_scores
    fixed = torch.tensor([2468, 1357], dtype=torch.int32, device=DEV)
    a, la = _setup(scb_baseline, graph=0)
    b, lb = _setup(scb_baseline, graph=1)
    for tr in (a, b):
        tr.engine._rng = lambda dev: fixed
    old = fp.SEED_SOURCE
    fp.SEED_SOURCE = lambda dev: fixed
    try:
        for it in range(4):
            da, db = la.get_batch(), lb.get_batch()
            oa = a.train_step(da, 0)
            ob = b.train_step(db, 0)
            torch.cuda.synchronize()
            if it == 0:  # (a) the fused reward against the reference arithmetic
                S = 5
                scorer = a._ensure_scorer()
                vid = da['video_index'].repeat_interleave(S)
                sc = scorer.score(oa['seq'], vid).float().view(-1, S)
                bc = da['bcmrscores'].float() if scb_baseline == 1 else None
                rref, mref, bref = cst_from_scores(sc, bc, S, scb_baseline)
                torch.testing.assert_close(oa['reward'], rref, rtol=1e-5, atol=1e-6)
                torch.testing.assert_close(torch.as_tensor(oa['b']).float(),
                                           torch.as_tensor(bref).float(), rtol=1e-5, atol=1e-6)
            assert torch.equal(oa['seq'], ob['seq'])
            torch.testing.assert_close(oa['reward'], ob['reward'], rtol=1e-5, atol=1e-6)
            for k in ('loss', 'm', 'b'):
                torch.testing.assert_close(torch.as_tensor(oa[k]).float(),
                                           torch.as_tensor(ob[k]).float(), rtol=1e-5, atol=1e-6)
    finally:
        fp.SEED_SOURCE = old
    assert b._graph is not None and a._graph is None
    pa = torch.cat([p.detach().reshape(-1) for p in a.model.parameters()])
    pb = torch.cat([p.detach().reshape(-1) for p in b.model.parameters()])
    assert ((pa - pb).norm() / pa.norm()).item() < 1e-4
