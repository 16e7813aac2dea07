"""The reverse LSTM loop as ONE persistent launch (csrc/kernels/lstm_loop.hip:
the K-split team GEMM with exchanged partials, and the row-read form) against
the launch-per-step form (csrc/kernels/lstm.hip lstm_step_bwd_kernel)
on identical inputs: the same forward (fixed RNG words), the REINFORCE /
cross-entropy backward run once per form.  Both compute the same products
with fp32 accumulation in a different summation order, so the gradients agree
to fp32 / bf16-rounding noise.  Also: the device error word catches a team
wait that runs out of polls (forced with a zero poll bound), and the per-step
form's fused-attention flag wait likewise."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _model(R_videos, S, H, V, seed=0, num_chunks=1):
    from cst_captioning_amd.config import default_opts
    from cst_captioning_amd.data import make_synthetic, CaptionLoader
    from cst_captioning_amd.models import CaptionModel
    from cst_captioning_amd.models.decoder_engine import DecoderEngine
    ds = make_synthetic('msrvtt', num_videos=2 * R_videos, vocab_size=V, seq_length=30, seed=seed,
                        num_chunks=num_chunks)
    opt = default_opts(vocab_size=V, seq_length=30, feat_dims=ds.feat_dims, train_seq_per_img=S,
                       rnn_size=H, input_encoding_size=H, drop_prob_lm=0.5, num_chunks=num_chunks)
    torch.manual_seed(seed)
    model = CaptionModel(opt).to(DEV)
    eng = DecoderEngine(model, opt)
    loader = CaptionLoader(ds, R_videos, S, 'train', DEV, seed=seed)
    return model, eng, loader


def _grads(model, eng, data, mode, reward):
    from cst_captioning_amd.models import CrossEntropyCriterion, RewardCriterion
    model.zero_grad(set_to_none=True)
    torch.manual_seed(11)  # (FeatPool dropout draws from the torch generator)
    labels = data['labels']
    if mode == 'rl':
        seq, g_sel, _ = eng.rollout(model, data['feats'], labels)
        RewardCriterion()(seq, g_sel, reward).backward()
    else:
        g_xe = eng.teacher_forced(model, data['feats'], labels)
        CrossEntropyCriterion()(g_xe, labels[:, 1:], data['masks'][:, 1:]).backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()
            if p.grad is not None}


@pytest.mark.parametrize('form', [1, 2], ids=['rowread', 'ksplit'])
@pytest.mark.parametrize('videos,S,H,V,mode', [
    (64, 20, 512, 10509, 'rl'),    # headline: 256 workgroups, 40-row blocks
    (64, 20, 512, 10509, 'xe'),
    (16, 20, 256, 3000, 'rl'),     # 8 x 40 rows, 4 unit blocks
    (10, 13, 128, 1299, 'rl'),     # ragged groups: 130 rows -> 17-row groups
], ids=['headline_rl', 'headline_xe', 'h256', 'h128_ragged'])
def test_persistent_loop_matches_per_step_launches(videos, S, H, V, mode, form):
    from cst_captioning_amd import _ext
    ops = _ext.ops()
    model, eng, loader = _model(videos, S, H, V)
    eng._rng = lambda dev: torch.tensor([13579, 2468], dtype=torch.int32, device=DEV)
    model.train()
    model.set_seq_per_img(S)
    model.set_mixer_from(1)
    data = loader.get_batch()
    torch.manual_seed(3)
    reward = torch.randn(videos * S, device=DEV)
    ops.reset_device_errors(0)
    try:
        ops.set_bwd_loop(0)
        ref = _grads(model, eng, data, mode, reward)
        ops.set_bwd_loop(form)
        got = _grads(model, eng, data, mode, reward)
    finally:
        ops.set_bwd_loop(1)
    assert ops.device_errors(0) == 0
    assert set(got) == set(ref)
    errs = {n: ((got[n] - ref[n]).norm() / (ref[n].norm() + 1e-20)).item() for n in ref}
    bad = {n: e for n, e in errs.items() if not e < 5e-3}
    assert not bad, errs


def test_persistent_loop_poll_timeout_counts_device_error():
    """A zero poll bound makes every team wait give up at once: the kernel
    still ends (no hang) and the device error word counts the failed waits."""
    from cst_captioning_amd import _ext
    from cst_captioning_amd.models import RewardCriterion
    ops = _ext.ops()
    model, eng, loader = _model(10, 13, 128, 1299)
    model.train()
    model.set_seq_per_img(13)
    data = loader.get_batch()
    ops.reset_device_errors(0)
    ops.set_poll_bound(0)
    try:
        seq, g_sel, _ = eng.rollout(model, data['feats'], data['labels'])
        RewardCriterion()(seq, g_sel, torch.ones(130, device=DEV)).backward()
        torch.cuda.synchronize()
        n = ops.device_errors(0)
    finally:
        ops.set_poll_bound(1 << 20)
        ops.reset_device_errors(0)
    assert n > 0


def test_fused_attention_wait_timeout_counts_device_error():
    """The per-step reverse kernel's fused attention backward (att8 path):
    its GEMM workgroups' bounded wait for the attention workgroups' flags
    counts itself in the device error word when it gives up."""
    from cst_captioning_amd import _ext
    from cst_captioning_amd.models import RewardCriterion
    ops = _ext.ops()
    model, eng, loader = _model(8, 20, 128, 1299, num_chunks=8)
    model.train()
    model.set_seq_per_img(20)
    data = loader.get_batch()
    ops.reset_device_errors(0)
    seq, g_sel, _ = eng.rollout(model, data['feats'], data['labels'])
    RewardCriterion()(seq, g_sel, torch.ones(160, device=DEV)).backward()
    torch.cuda.synchronize()
    assert ops.device_errors(0) == 0  # normal bound: the waits succeed
    ops.set_poll_bound(0)
    try:
        seq, g_sel, _ = eng.rollout(model, data['feats'], data['labels'])
        RewardCriterion()(seq, g_sel, torch.ones(160, device=DEV)).backward()
        torch.cuda.synchronize()
        n = ops.device_errors(0)
    finally:
        ops.set_poll_bound(1 << 20)
        ops.reset_device_errors(0)
    assert n > 0
