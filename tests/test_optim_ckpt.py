"""Optimizer NaN guard and checkpoint-format edge cases (CPU).

* FlatAdam skips an update whose gradient norm is not finite even when the
  loss is finite (an overflowing gradient), keeps the step count, and counts
  the skip (reference: no guard at all, /root/reference/train.py:216-218;
  SURVEY.md 5.3).
* A reference-shaped best-model checkpoint -- ``infos`` holding numpy float64
  scores after ``infos.update(scores)``, ``opt`` an ``argparse.Namespace``
  (/root/reference/train.py:403-407) -- loads with ``weights_only=True``.
"""
import argparse

import numpy as np
import pytest
import torch

from cst_captioning_amd.ops.adam import FlatAdam
from cst_captioning_amd.parallel import FlatGradBucket
from cst_captioning_amd.train import checkpoint as ckpt


def _opt(n=37, **kw):
    p = torch.nn.Parameter(torch.randn(n))
    q = torch.nn.Parameter(torch.randn(5, 3))
    b = FlatGradBucket([p, q])
    return b, FlatAdam(b, lr=1e-2, **kw)


def test_adam_skips_nonfinite_gradient_norm():
    b, opt = _opt()
    b.grad[:b.numel].normal_()
    opt.step()
    assert opt.step_count == 1
    p0, m0, v0 = b.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone()
    b.grad[3] = float('inf')  # finite loss, overflowing gradient
    opt.step()
    torch.testing.assert_close(b.data, p0, rtol=0, atol=0)
    torch.testing.assert_close(opt.exp_avg, m0, rtol=0, atol=0)
    torch.testing.assert_close(opt.exp_avg_sq, v0, rtol=0, atol=0)
    assert opt.step_count == 1 and int(opt.skipped()) == 1
    # the loss flag skips too, and a healthy step then resumes the count
    b.grad[3] = 0.5
    opt.step(torch.tensor(True))
    assert opt.step_count == 1 and int(opt.skipped()) == 2
    opt.step(torch.tensor(False))
    assert opt.step_count == 2 and int(opt.skipped()) == 2
    assert not torch.equal(b.data, p0)


def test_adam_grad_scale_equals_divided_buffer():
    """DP: the fp32 all-reduce sums over N ranks and the optimizer applies
    1/N (grad_scale) -- identical to dividing the buffer first."""
    torch.manual_seed(0)
    b1, o1 = _opt(grad_clip=0.25)
    torch.manual_seed(0)
    b2, o2 = _opt(grad_clip=0.25)
    for _ in range(3):
        g = torch.randn(b1.numel) * 3
        b1.grad[:b1.numel] = g * 4
        o1.grad_scale = 0.25
        b2.grad[:b2.numel] = g
        o1.step()
        o2.step()
    torch.testing.assert_close(b1.data, b2.data, rtol=1e-6, atol=1e-7)


def test_adam_state_roundtrip_keeps_counters():
    b, opt = _opt()
    b.grad[:b.numel].normal_()
    opt.step()
    b.grad[0] = float('nan')
    opt.step()
    s = opt.state_dict()
    assert s['step'] == 1 and s['skipped'] == 1
    b2, opt2 = _opt()
    opt2.load_state_dict(s)
    assert opt2.step_count == 1 and int(opt2.skipped()) == 1


def test_reference_shaped_checkpoint_with_numpy_scores(tmp_path):
    """The reference's best checkpoint pickles numpy float64 metric values in
    ``infos`` (coco-caption scores) next to a Namespace ``opt``."""
    path = str(tmp_path / 'ref.pth')
    sd = {'embed.weight': torch.randn(4, 3), 'logit.bias': torch.zeros(4)}
    infos = {'iter': 10, 'epoch': 2, 'best_score': np.float64(0.4321),
             'CIDEr': np.float64(0.4321), 'ROUGE_L': np.float64(0.5),
             'Bleu_4': np.float32(0.25), 'best_iter': np.int64(10), 'TrainLoss': 2.5}
    opt = argparse.Namespace(model_type='concat', vocab={0: '<end>'}, vocab_size=4,
                             seq_length=30, feat_dims=[2048], rnn_size=512)
    torch.save({'model': sd, 'infos': infos, 'opt': opt}, path)  # as train.py:403-407
    s = ckpt.load_checkpoint(path)
    assert s['opt'].model_type == 'concat' and s['opt'].feat_dims == [2048]
    assert s['infos']['CIDEr'] == pytest.approx(0.4321)
    assert type(s['infos']['CIDEr']) is float and type(s['infos']['best_iter']) is int
    torch.testing.assert_close(s['model']['embed.weight'], sd['embed.weight'])


def test_encode_tolerates_tuples_of_arrays(tmp_path):
    """A 5-tuple whose first element is an array (not the numpy RNG state)
    must not be mistaken for one."""
    arrs = tuple(np.arange(3) + i for i in range(5))
    obj = {'a': arrs, 'rng': np.random.get_state(), 't': (torch.ones(2),) * 5}
    path = str(tmp_path / 'x.pth')
    torch.save(ckpt._encode(obj), path)
    back = ckpt.load_checkpoint(path)
    for x, y in zip(back['a'], arrs):
        np.testing.assert_array_equal(x, y)
    assert back['rng'][0] == 'MT19937'
    np.testing.assert_array_equal(back['rng'][1], obj['rng'][1])
