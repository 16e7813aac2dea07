"""CIDEr-D kernel microbenchmark at the bench's shapes (synthetic MSR-VTT,
6,513 videos x 20 captions, V = 10,509): HIP-event time per launch for N
hypotheses of random tokens (a random-init rollout: no early EOS, W ~ 28)
and of ground-truth captions (short), N = 64 (greedy) ... 2,560.
Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cst_captioning_amd.data import make_synthetic
from cst_captioning_amd.ops.cider_d import CiderDScorer


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device('cuda')
    ds = make_synthetic('msrvtt', num_videos=6513, vocab_size=10509, seed=123)
    sc = CiderDScorer(ds, use_eos=1, device=dev)
    g = torch.Generator(device='cpu').manual_seed(0)
    res = {}
    labels = torch.from_numpy(ds.labels).long()
    for N in (64, 320, 1280, 2560):
        vid = torch.randint(0, 6513, (N,), generator=g).to(dev)
        rnd = torch.randint(3, 10509, (N, 30), generator=g).to(dev)
        rnd[:, 29] = 0
        res['random_N%d_us' % N] = round(timed(lambda: sc.score(rnd, vid)), 1)
        st = torch.from_numpy(ds.label_start_ix[vid.cpu().numpy()]).long()
        gt = labels[st].to(dev)[:, :30].contiguous()
        res['gt_N%d_us' % N] = round(timed(lambda: sc.score(gt, vid)), 1)
    # oracle check on a few rows
    vid = torch.randint(0, 6513, (16,), generator=g).to(dev)
    rnd = torch.randint(3, 200, (16, 30), generator=g).to(dev)
    got = sc.score(rnd, vid).cpu().double()
    ref = torch.from_numpy(sc.score_reference(rnd, vid))
    res['max_abs_err_vs_oracle'] = float((got - ref).abs().max())
    print(json.dumps(res))


if __name__ == '__main__':
    main()
