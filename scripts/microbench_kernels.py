"""Single-kernel microbenchmarks (HIP-event timed, back-to-back launches).

vocab_fwd at the rollout shape (R = 1280 rows) and the greedy shape (R = 64),
with the epilogue pieces switched on one at a time:
  mainloop = GEMM only; stats = max/LSE (+target); sample; sample+save
  (fp16 logits for the backward); argmax.  Also: token sort, per-token
gate-gradient sums (TGS=1), bias column sums (CS=1), attention (ATT=1).
VARIANTS="0 1 2 ..." times other <BN, STAGES, OCC> shapes of the vocab kernel
(launch_vocab_fwd_variant in csrc/kernels/vocab.hip).
"""
import json
import os

import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cst_captioning_amd import _ext

C = _ext.ops()
torch.manual_seed(0)
dev = 'cuda'
V, H = 10509, 512
W = (torch.randn(V, H, device=dev) * 0.05).bfloat16()
b = torch.randn(V, device=dev) * 0.1
res = {}
variants = [int(v) for v in os.environ.get('VARIANTS', '0').split()]
for R in (1280, 64):
    hd = torch.randn(R, H, device=dev).bfloat16()
    tgt = torch.randint(0, V, (R,), device=dev)
    none = torch.empty(0, dtype=torch.long, device=dev)
    for var in variants:
        for name, flags, save, t in (('mainloop', 4, False, None), ('stats', 0, False, tgt),
                                     ('sample', 1, False, None), ('sample_save', 1, True, None),
                                     ('argmax', 2, False, None)):
            us = C.vocab_fwd_bench(hd, W, b, t if t is not None else none, flags, save, 50, var)
            res['v%d_R%d_%s' % (var, R, name)] = round(us, 2)
toks = torch.randint(0, V, (28 * 1280,), device=dev)
res['token_sort_us'] = round(C.token_sort_bench(toks, V, 50), 2)
if os.environ.get('TGS', '1') == '1':  # per-token gate-gradient sums, alone on the GPU
    x = torch.randn(28 * 1280, 4 * H, device=dev).bfloat16()
    tk = toks.clone()
    tk[:1280] = 0  # step 0: every row's input is BOS (one long group)
    for _ in range(3):
        C.token_group_sum(x, tk, V)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(20):
        C.token_group_sum(x, tk, V)
    ev1.record()
    torch.cuda.synchronize()
    us = ev0.elapsed_time(ev1) * 1e3 / 20
    res['token_group_sum_op_us'] = round(us, 1)  # sort + sums + finalize
    res['token_group_sum_read_TBps'] = round(x.numel() * 2 / us / 1e6, 2)
if os.environ.get('CS', '1') == '1':  # bias-gradient column sums over the exp store
    n, R = 28, 1280
    ldl = (V + 63) // 64 * 64
    E = torch.rand(n, R, ldl, device=dev).bfloat16()
    alpha = torch.randn(n * R, device=dev) * 1e-3
    us = C.vgrad_colsum_bench(E, alpha, V, 10)
    res['colsum_T28_R1280_us'] = round(us, 1)
    res['colsum_TBps'] = round(n * R * V * 2 / us / 1e6, 2)
if os.environ.get('ATT', '1') == '1':  # temporal attention kernels, 8 frames
    Bv, Cf, A = 64, 8, H
    gv = torch.randn(Bv, Cf, 4 * H, device=dev) * 0.1
    P = torch.randn(Bv, Cf, A, device=dev) * 0.5
    wa = torch.randn(A, device=dev) * 0.1
    ba = torch.zeros(1, device=dev)
    for R in (1280, 64):
        q = torch.randn(R, A, device=dev) * 0.5
        res['att_fwd_R%d_us' % R] = round(C.att_bench(gv, P, q, wa, ba, R, 0, 50), 2)
        res['att_fwd_rpw2_R%d_us' % R] = round(C.att_bench(gv, P, q, wa, ba, R, 2, 50), 2)
        res['att_fwd_rpw1_R%d_us' % R] = round(C.att_bench(gv, P, q, wa, ba, R, 3, 50), 2)
        res['att_bwd_R%d_us' % R] = round(C.att_bench(gv, P, q, wa, ba, R, 1, 50), 2)
        res['att_bwd_rpw2_R%d_us' % R] = round(C.att_bench(gv, P, q, wa, ba, R, 4, 50), 2)
print(json.dumps(res))
