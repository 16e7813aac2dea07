"""Fused dS + dHd backward kernel (vocab_bwd.hip) alone, with ablations.

Headline shape: 28 steps x 1280 rows, V = 10,509, H = 512.  Prints us per
launch for the full kernel, each ablation bit (1 no A loads, 2 no dS store,
4 no MFMA, 8 no B DMA, 16 no transform, 32 no column sums, 64 no dHd store) and the two-pass route for reference.
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
n, R, V, H = 28, 1280, 10509, 512
ldl = (V + 63) // 64 * 64
ldw = (V + 31) // 32 * 32
logits = (torch.randn(n, R, ldl, device=dev) * 2).half()
lse = torch.logsumexp(logits[..., :V].float(), -1).reshape(-1).contiguous()
seq = torch.randint(0, V, (R, n), device=dev)
dg = torch.randn(R, n, device=dev)
wT = torch.zeros(H, ldw, device=dev, dtype=torch.bfloat16)
wT[:, :V] = (torch.randn(H, V, device=dev) * 0.05).bfloat16()
res = {}
for split in (1, 2, 4):
    res['split%d' % split] = round(C.vocab_bwd_dhd_bench(logits, lse, seq, dg, wT, V, split, 0, 20), 1)
for dbg in (1, 2, 4, 8, 16, 32, 64, 1 | 2, 4 | 8, 1 | 2 | 4 | 8 | 16, 31 | 32, 31 | 64, 127, 32 | 64):
    res['split2_dbg%d' % dbg] = round(C.vocab_bwd_dhd_bench(logits, lse, seq, dg, wT, V, 2, dbg, 20), 1)
res['two_pass_ds'] = round(C.vocab_bwd_ds_bench(logits, lse, seq, dg, 20), 1)
print(json.dumps(res))
