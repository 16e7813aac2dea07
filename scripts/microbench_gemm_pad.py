"""Vocab-head backward GEMMs with the vocabulary dimension padded.

dHd = A W (NR x Vp) . (Vp x H) and dW = A^T Hd (Vp x NR) . (NR x N) with
Vp = V (ragged K / M tail) or V rounded up to 64 / 128 / 256, A bf16 with
row stride max(10560, Vp); N = H or H + extra columns (the bias-gradient
column of the exp-store backward); fp32 output, hipBLASLt.  Every shape is
timed twice, in two passes, so clock ramp-up does not favour later shapes.
"""
import json
import time

import torch

dev = 'cuda'
NR, V, H = 28 * 1280, 10509, 512


def bench(f, n=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e3, 3)


res = {}
for rep in range(2):
    for Vp in (V, 10624, 10752):
        ldl = max(10560, Vp)
        buf = (torch.randn(NR, ldl, device=dev) * 1e-3).bfloat16()
        A = buf[:, :Vp]
        W = torch.randn(Vp, H, device=dev).bfloat16()
        o1 = torch.empty(NR, H, device=dev)
        res['dHd_%d_r%d' % (Vp, rep)] = bench(lambda: torch.mm(A, W, out_dtype=torch.float32, out=o1))
        for N in ((512, 528, 576, 640) if Vp == 10752 else (512,)):
            hd = torch.randn(NR, N, device=dev).bfloat16()
            o2 = torch.empty(Vp, N, device=dev)
            res['dW_%d_N%d_r%d' % (Vp, N, rep)] = bench(
                lambda: torch.mm(A.t(), hd, out_dtype=torch.float32, out=o2))
            del hd, o2
        del buf, A, W, o1
res['gflop_per_gemm'] = round(2 * NR * V * H / 1e9, 1)
print(json.dumps(res))
