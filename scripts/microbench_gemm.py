"""BLAS backend / layout sweep for the backward vocab-head GEMMs.

dHd = dS W  (NR x V) . (V x H)   and   dWlog = dS^T Hd  (V x NR) . (NR x H),
NR = 28 x 1280 rows, V = 10509, H = 512, bf16 operands (dS rows padded to
ldl), fp32 or bf16 output; per BLAS backend torch exposes on ROCm.
"""
import json
import time

import torch

dev = 'cuda'
NR, V, H = 28 * 1280, 10509, 512
ldl = (V + 7) // 8 * 8
dS = (torch.randn(NR, ldl, device=dev) * 1e-3).bfloat16()[:, :V]
W = torch.randn(V, H, device=dev).bfloat16()
hd = torch.randn(NR, H, device=dev).bfloat16()
WT = W.t().contiguous()


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
for lib in ('hipblaslt', 'rocblas', 'default'):
    try:
        if lib != 'default':
            torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:  # backend not available
        res[lib] = str(e)[:60]
        continue
    res[lib + '_dHd_f32'] = bench(lambda: torch.mm(dS, W, out_dtype=torch.float32))
    res[lib + '_dHd_bf16'] = bench(lambda: torch.mm(dS, W))
    res[lib + '_dHd_WT_f32'] = bench(lambda: torch.mm(dS, WT.t(), out_dtype=torch.float32))
    res[lib + '_dW_f32'] = bench(lambda: torch.mm(dS.t(), hd, out_dtype=torch.float32))
    res[lib + '_dW_bf16'] = bench(lambda: torch.mm(dS.t(), hd))
    res[lib + '_dWT_f32'] = bench(lambda: torch.mm(hd.t(), dS, out_dtype=torch.float32))
res['tflops_per_ms'] = round(2 * NR * V * H / 1e9, 1)
print(json.dumps(res))
