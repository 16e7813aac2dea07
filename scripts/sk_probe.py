"""X = E W (35,840 x 512, K = 10,560 padded) and dW = E^T Hs at the headline shape: the
hand-written persistent GEMM (csrc/kernels/gemm_sk.hip, variants 0 / 1) vs
PyTorch's hipBLASLt default and the measured-choice hipBLASLt plan
(csrc/host/blaslt_tuned.cpp).  Prints one JSON line (us per call, TFLOP/s,
relative error vs the default)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cst_captioning_amd import _ext  # noqa: E402

ops = _ext.ops()
dev = 'cuda'
NR, V, H, LDL = 28 * 1280, 10509, 512, 10560
torch.manual_seed(0)
E = torch.zeros(NR, LDL, device=dev, dtype=torch.bfloat16)
E[:, :V] = (torch.rand(NR, V, device=dev) * 1e-3).bfloat16()
W = (torch.randn(V, H, device=dev) * 0.05).bfloat16()
Ev = E[:, :V]
WT = ops.transpose_pad_bf16(W, LDL)


def bench(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e6, 1)


flop = 2.0 * NR * H * V
out = {}
X0 = torch.empty(NR, H, device=dev)
out['x_default_us'] = bench(lambda: torch.mm(Ev, W, out_dtype=torch.float32, out=X0))
X1 = torch.empty(NR, H, device=dev)
out['x_tuned_us'] = bench(lambda: ops.gemm_bf16_tuned(X1, Ev, False, W, False, 32))
out['transpose_us'] = bench(lambda: ops.transpose_pad_bf16(W, LDL))
for v in (0, 1):
    X2 = torch.empty(NR, H, device=dev)
    us = bench(lambda: ops.gemm_nt_sk(X2, E, WT, v))
    out['x_sk%d_us' % v] = us
    out['x_sk%d_tflops' % v] = round(flop / us * 1e-6, 1)
    out['x_sk%d_rel_err' % v] = float((X2 - X0).norm() / X0.norm())
out['x_default_tflops'] = round(flop / out['x_default_us'] * 1e-6, 1)
# dW = E^T Hs (10,509 x 512, K = 35,840): the TN path
Hs = (torch.randn(NR, H, device=dev) * 0.1).bfloat16()
D0 = torch.empty(V, H, device=dev)


def dw_split():
    kr = NR // 4
    a = E.as_strided((4, V, kr), (kr * LDL, 1, LDL))
    torch.sum(torch.bmm(a, Hs.view(4, kr, H), out_dtype=torch.float32), 0, out=D0)


out['dw_default_splitk4_us'] = bench(dw_split)
D1 = torch.empty(V, H, device=dev)
out['dw_tuned_us'] = bench(lambda: ops.gemm_bf16_tuned(D1, Ev, True, Hs, False, 32))
for v in (0, 1):
    D2 = torch.empty(V, H, device=dev)
    us = bench(lambda: ops.gemm_tn_sk(D2, Ev, Hs, v))
    out['dw_sk%d_us' % v] = us
    out['dw_sk%d_tflops' % v] = round(flop / us * 1e-6, 1)
    out['dw_sk%d_rel_err' % v] = float((D2 - D0).norm() / D0.norm())
out['x_tuned_tflops'] = round(flop / out['x_tuned_us'] * 1e-6, 1)
print(json.dumps(out))
