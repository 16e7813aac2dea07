"""hipBLASLt algorithm search for the vocab head's backward GEMMs at the
headline shape: X = E W (35,840 x 512, K = 10,509) and dW = E^T Hs (10,509 x
512, K = 35,840), bf16 operands, fp32 out.  Times PyTorch's default choice
(at::mm / the 4-way split-K bmm the engine ships) and every candidate of the
measured choice (csrc/host/blaslt_tuned.cpp); checks the result against the
default's.  Prints one JSON line."""
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
E = (torch.rand(NR, LDL, device=dev) * 1e-3).bfloat16()
W = (torch.randn(V, H, device=dev) * 0.05).bfloat16()
Hs = (torch.randn(NR, H, device=dev) * 0.1).bfloat16()
Ev = E[:, :V]


def bench(f, n=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e6, 1)


out = {}
X0 = torch.empty(NR, H, device=dev)
X1 = torch.empty(NR, H, device=dev)
out['x_default_us'] = bench(lambda: torch.mm(Ev, W, out_dtype=torch.float32, out=X0))
out['x_tuned_us'] = bench(lambda: ops.gemm_bf16_tuned(X1, Ev, False, W, False, 32))
out['x_candidates_us'] = ops.gemm_tuned_timings(X1, Ev, False, W, False)
out['x_rel_err'] = float((X1 - X0).norm() / X0.norm())
D0 = torch.empty(V, H, device=dev)
D1 = torch.empty(V, H, device=dev)


def dw_split():
    kr = NR // 4
    a = E.as_strided((4, V, kr), (kr * LDL, 1, LDL))
    torch.sum(torch.bmm(a, Hs.view(4, kr, H), out_dtype=torch.float32), 0, out=D0)


out['dw_default_splitk4_us'] = bench(dw_split)
out['dw_tuned_us'] = bench(lambda: ops.gemm_bf16_tuned(D1, Ev, True, Hs, False, 32))
out['dw_candidates_us'] = ops.gemm_tuned_timings(D1, Ev, True, Hs, False)
out['dw_rel_err'] = float((D1 - D0).norm() / D0.norm())
print(json.dumps(out))
