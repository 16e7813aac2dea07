"""dW_logit shapes: the split-K batch (4 x 8960 rows) as C (V x N) = A^T B
and as C^T (N x V) = B^T A, N = 512 / 528 (the alpha-augmented rows), via
torch.bmm (hipBLASLt's heuristic pick) and the tuned batched wrapper."""
import json
import torch
from cst_captioning_amd import _ext


def bench(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)


ops = _ext.ops()
V, ldl, NR, split = 10509, 10512, 35840, 4
kr = NR // split
E = torch.rand(NR, ldl, device='cuda').to(torch.bfloat16)
out = {}
for N in (512, 528, 544, 576):
    hs = (torch.randn(NR, N, device='cuda') * 0.1).to(torch.bfloat16)
    a = E.as_strided((split, V, kr), (kr * ldl, 1, ldl))       # (b, V, K)
    b = hs.view(split, kr, N)                                   # (b, K, N)
    out['bmm_VxN_%d' % N] = bench(lambda: torch.bmm(a, b, out_dtype=torch.float32))
    at = E.as_strided((split, kr, V), (kr * ldl, ldl, 1))      # (b, K, V)
    bt = hs.view(split, kr, N).transpose(1, 2)                  # (b, N, K)
    out['bmm_NxV_%d' % N] = bench(lambda: torch.bmm(bt, at, out_dtype=torch.float32))
    p = torch.empty(split, N, V, device='cuda')
    ops.gemm_bf16_tuned_batched(p, hs.view(split, kr, N), True, at, False, 32)
    out['tuned_NxV_%d' % N] = bench(lambda: ops.gemm_bf16_tuned_batched(p, hs.view(split, kr, N), True, at, False, 32))
print(json.dumps(out))
