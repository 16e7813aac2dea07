"""X = E W at the headline shape (35,840 x 10,509 x N) with N = 512 and W
padded with zero columns to N = 544 / 576 / 640: the tuned wrapper's best
candidate and its in-loop time."""
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
V, ldl, NR = 10509, 10512, 35840
E = torch.rand(NR, ldl, device='cuda').to(torch.bfloat16)
a = E[:, :V]
out = {}
for N in (512, 544, 576, 640):
    w = (torch.randn(V, N, device='cuda') * 0.05).to(torch.bfloat16)
    x = torch.empty(NR, N, device='cuda')
    ops.gemm_bf16_tuned(x, a, False, w, False, 48)
    out['N%d' % N] = bench(lambda: ops.gemm_bf16_tuned(x, a, False, w, False, 48))
    xt = torch.empty(N, NR, device='cuda')  # X^T = W^T E^T
    ops.gemm_bf16_tuned(xt, w, True, a, True, 48)
    out['N%d_T' % N] = bench(lambda: ops.gemm_bf16_tuned(xt, w, True, a, True, 48))
print(json.dumps(out))
