"""hipBLASLt shape sweep for the backward vocab-head GEMMs (dS^T [h | aug])."""
import json, time, torch
dev = 'cuda'
M, V = 35840, 10509
ldl = (V + 7) // 8 * 8
dS = (torch.randn(M, ldl, device=dev) * 1e-3).bfloat16()[:, :V]
res = {}
for aug in (0, 16, 64, 128):
    hd = torch.randn(M, 512 + aug, device=dev).bfloat16()
    f = lambda: torch.mm(dS.t(), hd, out_dtype=torch.float32)
    for _ in range(3): f()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): f()
    torch.cuda.synchronize(); res['dWlog_N%d' % (512 + aug)] = round((time.perf_counter() - t) / 10 * 1e3, 3)
W = torch.randn(V, 512, device=dev).bfloat16()
f = lambda: torch.mm(dS, W, out_dtype=torch.float32)
for _ in range(3): f()
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(10): f()
torch.cuda.synchronize(); res['dHd'] = round((time.perf_counter() - t) / 10 * 1e3, 3)
ones = torch.ones(1, M, device=dev).bfloat16()
f = lambda: torch.mm(ones, dS, out_dtype=torch.float32)
for _ in range(3): f()
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(10): f()
torch.cuda.synchronize(); res['gemv_bias'] = round((time.perf_counter() - t) / 10 * 1e3, 3)
f = lambda: dS.sum(0, dtype=torch.float32)
for _ in range(3): f()
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(10): f()
torch.cuda.synchronize(); res['sum_bias'] = round((time.perf_counter() - t) / 10 * 1e3, 3)
print(json.dumps(res))
