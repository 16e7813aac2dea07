"""TunableOp probe for the vocab-head backward GEMMs (bf16 operands, fp32 out).

Times dHd = E W and dW = E^T Hs at the headline shape with the default
hipBLASLt heuristic and after PyTorch TunableOp's search over the
hipBLASLt / rocBLAS solutions, and reports whether the mixed-output GEMMs are
tunable at all (entries in the results file).  Usage (GPU):
    PYTORCH_TUNABLEOP_ENABLED=1 python scripts/tunableop_probe.py OUT.csv
"""
import json
import os
import sys
import time

import torch

out_csv = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/tunableop_probe.csv'
dev = 'cuda'
NR, V, H, LDL = 28 * 1280, 10509, 512, 10560


def bench(f, n=10):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e3, 3)


buf = (torch.randn(NR, LDL, device=dev) * 1e-3).bfloat16()
E = buf[:, :V]
W = torch.randn(V, H, device=dev).bfloat16()
hs = torch.randn(NR, H, device=dev).bfloat16()
o1 = torch.empty(NR, H, device=dev)
o2 = torch.empty(V, H, device=dev)
gemms = {
    'dHd': lambda: torch.mm(E, W, out_dtype=torch.float32, out=o1),
    'dW': lambda: torch.mm(E.t(), hs, out_dtype=torch.float32, out=o2),
    'dHd_bf16out': lambda: torch.mm(E, W),
}
tun = torch.cuda.tunable
res = {}
tun.enable(False)
for k, f in gemms.items():
    res[k + '_default_ms'] = bench(f)
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename(out_csv, insert_device_ordinal=False)
t0 = time.time()
for k, f in gemms.items():
    f()
    torch.cuda.synchronize()
res['tuning_s'] = round(time.time() - t0, 1)
tun.tuning_enable(False)
for k, f in gemms.items():
    res[k + '_tuned_ms'] = bench(f)
res['results'] = [list(map(str, r)) for r in tun.get_results()]
res['validators'] = [list(map(str, v)) for v in tun.get_validators()]
print(json.dumps(res, indent=1), flush=True)
# the results file is written when the process exits
