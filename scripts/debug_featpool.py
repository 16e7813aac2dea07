"""Error pattern of the fused FeatPool backward vs fp32 (debug aid)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cst_captioning_amd import _ext
C = _ext.ops()
torch.manual_seed(0)
for rows, d in ((64, 256), (64, 2048), (32, 128)):
    x = torch.randn(rows, d, device='cuda')
    w = torch.randn(512, d, device='cuda') * 0.02
    b = torch.zeros(512, device='cuda')
    rng = torch.zeros(2, dtype=torch.int32, device='cuda')
    out = C.featpool_forward([x], [w], [b], 0.0, rng)
    ref = torch.relu(x @ w.t() + b)
    dout = torch.randn_like(out)
    dw, db = C.featpool_backward(dout, out, [x], [w], 0.0)
    dz = dout * (out > 0)
    rdw = dz.t() @ x
    err = (dw - rdw).abs()
    print('rows', rows, 'd', d, 'fwd rel', ((out - ref).norm() / ref.norm()).item(),
          'dw rel', ((dw - rdw).norm() / rdw.norm()).item(),
          'db rel', ((db - dz.sum(0)).norm() / dz.sum(0).norm()).item())
    # per 64x64 tile max error
    t = err.view(512 // 64, 64, -1, 64 if d % 64 == 0 else 1)
    print(' worst (u,k):', divmod(int(err.argmax()), d), 'max err', err.max().item(),
          'ref there', rdw.view(-1)[err.argmax()].item(), 'got', dw.view(-1)[err.argmax()].item())
    e2 = err.view(512, d)
    print(' err by unit%64 (mean):', [round(v, 4) for v in e2.view(8, 64, d).mean((0, 2))[:8].tolist()])
    print(' err by k%64 (mean):', [round(v, 4) for v in e2.view(512, -1, 64).mean((0, 1))[:8].tolist()] if d % 64 == 0 else '')
