"""Row-resident decode launch (vocab_rr.h) microbenchmark: us per launch at
the headline shape for the full kernel and with parts dropped (dbg bits:
1 no epilogue work, 2 no MFMAs, 4 no resident-row loads, 8 no recurrent
workgroups), and the tiled vocab kernel for comparison.  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cst_captioning_amd import _ext  # noqa: E402

C = _ext.ops()
dev = 'cuda'
R, H, V, vdiv = 1280, 512, 10509, 20
g = torch.Generator(device=dev).manual_seed(0)
hd = torch.randn(R, H, device=dev, generator=g).bfloat16()
h = torch.randn(R, H, device=dev, generator=g).bfloat16()
W = (torch.randn(V, H, device=dev, generator=g) * 0.05).bfloat16()
b = torch.randn(V, device=dev, generator=g)
whh = (torch.randn(4 * H, H, device=dev, generator=g) * 0.05).bfloat16()
vg = torch.randn(R // vdiv, 4 * H, device=dev, generator=g)
out = {}
for dbg in (0, 1, 2, 3, 4, 5, 7, 8, 9, 10, 11, 12):
    C.vocab_rr_bench(hd, h, W, b, whh, vg, vdiv, 5, dbg)
    out['rr_dbg%d' % dbg] = round(C.vocab_rr_bench(hd, h, W, b, whh, vg, vdiv, 50, dbg), 2)
# tiled vocab kernel (no recurrent tiles): sample + save, variant 0
tgt = torch.empty(0, dtype=torch.long, device=dev)
out['tiled_vocab_sample_save'] = round(C.vocab_fwd_bench(hd, W, b, tgt, 1, True, 50, 0), 2)
out['tiled_vocab_mainloop'] = round(C.vocab_fwd_bench(hd, W, b, tgt, 4, False, 50, 0), 2)
print(json.dumps(out), flush=True)
