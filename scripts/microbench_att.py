"""Attention kernels alone (HIP-event timed, back-to-back launches) at the
headline attention shape: 64 videos x 20 rows, C = 8 frames, A = H = 512.
which: 0 att_fwd (VALU, 4 rows / workgroup), 3 att_fwd (1 row), 1 att_bwd,
5 att_mfma forward workgroups, 6 att_bwd_mfma."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from cst_captioning_amd import _ext

C = _ext.ops()
torch.manual_seed(0)
dev = 'cuda'
Bv, vdiv, Cf, A, H = 64, 20, 8, 512, 512
R = Bv * vdiv
gv = torch.randn(Bv, Cf, 4 * H, device=dev)
P = torch.randn(Bv, Cf, A, device=dev)
q = torch.randn(R, A, device=dev)
wa = torch.randn(A, device=dev) * 0.1
ba = torch.zeros(1, device=dev)
res = {}
for which, name in ((0, 'att_fwd_rows4'), (1, 'att_bwd'), (5, 'att_mfma_fwd'), (6, 'att_bwd_mfma')):
    res[name + '_us'] = round(C.att_bench(gv, P, q, wa, ba, R, which, 50), 2)
print(json.dumps(res))

# per-workgroup phase stamps of one MFMA forward launch (wall clock, 100 MHz)
ph = C.att_mfma_phases(gv, P, wa, ba, R).cpu().double() * 10.0 / 1000.0  # us
t0 = ph[:, 0].min()
out = {}
names = ['start', 'operands', 'qgemm', 'scores', 'ticket', 'slots', 'end', 'softmax']
for k, n in enumerate(names):
    col = ph[:, k]
    ok = ph[:, k] >= 0
    if ok.any():
        v = (col[ok] - t0)
        out[n] = {'mean_us': round(float(v.mean()), 2), 'max_us': round(float(v.max()), 2)}
dur = (ph[:, 4] - ph[:, 0])
out['wg_to_ticket_mean_us'] = round(float(dur.mean()), 2)
last = ph[:, 6] >= 0
out['last_tail_mean_us'] = round(float((ph[last, 6] - ph[last, 4]).mean()), 2)
print(json.dumps({'phases': out}))
